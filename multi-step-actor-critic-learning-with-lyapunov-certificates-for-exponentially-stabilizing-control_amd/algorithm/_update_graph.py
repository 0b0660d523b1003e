"""Shared pieces of the device algorithms (not an algorithm plugin: the leading underscore keeps
it out of the create_alg registry, RL/create_pkg/create_alg.py:38-47).

* fused_adam: torch's single-kernel Adam, capturable (step counter on the device), so an update
  that contains optimiser steps can be captured into a HIP graph.
* UpdateGraph: replays a whole model update as ONE HIP graph per branch key (e.g. the
  (update-target, update-policy) flags of an iteration). First call per branch runs eagerly on
  static input copies (lazy hipBLASLt / Adam state init), the second captures, later calls copy
  the new batch into the static inputs and replay. Off under torch.distributed (the gradient
  all-reduces are not captured) and when disabled.
* polyak_: target-network averaging as multi-tensor ops (p_t <- (1-tau) p_t + tau p).
"""
from __future__ import annotations

import torch
from torch.optim import Adam

from ..utils import dist as D


def fused_adam(params, lr):
    params = list(params)
    try:
        return Adam(params, lr=lr, fused=True, capturable=True)
    except (RuntimeError, TypeError, ValueError):
        return Adam(params, lr=lr)


class UpdateGraph:
    def __init__(self, body, enabled=True):
        self.body = body
        self.enabled = enabled
        self._static = None
        self._shapes = None
        self._graphs = {}
        self._warm = set()

    def usable(self):
        return (self.enabled and D.world_size() == 1 and torch.cuda.is_available()
                and not torch.cuda.is_current_stream_capturing())

    def __call__(self, data, key):
        if not self.usable():
            return self.body(data, *key)
        shapes = tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(data.items()) if torch.is_tensor(v))
        if self._static is None or self._shapes != shapes:
            self._static = {k: v.clone() for k, v in data.items() if torch.is_tensor(v)}
            self._shapes = shapes
            self._graphs = {}
            self._warm = set()
        for k, v in self._static.items():
            if data[k].data_ptr() != v.data_ptr():
                v.copy_(data[k])
        if key not in self._warm:
            self._warm.add(key)
            return self.body(self._static, *key)
        if key not in self._graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                outs = self.body(self._static, *key)
            self._graphs[key] = (g, outs)
        g, outs = self._graphs[key]
        g.replay()
        return outs


def polyak_(net, target, tau):
    """p_t.mul_(polyak); p_t.add_((1 - polyak) * p) with polyak = 1 - tau, the reference's exact
    scalars (sac.py:204-217)."""
    polyak = 1 - tau
    with torch.no_grad():
        tp = [p.data for p in target.parameters()]
        torch._foreach_mul_(tp, polyak)
        torch._foreach_add_(tp, torch._foreach_mul([p.data for p in net.parameters()], 1 - polyak))


def set_requires_grad(modules, flag):
    for m in modules:
        for p in m.parameters():
            p.requires_grad = flag


def step(optimizer, params):
    """optimizer.step() after averaging the gradients across ranks (one flat RCCL bucket)."""
    D.allreduce_grads(list(params))
    optimizer.step()
