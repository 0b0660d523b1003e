"""Shared pieces of the device algorithms (not an algorithm plugin: the leading underscore keeps
it out of the create_alg registry, RL/create_pkg/create_alg.py:38-47).

* fused_adam: the algorithms' Adam. On HIP float32 parameters a HipAdam: torch.optim.Adam's
  capturable state (device float32 step, exp_avg, exp_avg_sq; same state_dict) whose step() is
  ONE mh_adam_multi launch per optimiser (csrc/optim.hip) — PyTorch's fused kernel gives each
  65,536-element chunk one workgroup (31 us per step for a 256 x 256 MLP) and increments the
  step counters in a second launch. Elsewhere torch's fused / plain Adam. Capturable either way,
  so an update that contains optimiser steps can be captured into a HIP graph.
* UpdateGraph: replays a whole model update as ONE HIP graph per branch key (e.g. the
  (update-target, update-policy) flags of an iteration). First call per branch runs eagerly on
  static input copies (lazy BLAS / Adam state init), the second captures, later calls copy
  the new batch into the static inputs and replay. Under torch.distributed the capture is cut at
  every gradient all-reduce (utils/dist.py GraphSegments: the collectives run eagerly between
  the replays, never inside a graph).
* polyak_: target-network averaging (p_t <- (1-tau) p_t + tau p), one mh_polyak_multi launch.
"""
from __future__ import annotations

import ctypes
import weakref

import torch
from torch.optim import Adam

from ..utils import dist as D


class HipAdam(Adam):
    """torch.optim.Adam (betas, eps; no weight decay / amsgrad / maximize) with capturable state.
    step(): one mh_adam_multi launch per parameter group when every parameter with a gradient is
    a contiguous HIP float32 tensor; otherwise torch's own step (fused where available) on the
    same state. The choice is made at each step: the algorithms build their optimisers before
    moving the networks to the device."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, fused=None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, capturable=True, fused=fused)
        self._ticket = None

    def _hip_entries(self, group):
        entries = []
        for p in group["params"]:
            if p.grad is None:
                continue
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()
                    and p.grad.dtype == torch.float32):
                return None
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            m, v, stp = st["exp_avg"], st["exp_avg_sq"], st["step"]
            if not (m.is_contiguous() and v.is_contiguous() and stp.is_cuda and stp.dtype == torch.float32):
                return None
            entries.append((p, p.grad, m, v, stp))
        return entries

    @torch.no_grad()
    def step(self, closure=None):
        groups = [(g, self._hip_entries(g)) for g in self.param_groups]
        if any(e is None for _, e in groups) or any(torch.is_tensor(g["lr"]) for g, _ in groups):
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from .. import _native as N
        for group, entries in groups:
            if not entries:
                continue
            dev = entries[0][0].device
            if self._ticket is None or self._ticket.device != dev:
                self._ticket = torch.zeros(1, dtype=torch.int32, device=dev)
            b1, b2 = group["betas"]
            arr = (N.AdamTensor * len(entries))()
            for i, (p, g, m, v, stp) in enumerate(entries):
                arr[i] = N.AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), stp.data_ptr(),
                                      p.numel())
            N.check(N.lib().mh_adam_multi(arr, len(entries), float(group["lr"]), float(b1), float(b2),
                                          float(group["eps"]), N.ptr(self._ticket), N.stream_of(dev)),
                    "mh_adam_multi")
        return loss


def adam_steps(*opts):
    """opt.step() for every optimiser in `opts`, as ONE Adam launch when they are all HipAdams
    with a single parameter group and the same betas / eps whose parameters all take the kernel
    (the twin critics; the policy and alpha optimisers): mh_adam_multi when their learning rates
    agree, mh_adam_multi_lr (one rate per tensor) when not. Each parameter keeps its own step
    counter, so the result is the separate steps'. Otherwise each optimiser steps on its own."""
    from .. import _native as N
    ok = len(opts) > 1 and all(isinstance(o, HipAdam) and len(o.param_groups) == 1 for o in opts)
    entries, lrs = [], []
    if ok:
        g0 = opts[0].param_groups[0]
        for o in opts:
            g = o.param_groups[0]
            if torch.is_tensor(g["lr"]) or tuple(g["betas"]) != tuple(g0["betas"]) or g["eps"] != g0["eps"]:
                ok = False
                break
            e = o._hip_entries(g)
            if e is None:
                ok = False
                break
            entries += e
            lrs += [float(g["lr"])] * len(e)
        ok = ok and len(entries) > 0  # (the C ABI chunks lists longer than its per-launch table)
    if not ok:
        for o in opts:
            o.step()
        return
    o0 = opts[0]
    dev = entries[0][0].device
    if o0._ticket is None or o0._ticket.device != dev:
        o0._ticket = torch.zeros(1, dtype=torch.int32, device=dev)
    b1, b2 = g0["betas"]
    arr = (N.AdamTensor * len(entries))()
    for i, (p, g, m, v, stp) in enumerate(entries):
        arr[i] = N.AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), stp.data_ptr(), p.numel())
    with torch.no_grad():
        if all(lr == lrs[0] for lr in lrs):
            N.check(N.lib().mh_adam_multi(arr, len(entries), lrs[0], float(b1), float(b2), float(g0["eps"]),
                                          N.ptr(o0._ticket), N.stream_of(dev)), "mh_adam_multi")
        else:
            lr_arr = (ctypes.c_double * len(lrs))(*lrs)
            N.check(N.lib().mh_adam_multi_lr(arr, len(entries), lr_arr, float(b1), float(b2), float(g0["eps"]),
                                             N.ptr(o0._ticket), N.stream_of(dev)), "mh_adam_multi_lr")


def fused_adam(params, lr):
    params = list(params)
    try:
        return HipAdam(params, lr=lr, fused=True)
    except (RuntimeError, TypeError, ValueError):
        return HipAdam(params, lr=lr)


def release_graph(g) -> None:
    """Free a captured update's graph(s) now (torch CUDAGraph or utils/dist.py GraphSegments)."""
    if g is not None:
        g.reset()  # CUDAGraph.reset / GraphSegments.reset


class UpdateGraph:
    def __init__(self, body, enabled=True):
        # the owner's bound method held weakly: an algorithm and its UpdateGraph form no reference
        # cycle, so a dropped algorithm frees its graphs at once (refcount), never later inside
        # the garbage collector (which may run during another pipeline's capture)
        self._body = weakref.WeakMethod(body) if hasattr(body, "__self__") else (lambda b=body: b)
        self.enabled = enabled
        self._static = None
        self._shapes = None
        self._graphs = {}
        self._warm = set()

    @property
    def body(self):
        b = self._body()
        if b is None:
            raise RuntimeError("UpdateGraph: its algorithm was released")
        return b

    def close(self):
        """Release every captured graph and the static inputs (idempotent)."""
        graphs, self._graphs = self._graphs, {}
        for g, _outs in graphs.values():
            release_graph(g)
        self._static = None
        self._shapes = None
        self._warm = set()

    def usable(self):
        return (self.enabled and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing())

    def __call__(self, data, key):
        if not self.usable() or not all(v.is_cuda for v in data.values() if torch.is_tensor(v)):
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
            if D.graph_segments_wanted():  # graphs cut at the gradient all-reduces (utils/dist.py)
                g = D.GraphSegments()
                with D.capturing(g):
                    outs = self.body(self._static, *key)
            else:
                g = torch.cuda.CUDAGraph()
                with D.cuda_graph(g):
                    outs = self.body(self._static, *key)
            self._graphs[key] = (g, outs)
        g, outs = self._graphs[key]
        g.replay()
        return outs


def polyak_pairs(pairs, tau):
    """polyak_ over several (net, target) pairs in one mh_polyak_multi launch when every tensor
    qualifies (the twin critics' targets); per pair otherwise."""
    polyak = 1 - tau
    with torch.no_grad():
        tp, sp = [], []
        for net, target in pairs:
            tp += [p.data for p in target.parameters()]
            sp += [p.data for p in net.parameters()]
        if tp and len(tp) == len(sp) and all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                                             and s.is_contiguous() and s.dtype == torch.float32 and t.shape == s.shape
                                             for t, s in zip(tp, sp)):
            from .. import _native as N
            arr = (N.PolyakTensor * len(tp))()
            for i, (t, s) in enumerate(zip(tp, sp)):
                arr[i] = N.PolyakTensor(t.data_ptr(), s.data_ptr(), t.numel())
            N.check(N.lib().mh_polyak_multi(arr, len(tp), float(polyak), N.stream_of(tp[0].device)),
                    "mh_polyak_multi")
            return
    for net, target in pairs:
        polyak_(net, target, tau)


def polyak_(net, target, tau):
    """p_t.mul_(polyak); p_t.add_((1 - polyak) * p) with polyak = 1 - tau, the reference's exact
    scalars (sac.py:204-217): one mh_polyak_multi launch on contiguous HIP float32 parameters,
    multi-tensor PyTorch ops otherwise."""
    polyak = 1 - tau
    with torch.no_grad():
        tp = [p.data for p in target.parameters()]
        sp = [p.data for p in net.parameters()]
        if tp and all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and s.is_contiguous()
                      and s.dtype == torch.float32 and t.shape == s.shape for t, s in zip(tp, sp)) \
                and len(tp) == len(sp):
            from .. import _native as N
            arr = (N.PolyakTensor * len(tp))()
            for i, (t, s) in enumerate(zip(tp, sp)):
                arr[i] = N.PolyakTensor(t.data_ptr(), s.data_ptr(), t.numel())
            N.check(N.lib().mh_polyak_multi(arr, len(tp), float(polyak), N.stream_of(tp[0].device)),
                    "mh_polyak_multi")
            return
        torch._foreach_mul_(tp, polyak)
        torch._foreach_add_(tp, torch._foreach_mul(sp, 1 - polyak))


def set_requires_grad(modules, flag):
    for m in modules:
        for p in m.parameters():
            p.requires_grad = flag


def step(optimizer, params):
    """optimizer.step() after averaging the gradients across ranks (one flat RCCL bucket)."""
    D.allreduce_grads(list(params))
    optimizer.step()
