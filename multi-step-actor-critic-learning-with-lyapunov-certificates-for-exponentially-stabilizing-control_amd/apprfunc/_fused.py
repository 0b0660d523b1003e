"""Device execution of the MLP layers (RL/apprfunc/mlp.py:18-30) under autograd.

The networks stay nn.Modules (nn.Sequential of nn.Linear + activation modules, the reference's
parameters and state_dict keys); on HIP tensors their forward runs each (Linear, activation)
pair as one autograd Function:
  forward   y = act(x W^T + b): ReLU fused into the GEMM epilogue (torch._addmm_activation),
            tanh applied in place on the GEMM output, identity = the GEMM alone
  backward  g = dy * act'(y) and the bias gradient (column sums of g) in one pass of
            mh_act_grad_colsum (csrc/mlp_grad.hip) instead of an elementwise backward kernel
            plus a reduction; then dx = g W and dW = g^T x as two GEMMs, each only when autograd
            needs it (frozen critics in the policy update skip dW / db).
Same math as the module's own forward/backward; the GEMM reduction order is the library's.
CPU tensors (and activations other than identity/ReLU/tanh) take the plain nn.Sequential path.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

ACT_IDS = {nn.Identity: 0, nn.ReLU: 1, nn.Tanh: 2}


def _native():
    from .. import _native as N
    return N


class LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act):
        if act == 1:
            y = torch._addmm_activation(bias, x, weight.t())
        else:
            y = torch.addmm(bias, x, weight.t())
            if act == 2:
                y = torch.tanh_(y)
        ctx.act = act
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        act = ctx.act
        dy = dy.contiguous()
        db = None
        if act == 0 and not need_b:
            g = dy
        else:
            N = _native()
            M, C = dy.shape
            chunks = ctypes.c_int32()
            N.check(N.lib().mh_act_grad_chunks(M, ctypes.byref(chunks)), "mh_act_grad_chunks")
            partial = torch.empty(chunks.value, C, dtype=dy.dtype, device=dy.device)
            g = dy if act == 0 else torch.empty_like(dy)
            db = torch.empty(C, dtype=dy.dtype, device=dy.device) if need_b else None
            N.check(N.lib().mh_act_grad_colsum(N.ptr(dy), N.ptr(y.contiguous()) if act else None, M, C, act,
                                               N.ptr(g) if act else None, N.ptr(db), N.ptr(partial),
                                               N.stream_of(dy.device)), "mh_act_grad_colsum")
        dx = g.mm(weight) if need_x else None
        dw = g.t().mm(x) if need_w else None
        return dx, dw, db, None


def fusable(seq: nn.Sequential) -> bool:
    mods = list(seq)
    if len(mods) % 2:
        return False
    for i in range(0, len(mods), 2):
        lin, act = mods[i], mods[i + 1]
        if not isinstance(lin, nn.Linear) or lin.bias is None or type(act) not in ACT_IDS:
            return False
    return True


class MLP(nn.Sequential):
    """nn.Sequential(Linear, act, Linear, act, ...) with the fused device path above."""

    def forward(self, x):
        if not (x.is_cuda and x.dtype == torch.float32 and self._fusable()):
            return super().forward(x)
        lead = x.shape[:-1]
        h = x.reshape(-1, x.shape[-1])
        if not h.is_contiguous():
            h = h.contiguous()
        mods = list(self)
        for i in range(0, len(mods), 2):
            lin, act = mods[i], mods[i + 1]
            h = LinearAct.apply(h, lin.weight, lin.bias, ACT_IDS[type(act)])
        return h.reshape(*lead, h.shape[-1])

    def _fusable(self):
        f = getattr(self, "_fusable_cache", None)
        if f is None:
            f = fusable(self)
            self._fusable_cache = f
        return f
