"""The twin critics q1, q2 of the MSACL / SAC-style updates as ONE grouped network on the device.

The reference evaluates its two ActionValue critics (RL/apprfunc/mlp.py ActionValue: [obs | act]
-> Linear -> ReLU -> Linear -> ReLU -> Linear -> 1) one after the other on the same input, in the
critic update (RL/algorithm/msacl.py:227-266) and, frozen, in the policy step (msacl.py:383-391),
and autograd differentiates each. Here the two networks' parameters live side by side in joint
buffers (each nn.Parameter of q1 / q2 becomes a view into them: the modules, their state_dict keys
and the optimisers are unchanged), so each layer of BOTH critics is one launch:
  layer 1   h1 [rows][2H] = ReLU(x W1j^T + b1j), W1j = [W1(q1); W1(q2)]       (one GEMM, N = 2H)
  layer 2   h2[:, qH:(q+1)H] = ReLU(h1[:, qH:(q+1)H] W2(q)^T + b2(q))        (mh_gemm_f32_grouped)
  layer 3   q[q] = h2[:, qH:(q+1)H] . w3(q) + b3(q)                          (grouped one-output GEMV)
backward (weights): grouped head backward, grouped fused layer backward (dx of layer 2 and the
weight / bias gradients), and layer 1's weight / bias gradients as one deep product over the
joint [rows][2H] gradient (n_out = 2H); backward (input, frozen critics): the same without weight
gradients, and dx = g1 W1j as ONE narrow product over n_out = 2H — the sum of the two critics'
input gradients that autograd would form with a separate add.
Numerics: each group runs the ungrouped kernels' arithmetic on its own operands (layers 2-3
bit-identical to the per-critic path); layer 1's weight gradient and the summed input gradient
add the same f32 products in a different order.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

# the q heads' weight gradients folded into the backward chain launch (mh_mlp3_backward_w3);
# MSACL_FOLD_W3=0: the separate grouped head backward (the A/B and the bit-equality test)
_FOLD_W3 = os.environ.get("MSACL_FOLD_W3", "1") == "1"


def _native():
    from .. import _native as N
    return N


def _linears(q):
    """The three nn.Linear of an ActionValue critic [K -> H -> ReLU -> H -> ReLU -> 1], or None."""
    seq = getattr(q, "q", None)
    if not isinstance(seq, nn.Sequential):
        return None
    mods = list(seq)
    if len(mods) != 6:
        return None
    l1, a1, l2, a2, l3, a3 = mods
    if not (isinstance(l1, nn.Linear) and isinstance(l2, nn.Linear) and isinstance(l3, nn.Linear)
            and isinstance(a1, nn.ReLU) and isinstance(a2, nn.ReLU) and isinstance(a3, nn.Identity)):
        return None
    if l1.bias is None or l2.bias is None or l3.bias is None:
        return None
    H = l1.out_features
    if l2.in_features != H or l2.out_features != H or l3.in_features != H or l3.out_features != 1:
        return None
    return l1, l2, l3


class TwinCritic:
    """Joint-storage view of two identically shaped ActionValue critics (see the module doc).
    build() returns None when the critics do not qualify (other shapes, CPU, not float32)."""

    @staticmethod
    def build(q1, q2, min_rows=2048):
        a, b = _linears(q1), _linears(q2)
        if a is None or b is None:
            return None
        K, H = a[0].in_features, a[0].out_features
        if b[0].in_features != K or b[0].out_features != H or H % 64 or K % 4 or K > 32:
            return None
        ps = [p for l in a + b for p in (l.weight, l.bias)]
        if any(not p.is_cuda or p.dtype != torch.float32 for p in ps) or len({p.device for p in ps}) != 1:
            return None
        return TwinCritic(a, b, K, H, min_rows)

    def __init__(self, a, b, K, H, min_rows):
        self.K, self.H, self.min_rows = K, H, min_rows
        self.layers = (a, b)
        dev = a[0].weight.device
        self.device = dev
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.W1, self.b1 = f(2 * H, K), f(2 * H)
        self.W2, self.b2 = f(2, H, H), f(2, H)
        self.W3, self.b3 = f(2, H), f(2)
        self.gW1, self.gb1 = f(2 * H, K), f(2 * H)
        self.gW2, self.gb2 = f(2, H, H), f(2, H)
        self.gW3, self.gb3 = f(2, H), f(2)
        self._ws = {}
        self.version = 0
        self._join()

    # ------------------------------------------------------------------ joint storage
    def _views(self, q, W1, b1, W2, b2, W3, b3):
        H = self.H
        return ((W1[q * H:(q + 1) * H], b1[q * H:(q + 1) * H]), (W2[q], b2[q]),
                (W3[q].view(1, H), b3[q:q + 1]))

    def _join(self):
        """Copy the critics' current parameters into the joint buffers and point each parameter at
        its slice (p.data = view: the Parameter objects, hence the optimisers, are unchanged)."""
        with torch.no_grad():
            for q, lin in enumerate(self.layers):
                for (w, bb), l in zip(self._views(q, self.W1, self.b1, self.W2, self.b2, self.W3, self.b3), lin):
                    w.copy_(l.weight.detach().reshape(w.shape))
                    bb.copy_(l.bias.detach().reshape(bb.shape))
                    l.weight.data = w
                    l.bias.data = bb
        self._ptrs = self._param_ptrs()
        self.version += 1

    def _param_ptrs(self):
        return tuple(p.data_ptr() for lin in self.layers for l in lin for p in (l.weight, l.bias))

    def joined(self) -> bool:
        """The parameters still live in the joint buffers (a .to() round trip or a load with
        assign=True would have replaced them): re-joins when not. Returns True when it had to."""
        if self._param_ptrs() == self._ptrs:
            return False
        self._join()
        return True

    def applies(self, rows) -> bool:
        return rows >= self.min_rows

    def _grads(self):
        """Point every parameter's .grad at its slice of the joint gradient buffers (optimiser
        zero_grad sets them to None; the kernels overwrite the buffers, no zero fill needed)."""
        for q, lin in enumerate(self.layers):
            for (gw, gb), l in zip(self._views(q, self.gW1, self.gb1, self.gW2, self.gb2, self.gW3, self.gb3), lin):
                l.weight.grad = gw.view(l.weight.shape)
                l.bias.grad = gb.view(l.bias.shape)

    def _workspace(self, key, floats):
        t = self._ws.get(key)
        if t is None or t.numel() < floats:
            t = self._ws[key] = torch.empty(max(floats, 1), dtype=torch.float32, device=self.device)
        return t

    # ------------------------------------------------------------------ forward / backward
    def forward(self, x, keep=True):
        """x [rows][K] contiguous -> (q [2][rows], h1 [rows][2H], h2 [rows][2H]); h1 / h2 are None
        when not kept (no backward follows). One grouped mh_mlp3_forward launch for both critics
        (apprfunc/_fused.py mlp3_forward), or the per-layer launches with MSACL_MLP3=0."""
        N = _native()
        M, H = x.shape[0], self.H
        from ._fused import _MLP3, mlp3_forward
        if _MLP3["on"] and H == 256:
            q = torch.empty(2, M, dtype=torch.float32, device=x.device)
            _, h1, h2 = mlp3_forward(x, ((self.W1, self.b1), (self.W2[0], self.b2[0]), (self.W3[0:1], self.b3)),
                                     (1, 1, 0), keep, groups=2,
                                     strides=(0, H * self.K, H, H * H, H, H, 1, H, M), ldh=2 * H, y=q, ldy=1)
            return q, h1, h2
        h1 = torch._addmm_activation(self.b1, x, self.W1.t())  # one library GEMM + ReLU for both layer-1s
        h2 = torch.empty(M, 2 * H, dtype=torch.float32, device=x.device)
        q = torch.empty(2, M, dtype=torch.float32, device=x.device)
        st = N.stream_of(x.device)
        N.check(N.lib().mh_gemm_f32_grouped(N.ptr(h1), N.ptr(self.W2), N.ptr(self.b2), N.ptr(h2), M, H, H, 2 * H, H,
                                            2 * H, 0, 1, 1, 2, H, H * H, H, H, st), "mh_gemm_f32_grouped (layer 2)")
        N.check(N.lib().mh_gemm_f32_grouped(N.ptr(h2), N.ptr(self.W3), N.ptr(self.b3), N.ptr(q), M, 1, H, 2 * H, H,
                                            1, 0, 1, 0, 2, H, H, 1, M, st), "mh_gemm_f32_grouped (layer 3)")
        return q, h1, h2

    def forward_pair(self, x, other, x_other):
        """(q, h1, h2) = self.forward(x) and q_other = other.forward(x_other, keep=False)[0] in ONE
        launch (mh_mlp3_forward_pair: `other` — the target critics — as the launch's second network
        set); None when the fused path does not apply (the caller runs the two forwards)."""
        from ._fused import _MLP3
        M, H, K = x.shape[0], self.H, self.K
        if not (_MLP3["on"] and H == 256 and other.H == H and other.K == K and x_other.shape == x.shape
                and x.is_contiguous() and x_other.is_contiguous()):
            return None
        N = _native()
        q = torch.empty(2, M, dtype=torch.float32, device=x.device)
        qo = torch.empty(2, M, dtype=torch.float32, device=x.device)
        h1 = torch.empty(M, 2 * H, dtype=torch.float32, device=x.device)
        h2 = torch.empty(M, 2 * H, dtype=torch.float32, device=x.device)
        arr = lambda t: (ctypes.c_void_p * 6)(*[p.data_ptr() for p in (t.W1, t.b1, t.W2, t.b2, t.W3, t.b3)])  # noqa: E731
        gs = (ctypes.c_int64 * 9)(0, H * K, H, H * H, H, H, 1, H, M)
        N.check(N.lib().mh_mlp3_forward_pair(N.ptr(x), N.ptr(x_other), M, K, K, arr(self), arr(other), H, 1, 1, 1, 0,
                                             N.ptr(h1), N.ptr(h2), 2 * H, N.ptr(q), N.ptr(qo), 1, 2, gs,
                                             N.stream_of(x.device)), "mh_mlp3_forward_pair")
        return q, h1, h2, qo

    def _back_l23(self, dq, h1, h2, want_w):
        N = _native()
        M, H = h1.shape[0], self.H
        dev = h1.device
        st = N.stream_of(dev)
        dh2 = torch.empty(M, 2 * H, dtype=torch.float32, device=dev)
        dh1 = torch.empty(M, 2 * H, dtype=torch.float32, device=dev)
        wsh = None
        if want_w:
            n = ctypes.c_int64()
            N.check(N.lib().mh_head_backward_workspace(M, 1, H, ctypes.byref(n)), "mh_head_backward_workspace")
            wsh = self._workspace(("head", M), 2 * n.value)
        N.check(N.lib().mh_head_backward_grouped(
            N.ptr(dq), N.ptr(h2), N.ptr(self.W3), M, 1, H, 2 * H, 2 * H, 2, M, H, H, H, H, 1, N.ptr(dh2),
            N.ptr(self.gW3) if want_w else None, N.ptr(self.gb3) if want_w else None, N.ptr(wsh), st),
            "mh_head_backward_grouped")
        ok, n = ctypes.c_int32(), ctypes.c_int64()
        N.check(N.lib().mh_linear_backward_plan(M, H, H, 1, int(want_w), int(want_w), ctypes.byref(ok),
                                                ctypes.byref(n)), "mh_linear_backward_plan")
        if not ok.value:
            raise RuntimeError("TwinCritic: layer-2 backward shape not supported")
        wsl = self._workspace(("l2", M, want_w), 2 * n.value) if n.value else None
        N.check(N.lib().mh_linear_backward_grouped(
            N.ptr(dh2), N.ptr(h2), 1, N.ptr(h1), N.ptr(self.W2), M, H, H, 2 * H, 2 * H, 2 * H, 2, H, H, H * H, H,
            H * H, H, N.ptr(dh1), N.ptr(self.gW2) if want_w else None, N.ptr(self.gb2) if want_w else None,
            N.ptr(wsl), st), "mh_linear_backward_grouped")
        return dh1

    def backward_weights(self, x, dq, h1, h2):
        """Gradients of sum_q <dq[q], q-critic(x)> w.r.t. both critics' parameters, written into the
        joint gradient buffers and bound as the parameters' .grad. With the fused path: both critics'
        g2 / g1 from one mh_mlp3_backward launch, the output layers' gradients from the grouped head
        backward, and the hidden layers' (both critics' layer 2 and the joint layer 1) from one
        mh_weight_grads pair of launches."""
        N = _native()
        M = x.shape[0]
        from ._fused import _MLP3, weight_grads, wgrad_ok
        H, K = self.H, self.K
        if (_MLP3["on"] and H == 256 and wgrad_ok(x, K, x, K, 2 * H, K, M)
                and wgrad_ok(h1, 2 * H, h1, 2 * H, H, H, M)):
            dev = x.device
            st = N.stream_of(dev)
            g2 = torch.empty(M, 2 * H, dtype=torch.float32, device=dev)
            g1 = torch.empty(M, 2 * H, dtype=torch.float32, device=dev)
            gs = (ctypes.c_int64 * 6)(M, H, H * K, H * H, H, H)
            if _FOLD_W3:
                # the q heads' dW3 / db3 from the chain launch's own partials (+ one finish launch)
                n = ctypes.c_int64()
                N.check(N.lib().mh_mlp3_backward_w3_workspace(M, H, 1, 2, ctypes.byref(n)),
                        "mh_mlp3_backward_w3_workspace")
                wsh = self._workspace(("w3", M), n.value)
                N.check(N.lib().mh_mlp3_backward_w3(
                    N.ptr(dq), 1, N.ptr(h1), N.ptr(h2), 2 * H, N.ptr(self.W1), N.ptr(self.W2), N.ptr(self.W3), M, K, H,
                    1, 1, 1, N.ptr(g2), N.ptr(g1), 2 * H, None, K, 2, gs, N.ptr(self.gW3), N.ptr(self.gb3), H, 1,
                    N.ptr(wsh), st), "mh_mlp3_backward_w3 (twin weights)")
            else:
                N.check(N.lib().mh_mlp3_backward(N.ptr(dq), 1, N.ptr(h1), N.ptr(h2), 2 * H, N.ptr(self.W1),
                                                 N.ptr(self.W2), N.ptr(self.W3), M, K, H, 1, 1, 1, N.ptr(g2), N.ptr(g1),
                                                 2 * H, None, K, 2, gs, st), "mh_mlp3_backward (twin weights)")
                n = ctypes.c_int64()
                N.check(N.lib().mh_head_backward_workspace(M, 1, H, ctypes.byref(n)), "mh_head_backward_workspace")
                wsh = self._workspace(("head", M), 2 * n.value)
                N.check(N.lib().mh_head_backward_grouped(
                    N.ptr(dq), N.ptr(h2), N.ptr(self.W3), M, 1, H, 2 * H, 2 * H, 2, M, H, H, H, H, 1, None,
                    N.ptr(self.gW3), N.ptr(self.gb3), N.ptr(wsh), st), "mh_head_backward_grouped (dW3)")
            prods = [(g2[:, q * H:], 2 * H, h1[:, q * H:], 2 * H, H, H, self.gW2[q], self.gb2[q]) for q in range(2)]
            prods.append((g1, 2 * H, x, K, 2 * H, K, self.gW1, self.gb1))
            weight_grads(prods, M, dev)
            self._grads()
            return
        dh1 = self._back_l23(dq, h1, h2, True)
        ok, n = ctypes.c_int32(), ctypes.c_int64()
        N.check(N.lib().mh_linear_backward_plan(M, 2 * self.H, self.K, 0, 1, 1, ctypes.byref(ok), ctypes.byref(n)),
                "mh_linear_backward_plan")
        if not ok.value:
            raise RuntimeError("TwinCritic: layer-1 backward shape not supported")
        ws = self._workspace(("l1", M), n.value) if n.value else None
        N.check(N.lib().mh_linear_backward(N.ptr(dh1), N.ptr(h1), 1, N.ptr(x), N.ptr(self.W1), M, 2 * self.H, self.K,
                                           None, N.ptr(self.gW1), N.ptr(self.gb1), N.ptr(ws), N.stream_of(x.device)),
                "mh_linear_backward (layer 1)")
        self._grads()

    def input_grad(self, dq, h1, h2):
        """d/dx of sum_q <dq[q], q-critic(x)> (frozen critics): [rows][K]. One mh_mlp3_backward
        launch for both critics' whole input-gradient chain (the sum of the two input gradients
        formed in registers), or the per-layer launches with MSACL_MLP3=0."""
        N = _native()
        M = h1.shape[0]
        from ._fused import _MLP3
        if _MLP3["on"] and self.H == 256:
            H, K = self.H, self.K
            dx = torch.empty(M, K, dtype=torch.float32, device=h1.device)
            gs = (ctypes.c_int64 * 6)(M, H, H * K, H * H, H, 0)
            N.check(N.lib().mh_mlp3_backward(N.ptr(dq), 1, N.ptr(h1), N.ptr(h2), 2 * H, N.ptr(self.W1), N.ptr(self.W2),
                                             N.ptr(self.W3), M, K, H, 1, 1, 1, None, None, H, N.ptr(dx), K, 2, gs,
                                             N.stream_of(h1.device)), "mh_mlp3_backward (twin input gradient)")
            return dx
        dh1 = self._back_l23(dq, h1, h2, False)
        dx = torch.empty(M, self.K, dtype=torch.float32, device=h1.device)
        N.check(N.lib().mh_dx_narrow(N.ptr(dh1), N.ptr(h1), 1, N.ptr(self.W1), M, 2 * self.H, self.K, N.ptr(dx),
                                     N.stream_of(h1.device)), "mh_dx_narrow (layer 1)")
        return dx


class TwinQ(torch.autograd.Function):
    """(q1(x), q2(x)) of frozen twin critics under autograd (the policy step, msacl.py:383-391):
    forward = TwinCritic.forward, backward = TwinCritic.input_grad (the two critics' input
    gradients summed, as autograd accumulates them)."""

    @staticmethod
    def forward(ctx, x, twin):
        xc = x.contiguous()
        q, h1, h2 = twin.forward(xc)
        ctx.twin = twin
        ctx.save_for_backward(h1, h2)
        return q[0], q[1]

    @staticmethod
    def backward(ctx, d1, d2):
        h1, h2 = ctx.saved_tensors
        M = h1.shape[0]
        if (d1 is not None and d2 is not None and d1.is_contiguous() and d2.is_contiguous() and d1.dtype == torch.float32
                and d1.untyped_storage().data_ptr() == d2.untyped_storage().data_ptr()
                and d2.data_ptr() == d1.data_ptr() + 4 * M):
            # the two gradients are the halves of one buffer (MSACL's objective backward): no copy
            return ctx.twin.input_grad(d1.as_strided((2, M), (M, 1)), h1, h2), None
        dq = torch.empty(2, M, dtype=torch.float32, device=h1.device)
        if d1 is None:
            dq[0].zero_()
        else:
            dq[0].copy_(d1.reshape(M))
        if d2 is None:
            dq[1].zero_()
        else:
            dq[1].copy_(d2.reshape(M))
        return ctx.twin.input_grad(dq, h1, h2), None
