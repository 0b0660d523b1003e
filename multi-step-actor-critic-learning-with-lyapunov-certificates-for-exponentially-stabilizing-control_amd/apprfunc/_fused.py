"""Device execution of the MLP layers (RL/apprfunc/mlp.py:18-30) under autograd.

The networks stay nn.Modules (nn.Sequential of nn.Linear + activation modules, the reference's
parameters and state_dict keys); on HIP tensors their forward runs each (Linear, activation)
pair as one autograd Function:
  forward   y = act(x W^T + b): one mh_gemm_f32 launch (csrc/gemm.hip, f32 MFMA) with the bias
            and ReLU / tanh in its epilogue
  backward  by default (MSACL_FUSED_BACKWARD=0: off) for the B x n-row 256-wide layers,
            mh_linear_backward (csrc/gemm.hip): dx = g W and dW = g^T x, db = column sums of g,
            with g = dy * act'(y) formed inside the two GEMMs' operand staging (never written);
            for the other layers g and the bias gradient in one pass
            of mh_act_grad_colsum (csrc/mlp_grad.hip) instead of an elementwise backward kernel
            plus a reduction, then dx = g W and dW = g^T x as two mh_gemm_f32 launches. Each
            output only when autograd needs it (frozen critics in the policy update skip dW / db).
Same math as the module's own forward/backward, f32 throughout; the GEMM summation order is the
kernel's. Backend (`set_gemm_backend`, config key `update_gemm`):
  "auto" (default)  mh_gemm_f32 where it measured faster than the BLAS library on the update's
                    shapes (tools/gemm_shapes.py, profiles/r01_gemm_shapes.json): forwards on
                    <= 1,024 rows (the B = 256 rows of the first-step networks: 8 vs 63 us, where
                    the library runs a 256^3 product on one workgroup), into one output column
                    (critic heads) or through tanh from a short input (epilogue instead of a
                    separate tanh launch), forwards and input gradients of the B x n-row
                    256-wide layers (the tall-product kernel), and weight gradients of one-output
                    layers; the library (torch.addmm / _addmm_activation / mm) elsewhere
  "hip"             every GEMM through mh_gemm_f32
  "blas"            every GEMM through the library
CPU tensors (and activations other than identity/ReLU/tanh) take the plain nn.Sequential path.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

ACT_IDS = {nn.Identity: 0, nn.ReLU: 1, nn.Tanh: 2}


def _native():
    from .. import _native as N
    return N


_GEMM_BACKEND = {"name": "auto"}
_COLSUM_TICKETS = {}


_TICKET_POOL = {}


def _colsum_tickets(dev, cols):
    """Arrival counters of mh_act_grad_colsum's in-launch bias-gradient finish, one set per
    (device, stream): zeroed once, left zero by every launch, never shared by launches that can
    run concurrently (the MSACL update runs several streams). Sets are slices of one per-device
    pool zeroed at its first use, so a stream first seen inside a graph capture (torch captures
    on its own stream) adds no zero-fill node to the replayed graph."""
    need = (cols + 63) // 64
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    t = _COLSUM_TICKETS.get(key)
    if t is None or t.numel() < need:
        width = max(need, 64)
        pool = _TICKET_POOL.get(dev)
        if pool is None:
            pool = _TICKET_POOL[dev] = [torch.zeros(64 * 256, dtype=torch.int32, device=dev), 0]
        buf, used = pool
        if used + width <= buf.numel():
            t = buf[used:used + width]
            pool[1] = used + width
        else:  # pool exhausted (many streams or very wide layers): a set of its own
            t = torch.zeros(width, dtype=torch.int32, device=dev)
        _COLSUM_TICKETS[key] = t
    return t
_WS = {}


def set_gemm_backend(name: str):
    """"auto" (default), "hip" (mh_gemm_f32 everywhere) or "blas" (PyTorch's GEMM library)."""
    if name not in ("auto", "hip", "blas"):
        raise ValueError(f"update_gemm must be 'auto', 'hip' or 'blas', got {name!r}")
    _GEMM_BACKEND["name"] = name


def _tall(rows, n, k):
    """mh_gemm_f32's tall-product kernel (k_gemm_tall: >= 2,048 rows, N % 64 == 0) on a K deep
    enough for its pipeline: 10.6 vs 12.4 us (forward) and 10.9 vs 12.1 us (input gradient) at
    5,120 x 256 x 256 (tools/tall_probe.py); the library stays faster for K < 64."""
    return rows >= 2048 and n % 64 == 0 and k % 4 == 0 and k >= 64


def _hip_forward(rows, out_features, act=0, in_features=0):
    b = _GEMM_BACKEND["name"]
    # tanh layers with a short K: the epilogue saves the library path's separate tanh launch.
    # ReLU first layers (K <= 32) stay on the library: its fused addmm+relu beats mh_gemm_f32's
    # short-K kernel there (5.1 vs 9.0 us at 5,120 x 256 x 16, tools/gemm_shapes.py)
    return b == "hip" or (b == "auto" and (rows <= 1024 or out_features == 1 or (act == 2 and in_features <= 64)
                                           or _tall(rows, out_features, in_features)))


def _hip_dx(rows=0, in_features=0, out_features=0):
    b = _GEMM_BACKEND["name"]
    return b == "hip" or (b == "auto" and _tall(rows, in_features, out_features))


def _hip_dw(out_features, in_features=0, rows=0):
    """Weight gradients: one-output layers, and g^T x of 64-multiple layers over >= 1,024 rows
    (the deep-product kernel k_gemm_deep: 14.7 vs 18.6 us at 256 x 256 x 5,120)."""
    b = _GEMM_BACKEND["name"]
    return b == "hip" or (b == "auto" and (out_features == 1 or (out_features % 64 == 0 and in_features % 64 == 0
                                                                   and rows >= 1024)))


def gemm_backend() -> str:
    return _GEMM_BACKEND["name"]


def gemm(a, b, bias, M, N, K, lda, ldb, ta, tb, act=0):
    """C[M][N] = act(op(a) op(b) + bias) on the f32 MFMA (include/msacl_hip.h: mh_gemm_f32)."""
    N_ = _native()
    key = (M, N, K)
    wsf = _WS.get(key)
    if wsf is None:
        wf = ctypes.c_int64()
        N_.check(N_.lib().mh_gemm_workspace(M, N, K, ctypes.byref(wf)), "mh_gemm_workspace")
        wsf = _WS[key] = wf.value
    dev = a.device
    c = torch.empty(M, N, dtype=torch.float32, device=dev)
    work = torch.empty(wsf, dtype=torch.float32, device=dev) if wsf else None
    N_.check(N_.lib().mh_gemm_f32(N_.ptr(a), N_.ptr(b), N_.ptr(bias), N_.ptr(c), M, N, K, lda, ldb, N, ta, tb, act,
                                  N_.ptr(work), N_.stream_of(dev)), "mh_gemm_f32")
    return c


_LB_PLAN = {}
# On by default since round 2: measured neutral in round 1 (update 1.08-1.12 ms either way), but
# with the update's other launches trimmed the colsum launch it removes is on the critical path:
# 696-708 vs 674-678 M env-steps/s, 3 alternating pairs on one box
# (profiles/r02_fused_backward_ab.jsonl); MSACL_FUSED_BACKWARD=0 turns it off.
_FUSED_BACKWARD = {"on": os.environ.get("MSACL_FUSED_BACKWARD", "1") == "1"}


def _linear_backward_fused(dy, y, act, x, weight, need_x, need_w, need_b):
    """The whole layer backward as mh_linear_backward (csrc/gemm.hip: g = dy * act'(y) formed
    inside the tall dx and deep dW GEMMs, the bias gradient inside the latter) when the shape and
    request qualify; None otherwise (the colsum + GEMM path)."""
    if _GEMM_BACKEND["name"] == "blas" or not (need_x or need_w):
        return None
    rows, n_out = dy.shape
    n_in = x.shape[1]
    key = (rows, n_out, n_in, bool(need_x), bool(need_w), bool(need_b))
    plan = _LB_PLAN.get(key)
    if plan is None:
        N = _native()
        ok, ws = ctypes.c_int32(), ctypes.c_int64()
        N.check(N.lib().mh_linear_backward_plan(rows, n_out, n_in, int(need_x), int(need_w), int(need_b),
                                                ctypes.byref(ok), ctypes.byref(ws)), "mh_linear_backward_plan")
        plan = _LB_PLAN[key] = (bool(ok.value), ws.value)
    if not plan[0]:
        return None
    w = weight.contiguous()
    xc = x.contiguous()
    yc = y.contiguous()
    if any(t.data_ptr() % 16 for t in (dy, yc, xc, w)):
        return None
    N = _native()
    dev = dy.device
    dx = torch.empty(rows, n_in, dtype=dy.dtype, device=dev) if need_x else None
    dw = torch.empty(n_out, n_in, dtype=dy.dtype, device=dev) if need_w else None
    db = torch.empty(n_out, dtype=dy.dtype, device=dev) if need_b else None
    work = torch.empty(plan[1], dtype=torch.float32, device=dev) if plan[1] else None
    N.check(N.lib().mh_linear_backward(N.ptr(dy), N.ptr(yc) if act else None, act, N.ptr(xc), N.ptr(w), rows, n_out,
                                       n_in, N.ptr(dx), N.ptr(dw), N.ptr(db), N.ptr(work), N.stream_of(dev)),
            "mh_linear_backward")
    return dx, dw, db, None


_HEAD_WS = {}
_HEAD_BACKWARD = {"on": os.environ.get("MSACL_HEAD_BACKWARD", "1") == "1"}  # A/B switch


def _head_backward(dy, x, weight, need_x, need_w, need_b):
    """Backward of a narrow identity output layer (n_out <= 16, the critic / policy heads) as
    mh_head_backward (csrc/mlp_grad.hip): dx = dy W, dW = dy^T x and db in one pass over x + a
    block-ordered finish; None when the request does not qualify."""
    rows, n_out = dy.shape
    n_in = x.shape[1]
    if (need_b and not need_w) or not (need_x or need_w) or rows < 1024 or n_out > 16:
        return None
    N = _native()
    dev = dy.device
    key = (rows, n_out, n_in)
    ws = _HEAD_WS.get(key)
    if ws is None:
        wf = ctypes.c_int64()
        N.check(N.lib().mh_head_backward_workspace(rows, n_out, n_in, ctypes.byref(wf)), "mh_head_backward_workspace")
        ws = _HEAD_WS[key] = wf.value
    xc = x.contiguous()
    w = weight.contiguous()
    dx = torch.empty(rows, n_in, dtype=dy.dtype, device=dev) if need_x else None
    dw = torch.empty(n_out, n_in, dtype=dy.dtype, device=dev) if need_w else None
    db = torch.empty(n_out, dtype=dy.dtype, device=dev) if need_b else None
    work = torch.empty(ws, dtype=torch.float32, device=dev) if need_w else None
    N.check(N.lib().mh_head_backward(N.ptr(dy), N.ptr(xc), N.ptr(w), rows, n_out, n_in, N.ptr(dx), N.ptr(dw), N.ptr(db),
                                     N.ptr(work), N.stream_of(dev)), "mh_head_backward")
    return dx, dw, db, None


class LinearAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act):
        M, K = x.shape
        Nout = weight.shape[0]
        if _hip_forward(M, Nout, act, K):
            y = gemm(x, weight.contiguous(), bias.contiguous(), M, Nout, K, K, K, 0, 1, act)
        elif act == 1:
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
        dx, dw, db = layer_backward(dy, x, weight, y, ctx.act, need_x, need_w, need_b)
        return dx, dw, db, None


def layer_backward(dy, x, weight, y, act, need_x, need_w, need_b):
    """The backward of y = act(x W^T + b) for the requested gradients: (dx, dW, db), each None
    when not requested (LinearAct.backward, also the per-layer backward of MLP3)."""
    dy = dy.contiguous()
    if act == 0 and _HEAD_BACKWARD["on"] and _GEMM_BACKEND["name"] != "blas":
        head = _head_backward(dy, x, weight, need_x, need_w, need_b)
        if head is not None:
            return head[:3]
    if (need_x and not need_w and not need_b and _FUSED_BACKWARD["on"] and _GEMM_BACKEND["name"] != "blas"
            and x.shape[1] <= 32 and dy.shape[0] >= 1024 and dy.shape[1] <= 1024):
        # narrow input, input gradient only (a frozen critic's first layer): one launch
        N = _native()
        rows, n_out = dy.shape
        dx = torch.empty(rows, x.shape[1], dtype=dy.dtype, device=dy.device)
        N.check(N.lib().mh_dx_narrow(N.ptr(dy), N.ptr(y.contiguous()) if act else None, act,
                                     N.ptr(weight.contiguous()), rows, n_out, x.shape[1], N.ptr(dx),
                                     N.stream_of(dy.device)), "mh_dx_narrow")
        return dx, None, None
    if _FUSED_BACKWARD["on"]:
        fused = _linear_backward_fused(dy, y, act, x, weight, need_x, need_w, need_b)
        if fused is not None:
            return fused[:3]
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
                                           N.ptr(_colsum_tickets(dy.device, C)), N.stream_of(dy.device)),
                "mh_act_grad_colsum")
    M, Nout = g.shape
    K = x.shape[1]
    dx = dw = None
    if need_x:
        dx = gemm(g, weight.contiguous(), None, M, K, Nout, Nout, K, 0, 0) if _hip_dx(M, K, Nout) else g.mm(weight)
    if need_w:
        dw = gemm(g, x, None, Nout, K, M, Nout, K, 1, 0) if _hip_dw(Nout, K, M) else g.t().mm(x)
    return dx, dw, db


# The whole 3-layer MLP forward as one launch (mh_mlp3_forward, csrc/mlp_fused.hip) where the
# shape qualifies; MSACL_MLP3=0 restores the per-layer launches (A/B)
_MLP3 = {"on": os.environ.get("MSACL_MLP3", "1") == "1",
         # wide outputs (N3 a multiple of 64: the policy trunk) through the one-launch kernel too
         # (two row tiles per wave: 30.0 us standalone, the per-layer kernels 30.2; in the bench
         # 1.114-1.125 vs 1.109-1.119 G env-steps/s); MSACL_MLP3_WIDE=0: the per-layer kernels
         "wide_fwd": os.environ.get("MSACL_MLP3_WIDE", "1") == "1",
         # LyapunovValue's square sums inside the MLP's launches (MLP3SquareSum); 0: SquareSum (A/B)
         "sqsum": os.environ.get("MSACL_MLP3_SQSUM", "1") == "1"}


def _linear_act(x, W, b, act):
    """LinearAct's forward kernels without autograd: act(x W^T + b)."""
    M, K = x.shape
    Nout = W.shape[0]
    if _hip_forward(M, Nout, act, K):
        return gemm(x, W.contiguous(), b.contiguous(), M, Nout, K, x.stride(0), K, 0, 1, act)
    if act == 1:
        return torch._addmm_activation(b, x, W.t())
    y = torch.addmm(b, x, W.t())
    return torch.tanh_(y) if act == 2 else y


def mlp3_forward(x, layers, acts, h_keep, groups=1, strides=None, ldh=None, y=None, ldy=None):
    """mh_mlp3_forward: x [M][K1] -> (y, h1, h2); h1 / h2 only when h_keep. `layers` are the three
    (weight, bias) pairs (group 0's when groups > 1)."""
    N = _native()
    (W1, b1), (W2, b2), (W3, b3) = layers
    M, K1 = x.shape[0], x.shape[1]
    H, N3 = W2.shape[-1], W3.shape[0]
    dev = x.device
    if ldh is None:
        ldh = H
    h1 = torch.empty(M, ldh, dtype=torch.float32, device=dev) if h_keep else None
    h2 = torch.empty(M, ldh, dtype=torch.float32, device=dev) if h_keep else None
    if y is None:
        y = torch.empty(M, N3, dtype=torch.float32, device=dev)
        ldy = N3
    gs = (ctypes.c_int64 * 9)(*strides) if strides is not None else None
    N.check(N.lib().mh_mlp3_forward(N.ptr(x), M, K1, x.stride(0), N.ptr(W1), N.ptr(b1), N.ptr(W2), N.ptr(b2),
                                    N.ptr(W3), N.ptr(b3), H, N3, acts[0], acts[1], acts[2], N.ptr(h1), N.ptr(h2), ldh,
                                    N.ptr(y), ldy, groups, gs, N.stream_of(dev)), "mh_mlp3_forward")
    return y, h1, h2


_WG_WS = {}


def wgrad_ok(g, ld_g, x, ld_x, n_out, n_in, rows):
    """mh_weight_grads takes this product (include/msacl_hip.h)."""
    if rows < 1024 or ld_g % 4 or ld_x % 4 or g.data_ptr() % 16 or x.data_ptr() % 16:
        return False
    if n_out % 64 == 0 and n_in % 4 == 0:
        return True
    return n_out < 64 and n_out % 4 == 0 and n_in % 64 == 0 and ld_g == n_out


def weight_grads(products, rows, dev):
    """mh_weight_grads over `products` = [(g, ld_g, x, ld_x, n_out, n_in, dw, db)] (dw / db tensors,
    db may be None): every dw = g^T x and db = column sums of g in two launches."""
    N = _native()
    arr = (N.Wgrad * len(products))()
    for i, (g, ld_g, x, ld_x, n_out, n_in, dw, db) in enumerate(products):
        arr[i] = N.Wgrad(g.data_ptr(), ld_g, x.data_ptr(), ld_x, n_out, n_in, dw.data_ptr(),
                         db.data_ptr() if db is not None else None)
    # only the workspace SIZE is cached: the buffer itself comes from the caching allocator on the
    # current stream for every call (under graph capture: the graph's pool), so two concurrent
    # calls of one shape on different streams (the twin critics' q1 / q2) never share it
    key = (rows, tuple((p[4], p[5], p[1], p[3], p[7] is not None) for p in products))
    nws = _WG_WS.get(key)
    if nws is None:
        f = ctypes.c_int64()
        N.check(N.lib().mh_weight_grads_workspace(arr, len(products), rows, ctypes.byref(f)), "mh_weight_grads_workspace")
        nws = _WG_WS[key] = max(f.value, 1)
    ws = torch.empty(nws, dtype=torch.float32, device=dev)
    N.check(N.lib().mh_weight_grads(arr, len(products), rows, N.ptr(ws), N.stream_of(dev)), "mh_weight_grads")


class MLP3(torch.autograd.Function):
    """Linear -> act -> Linear -> act -> Linear -> act under autograd: forward = one
    mh_mlp3_forward launch (h1 / h2 kept only when a gradient will be taken), backward = the
    three layers' LinearAct backwards (layer_backward) on the kept activations."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3, acts, grad=True):
        # h1 / h2 are written to HBM only when a backward can follow: `grad` is the caller's grad
        # mode (Function.forward itself always runs without grad, and needs_input_grad is True
        # under torch.no_grad() whenever the parameters require grad)
        keep = grad and any(ctx.needs_input_grad[:7])
        if W3.shape[0] > 16 and not _MLP3["wide_fwd"]:
            h1 = _linear_act(x, W1, b1, acts[0])
            h2 = _linear_act(h1, W2, b2, acts[1])
            y = _linear_act(h2, W3, b3, acts[2])
        else:
            y, h1, h2 = mlp3_forward(x, ((W1, b1), (W2, b2), (W3, b3)), acts, keep)
        ctx.acts = acts
        if keep:
            ctx.save_for_backward(x, W1, W2, W3, h1, h2, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W1, W2, W3, h1, h2, y = ctx.saved_tensors
        nx, nW1, nb1, nW2, nb2, nW3, nb3 = ctx.needs_input_grad[:7]
        a1, a2, a3 = ctx.acts
        need_h2 = nx or nW1 or nb1 or nW2 or nb2
        if nx and not (nW1 or nb1 or nW2 or nb2 or nW3 or nb3) and a3 == 0:
            # input gradient only (a frozen network): the whole chain in one mh_mlp3_backward launch
            N = _native()
            M, K1 = x.shape
            dx = torch.empty(M, K1, dtype=torch.float32, device=x.device)
            dyc = dy.contiguous()
            N.check(N.lib().mh_mlp3_backward(N.ptr(dyc), dyc.shape[1], N.ptr(h1), N.ptr(h2), h1.shape[1], N.ptr(W1),
                                             N.ptr(W2), N.ptr(W3), M, K1, W2.shape[0], W3.shape[0], a1, a2, None,
                                             None, W2.shape[0], N.ptr(dx), K1, 1, None, N.stream_of(x.device)),
                    "mh_mlp3_backward")
            return dx, None, None, None, None, None, None, None, None
        if a3 == 0 and _MLP3["on"]:
            # the input-gradient chain in one launch (g2 / g1 kept for the weight gradients), then
            # every layer's weight / bias gradient in two more (mh_weight_grads); a product that
            # launch does not take goes through the per-layer path
            N = _native()
            M, K1 = x.shape
            H, N3, dev = W2.shape[0], W3.shape[0], x.device
            want2, want1 = nW2 or nb2, nW1 or nb1
            e = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)  # noqa: E731
            g2 = e(M, H) if want2 else None
            g1 = e(M, H) if want1 else None
            dx = e(M, K1) if nx else None
            dyc = dy.contiguous()
            if want2 or want1 or nx:
                N.check(N.lib().mh_mlp3_backward(N.ptr(dyc), N3, N.ptr(h1), N.ptr(h2), H, N.ptr(W1), N.ptr(W2),
                                                 N.ptr(W3), M, K1, H, N3, a1, a2, N.ptr(g2), N.ptr(g1), H, N.ptr(dx), K1,
                                                 1, None, N.stream_of(dev)), "mh_mlp3_backward")
            out = {}
            prods = []
            for name, want, nw, nb, g, ld_g, xin, ld_x, n_out, n_in, W in (
                    ("3", nW3 or nb3, nW3, nb3, dyc, N3, h2, H, N3, H, W3),
                    ("2", want2, nW2, nb2, g2, H, h1, H, H, H, W2),
                    ("1", want1, nW1, nb1, g1, H, x, K1, H, K1, W1)):
                if not want:
                    out[name] = (None, None)
                    continue
                dw, db = e(n_out, n_in), (e(n_out) if nb else None)
                if wgrad_ok(g, ld_g, xin, ld_x, n_out, n_in, M):
                    prods.append((g, ld_g, xin, ld_x, n_out, n_in, dw, db))
                    out[name] = (dw if nw else None, db)
                else:  # the per-layer path on the chain's gradient (identity: it is already g)
                    _, dw2, db2_ = layer_backward(g, xin, W, g, 0, False, nw, nb)
                    out[name] = (dw2, db2_)
            if prods:
                weight_grads(prods, M, dev)
            return (dx, out["1"][0], out["1"][1], out["2"][0], out["2"][1], out["3"][0], out["3"][1], None, None)
        dh2, dW3, db3 = layer_backward(dy, h2, W3, y, a3, need_h2, nW3, nb3)
        dx = dW1 = db1 = dW2 = db2 = None
        if need_h2:
            need_h1 = nx or nW1 or nb1
            dh1, dW2, db2 = layer_backward(dh2, h1, W2, h2, a2, need_h1, nW2, nb2)
            if need_h1:
                dx, dW1, db1 = layer_backward(dh1, x, W1, h1, a1, nx, nW1, nb1)
        return dx, dW1, db1, dW2, db2, dW3, db3, None, None


class MLP3SquareSum(torch.autograd.Function):
    """LyapunovValue's V = sum(MLP(x)^2, -1) (mlp.py LyapunovValue) over a 3-layer MLP with a wide
    output (N3 a multiple of 64): the forward is mh_mlp3_forward_sqsum (the square sums formed in
    the MLP's launch, SquareSum's bits), the backward mh_mlp3_backward_sqsum (dy = dV 2y formed
    in the chain's launch, SquareSum.backward's bits, kept for the weight gradients) plus
    mh_weight_grads: the square-sum launch and its backward launch disappear."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3, acts, grad=True):
        N = _native()
        M, K1 = x.shape
        H, N3, dev = W2.shape[0], W3.shape[0], x.device
        # h1 / h2 are written to HBM only when a backward can follow: `grad` is the caller's grad
        # mode (Function.forward itself always runs without grad, and needs_input_grad is True
        # under torch.no_grad() whenever the parameters require grad)
        keep = grad and any(ctx.needs_input_grad[:7])
        e = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)  # noqa: E731
        y, v = e(M, N3), e(M)
        h1, h2 = (e(M, H), e(M, H)) if keep else (None, None)
        ps = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in (W1, b1, W2, b2, W3, b3)])
        N.check(N.lib().mh_mlp3_forward_sqsum(N.ptr(x), M, K1, x.stride(0), ps, H, N3, acts[0], acts[1], acts[2],
                                              N.ptr(h1), N.ptr(h2), H, N.ptr(y), N3, N.ptr(v), N.stream_of(dev)),
                "mh_mlp3_forward_sqsum")
        ctx.acts = acts
        if keep:
            ctx.save_for_backward(x, W1, W2, W3, h1, h2, y)
        return v

    @staticmethod
    def backward(ctx, dv):
        N = _native()
        x, W1, W2, W3, h1, h2, y = ctx.saved_tensors
        nx, nW1, nb1, nW2, nb2, nW3, nb3 = ctx.needs_input_grad[:7]
        a1, a2, _a3 = ctx.acts
        M, K1 = x.shape
        H, N3, dev = W2.shape[0], W3.shape[0], x.device
        e = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)  # noqa: E731
        g3, g2, g1 = e(M, N3), e(M, H), e(M, H)
        dx = e(M, K1) if nx else None
        N.check(N.lib().mh_mlp3_backward_sqsum(N.ptr(y), N3, N.ptr(dv.contiguous()), N.ptr(h1), N.ptr(h2), H,
                                               N.ptr(W1), N.ptr(W2), N.ptr(W3), M, K1, H, N3, a1, a2, N.ptr(g3),
                                               N.ptr(g2), N.ptr(g1), H, N.ptr(dx), K1, N.stream_of(dev)),
                "mh_mlp3_backward_sqsum")
        out, prods = {}, []
        for name, nw, nb, g, ld_g, xin, ld_x, n_out, n_in, W in (
                ("3", nW3, nb3, g3, N3, h2, H, N3, H, W3), ("2", nW2, nb2, g2, H, h1, H, H, H, W2),
                ("1", nW1, nb1, g1, H, x, K1, H, K1, W1)):
            if not (nw or nb):
                out[name] = (None, None)
                continue
            dw, db = e(n_out, n_in), (e(n_out) if nb else None)
            if wgrad_ok(g, ld_g, xin, ld_x, n_out, n_in, M):
                prods.append((g, ld_g, xin, ld_x, n_out, n_in, dw, db))
                out[name] = (dw if nw else None, db)
            else:
                _, dw2, db2_ = layer_backward(g, xin, W, g, 0, False, nw, nb)
                out[name] = (dw2, db2_)
        if prods:
            weight_grads(prods, M, dev)
        return (dx, out["1"][0], out["1"][1], out["2"][0], out["2"][1], out["3"][0], out["3"][1], None, None)


def square_sum_mlp(seq, x):
    """V = sum(seq(x)^2, -1) through MLP3SquareSum when the fused path takes `seq` (a 3-layer MLP
    with a wide identity output), else None (the caller runs seq and SquareSum)."""
    if not (_MLP3["on"] and _MLP3["wide_fwd"] and _MLP3["sqsum"] and _GEMM_BACKEND["name"] != "blas" and x.is_cuda
            and x.dtype == torch.float32):
        return None
    spec = mlp3_layers(seq)
    if spec is None:
        return None
    (l1, l2, l3), acts = spec
    if acts[2] != 0 or l3[0].shape[0] % 64 != 0:
        return None
    lead = x.shape[:-1]
    h = x.reshape(-1, x.shape[-1])
    if not h.is_contiguous():
        h = h.contiguous()
    if h.data_ptr() % 4:
        return None
    v = MLP3SquareSum.apply(h, l1[0], l1[1], l2[0], l2[1], l3[0], l3[1], acts, torch.is_grad_enabled())
    return v.reshape(lead)


class MLP3Kept(torch.autograd.Function):
    """MLP3 whose forward already ran (mlp3_forward with the activations kept, e.g. by an earlier
    no-grad use of the same network on the same rows with the same weights): returns the kept
    output, backward exactly as MLP3's. `kept` = (h1, h2, y)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3, acts, kept):
        h1, h2, y = kept
        ctx.acts = acts
        ctx.save_for_backward(x, W1, W2, W3, h1, h2, y)
        return y.view_as(y)

    @staticmethod
    def backward(ctx, dy):
        return MLP3.backward(ctx, dy)  # (its last None stands for `kept`)


def mlp3_forward_kept(seq, x):
    """(y, kept) of the MLP `seq` on x [rows][K1] through mh_mlp3_forward with h1 / h2 kept, for a
    later MLP3Kept.apply(x, *params, acts, kept); None when the fused path does not take `seq`."""
    if not (_MLP3["on"] and _GEMM_BACKEND["name"] != "blas" and x.is_cuda and x.dtype == torch.float32
            and x.is_contiguous() and x.data_ptr() % 4 == 0):
        return None
    spec = mlp3_layers(seq)
    if spec is None:
        return None
    (l1, l2, l3), acts = spec
    if l3[0].shape[0] > 16 and not _MLP3["wide_fwd"]:
        return None
    y, h1, h2 = mlp3_forward(x, (l1, l2, l3), acts, True)
    return y, (h1, h2, y), (l1, l2, l3), acts


def mlp3_layers(seq):
    """((W1, b1), (W2, b2), (W3, b3)), (act ids) of an MLP [K1 <= 32, 256, 256, N3] that
    mh_mlp3_forward runs, else None."""
    mods = list(seq)
    if len(mods) != 6:
        return None
    l1, a1, l2, a2, l3, a3 = mods
    if not all(isinstance(l, nn.Linear) and l.bias is not None for l in (l1, l2, l3)):
        return None
    if any(type(a) not in ACT_IDS for a in (a1, a2, a3)):
        return None
    H, K1, N3 = l1.out_features, l1.in_features, l3.out_features
    if H != 256 or l2.in_features != H or l2.out_features != H or l3.in_features != H or K1 > 32:
        return None
    if not (N3 <= 16 or (N3 % 64 == 0 and N3 <= 256)):
        return None
    ps = (l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)
    if any(not p.is_contiguous() or p.dtype != torch.float32 or p.data_ptr() % 16 for p in ps):
        return None
    return ((l1.weight, l1.bias), (l2.weight, l2.bias), (l3.weight, l3.bias)), tuple(ACT_IDS[type(a)] for a in (a1, a2, a3))


class SquareSum(torch.autograd.Function):
    """torch.pow(y, 2).sum(-1) over the last dimension (LyapunovValue.forward) as one launch
    forward and one backward (mh_square_sum[_backward]); the backward's bits are pow's."""

    @staticmethod
    def forward(ctx, y):
        N = _native()
        cols = y.shape[-1]
        yc = y.contiguous()
        rows = yc.numel() // cols
        out = torch.empty(y.shape[:-1], dtype=y.dtype, device=y.device)
        N.check(N.lib().mh_square_sum(N.ptr(yc), rows, cols, N.ptr(out), N.stream_of(y.device)), "mh_square_sum")
        ctx.save_for_backward(yc)
        return out

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        N = _native()
        cols = y.shape[-1]
        rows = y.numel() // cols
        dy = torch.empty_like(y)
        N.check(N.lib().mh_square_sum_backward(N.ptr(y), N.ptr(g.contiguous()), rows, cols, N.ptr(dy),
                                               N.stream_of(y.device)), "mh_square_sum_backward")
        return dy


class StochaHead(torch.autograd.Function):
    """[mean | log_std] -> [mean | exp(clamp(log_std, lo, hi))] (StochaPolicy.forward, mlp.py:132-136)
    as one launch forward and one backward (mh_stocha_head[_backward], csrc/dist_kernels.hip)."""

    @staticmethod
    def forward(ctx, raw, lo, hi):
        N = _native()
        A = raw.shape[-1] // 2
        rows = raw.numel() // max(2 * A, 1)
        out = torch.empty_like(raw)
        N.check(N.lib().mh_stocha_head(N.ptr(raw), rows, A, lo, hi, N.ptr(out), N.stream_of(raw.device)),
                "mh_stocha_head")
        ctx.save_for_backward(raw, out)
        ctx.lo, ctx.hi = lo, hi
        return out

    @staticmethod
    def backward(ctx, d_out):
        raw, out = ctx.saved_tensors
        N = _native()
        A = raw.shape[-1] // 2
        rows = raw.numel() // max(2 * A, 1)
        d_raw = torch.empty_like(raw)
        N.check(N.lib().mh_stocha_head_backward(N.ptr(raw), N.ptr(out), N.ptr(d_out.contiguous()), rows, A, ctx.lo,
                                                ctx.hi, N.ptr(d_raw), N.stream_of(raw.device)),
                "mh_stocha_head_backward")
        return d_raw, None, None


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
        if _MLP3["on"] and _GEMM_BACKEND["name"] != "blas" and h.data_ptr() % 4 == 0:
            spec = mlp3_layers(self)
            if spec is not None:
                (l1, l2, l3), acts = spec
                y = MLP3.apply(h, l1[0], l1[1], l2[0], l2[1], l3[0], l3[1], acts, torch.is_grad_enabled())
                return y.reshape(*lead, y.shape[-1])
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
