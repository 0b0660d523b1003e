"""GPU: the fused layer backward mh_linear_backward (csrc/gemm.hip: g = dy * act'(y) formed inside
the tall dx GEMM and the deep dW GEMM, the bias gradient inside the latter) against PyTorch
autograd of the same nn.Linear + activation (RL/apprfunc/mlp.py:18-30), float64 reference.
Tolerance: each gradient within 2e-6 * sqrt(K) * (sum of |terms|) + 1e-6 of the float64 value
(K = the summed dimension), the f32-accumulation bound the GEMM tests use."""
import ctypes
import os

import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.apprfunc._fused import _linear_backward_fused

pytestmark = pytest.mark.gpu


def _case(rows, n_in, n_out, act, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(rows, n_in, device="cuda", generator=g)
    w = torch.randn(n_out, n_in, device="cuda", generator=g) / n_in ** 0.5
    b = torch.randn(n_out, device="cuda", generator=g) * 0.1
    pre = x @ w.t() + b
    y = torch.relu(pre) if act == 1 else (torch.tanh(pre) if act == 2 else pre)
    dy = torch.randn(rows, n_out, device="cuda", generator=g)
    return x, w, y.contiguous(), dy


def _check(got, ref, mag, K):
    err = (got.double() - ref).abs()
    tol = 2e-6 * (K ** 0.5) * mag + 1e-6
    assert bool((err <= tol).all()), f"max err {float(err.max()):.3e}"


@pytest.mark.parametrize("rows,n_in,n_out", [(5120, 256, 256), (10240, 256, 256), (3001, 128, 64), (5120, 64, 256)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_linear_backward_matches_float64(rows, n_in, n_out, act):
    x, w, y, dy = _case(rows, n_in, n_out, act, rows + n_in + act)
    out = _linear_backward_fused(dy, y, act, x, w, True, True, True)
    assert out is not None, "fused path not taken"
    dx, dw, db, _ = out
    yd = y.double()
    gd = dy.double() * ((yd > 0).double() if act == 1 else (1 - yd * yd) if act == 2 else 1.0)
    _check(dx, gd @ w.double(), gd.abs() @ w.double().abs(), n_out)
    _check(dw, gd.t() @ x.double(), gd.abs().t() @ x.double().abs(), rows)
    _check(db, gd.sum(0), gd.abs().sum(0), rows)
    # deterministic: repeat launches agree bit for bit
    dx2, dw2, db2, _ = _linear_backward_fused(dy, y, act, x, w, True, True, True)
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("need", [(True, False, False), (False, True, True), (False, True, False)])
def test_linear_backward_partial_requests(need):
    x, w, y, dy = _case(5120, 256, 256, 1, 7)
    out = _linear_backward_fused(dy, y, 1, x, w, *need)
    assert out is not None
    for got, wanted in zip(out[:3], need):
        assert (got is not None) == wanted
    gd = dy.double() * (y.double() > 0).double()
    if need[0]:
        _check(out[0], gd @ w.double(), gd.abs() @ w.double().abs(), 256)
    if need[1]:
        _check(out[1], gd.t() @ x.double(), gd.abs().t() @ x.double().abs(), 5120)
    if need[2]:
        _check(out[2], gd.sum(0), gd.abs().sum(0), 5120)


def test_linear_backward_plan_rejects():
    ok, ws = ctypes.c_int32(), ctypes.c_int64()
    for args in [(256, 256, 256, 1, 1, 1), (5120, 8, 256, 1, 1, 1), (5120, 256, 256, 0, 0, 1), (5120, 256, 12, 1, 0, 0)]:
        assert N.lib().mh_linear_backward_plan(*args, ctypes.byref(ok), ctypes.byref(ws)) == 0
        assert ok.value == 0, args
    assert N.lib().mh_linear_backward_plan(5120, 256, 256, 1, 1, 1, ctypes.byref(ok), ctypes.byref(ws)) == 0
    # dW partials + bias partials per split x column tile: S = 8 splits (the deep products' target
    # of 128 workgroups over 16 tiles of 64 x 64; MH_DEEP_WGS overrides it)
    S = _deep_splits(256, 256, 5120)
    assert ok.value == 1 and ws.value == S * 256 * 256 + S * 4 * 256


@pytest.mark.parametrize("rows,n_in", [(5120, 12), (5120, 16), (10240, 12), (3001, 4), (5120, 60)])
@pytest.mark.parametrize("act", [1, 2])
def test_linear_backward_narrow_input_dw_db(rows, n_in, act):
    """First layers (n_in < 64: the observation / observation + action inputs): dW and db through
    the deep kernel's single, partly used column tile (its columns past n_in read as zeros and are
    not stored), against float64; deterministic."""
    x, w, y, dy = _case(rows, n_in, 256, act, rows + n_in + 11 * act)
    out = _linear_backward_fused(dy, y, act, x, w, False, True, True)
    assert out is not None, "fused path not taken"
    _, dw, db, _ = out
    yd = y.double()
    gd = dy.double() * ((yd > 0).double() if act == 1 else (1 - yd * yd))
    _check(dw, gd.t() @ x.double(), gd.abs().t() @ x.double().abs(), rows)
    _check(db, gd.sum(0), gd.abs().sum(0), rows)
    _, dw2, db2, _ = _linear_backward_fused(dy, y, act, x, w, False, True, True)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


def _deep_splits(M, N, K):
    """gemm.hip deep_splits: about deep_target() workgroups (MH_DEEP_WGS, default 128) per product,
    slices of >= 2 of the K range's 64-deep chunks."""
    target = int(os.environ.get("MH_DEEP_WGS", "128"))
    tiles = (M // 64) * ((N + 63) // 64)
    chunks = -(-K // 64)
    S = max(1, min(-(-target // tiles), chunks // 2))
    per = -(-chunks // S)
    return -(-chunks // per)


def test_linear_backward_plan_narrow_input():
    ok, ws = ctypes.c_int32(), ctypes.c_int64()
    assert N.lib().mh_linear_backward_plan(5120, 256, 12, 0, 1, 1, ctypes.byref(ok), ctypes.byref(ws)) == 0
    # S splits (about deep_target() workgroups over the 4 row tiles) x (dW + one bias tile)
    S = _deep_splits(256, 12, 5120)
    assert ok.value == 1 and ws.value == S * 256 * 12 + S * 1 * 256
    for args in [(5120, 256, 12, 1, 1, 1), (5120, 256, 6, 0, 1, 1), (5120, 256, 68, 0, 1, 1)]:
        assert N.lib().mh_linear_backward_plan(*args, ctypes.byref(ok), ctypes.byref(ws)) == 0
        assert ok.value == 0, args


@pytest.mark.parametrize("rows,n_out,n_in", [(5120, 1, 256), (5120, 8, 256), (10240, 16, 256), (3001, 3, 128),
                                             (1024, 8, 300)])
@pytest.mark.parametrize("need", [(True, True, True), (True, False, False), (False, True, True)])
def test_head_backward_matches_float64(rows, n_out, n_in, need):
    """mh_head_backward (the identity output layer of a narrow head, n_out <= 16): dx = dy W,
    dW = dy^T x, db = column sums of dy, against float64; deterministic; each output only when
    requested."""
    from msacl_amd.apprfunc._fused import _head_backward
    x, w, _, dy = _case(rows, n_in, n_out, 0, rows + 7 * n_out + n_in)
    out = _head_backward(dy, x, w, *need)
    assert out is not None
    for got, wanted in zip(out[:3], need):
        assert (got is not None) == wanted
    dd = dy.double()
    if need[0]:
        _check(out[0], dd @ w.double(), dd.abs() @ w.double().abs(), n_out)
    if need[1]:
        _check(out[1], dd.t() @ x.double(), dd.abs().t() @ x.double().abs(), rows)
        _check(out[2], dd.sum(0), dd.abs().sum(0), rows)
    again = _head_backward(dy, x, w, *need)
    for a, b in zip(out[:3], again[:3]):
        assert a is None or torch.equal(a, b)


@pytest.mark.parametrize("rows,cols", [(10240, 256), (5376, 256), (77, 33), (1, 4)])
def test_square_sum_matches_torch(rows, cols):
    """mh_square_sum[_backward] (LyapunovValue's torch.pow(y, 2).sum(-1)): the value within f32
    summation-order rounding of torch's, the gradient bit-identical to pow's backward."""
    from msacl_amd.apprfunc._fused import SquareSum
    g = torch.Generator(device="cuda").manual_seed(rows + cols)
    y = torch.randn(rows, cols, device="cuda", generator=g)
    up = torch.randn(rows, device="cuda", generator=g)
    a, b = y.clone().requires_grad_(True), y.clone().requires_grad_(True)
    out = SquareSum.apply(a)
    ref = torch.pow(b, 2).sum(dim=-1, keepdim=True).squeeze(-1)
    _check(out, (y.double() ** 2).sum(-1), (y.double() ** 2).sum(-1), cols)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
    out.backward(up)
    ref.backward(up)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("rows,n_in,n_out", [(5120, 16, 256), (5120, 12, 256), (1031, 32, 100), (2048, 1, 7),
                                            (5119, 16, 512), (100, 7, 64), (33, 16, 128)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_dx_narrow_matches_float64(rows, n_in, n_out, act):
    """mh_dx_narrow (input gradient only of a narrow-input layer, act' on the fly) against float64."""
    x, w, y, dy = _case(rows, n_in, n_out, act, rows + n_in + n_out + act)
    dx = torch.empty(rows, n_in, device="cuda")
    N.check(N.lib().mh_dx_narrow(N.ptr(dy), N.ptr(y), act, N.ptr(w), rows, n_out, n_in, N.ptr(dx),
                                 N.stream_of(dy.device)), "mh_dx_narrow")
    yd = y.double()
    gd = dy.double() * ((yd > 0).double() if act == 1 else (1 - yd * yd) if act == 2 else 1.0)
    _check(dx, gd @ w.double(), gd.abs() @ w.double().abs(), n_out)
