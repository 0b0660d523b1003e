"""GPU: the fused 3-layer MLP forward (mh_mlp3_forward, csrc/mlp_fused.hip) against a float64
evaluation of each layer (RL/apprfunc/mlp.py:18-30: Linear -> act -> Linear -> act -> Linear -> act).

Each layer is checked on the kernel's own input to it (h1 and h2 as the kernel wrote them), so the
bound does not compound: |err| <= 2e-6 sqrt(K) sum_k |a_k w_k| + 1e-6 (tests/test_gpu_gemm.py's
f32-accumulation bound), plus tanhf's ulp where the activation is tanh. Shapes: the policy
(K1 = D, ReLU, N3 = 2A), the critics (K1 = D + A, N3 = 1), the Lyapunov network (tanh, N3 = 256),
ragged row counts and every supported K1; the grouped (twin-critic) launch; and the MLP module's
forward / backward through the fused launch against the per-layer launches."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn as nn

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.apprfunc import _fused as F

pytestmark = pytest.mark.gpu
ACT = {0: lambda v: v, 1: lambda v: np.maximum(v, 0.0), 2: np.tanh}


def _params(K1, N3, seed, H=256, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    f = lambda *s: (torch.rand(*s, generator=g) * 2 - 1)  # noqa: E731
    W1, b1 = f(H, K1) / K1 ** 0.5 * scale, f(H) * 0.1
    W2, b2 = f(H, H) / H ** 0.5 * scale, f(H) * 0.1
    W3, b3 = f(N3, H) / H ** 0.5 * scale, f(N3) * 0.1
    return [t.cuda().contiguous() for t in (W1, b1, W2, b2, W3, b3)]


def _check_layer(out, inp, W, b, act, what):
    a, w = inp.double().cpu().numpy(), W.double().cpu().numpy()
    lin = a @ w.T + b.double().cpu().numpy()
    mag = np.abs(a) @ np.abs(w).T + np.abs(b.double().cpu().numpy())
    ref = ACT[act](lin)
    tol = 2e-6 * (a.shape[1] ** 0.5) * mag + 1e-6 + (2e-7 * np.abs(ref) if act == 2 else 0.0)
    err = np.abs(out.double().cpu().numpy() - ref)
    assert np.all(err <= tol), f"{what}: max err {err.max():.3e}, worst ratio {(err / tol).max():.3f}"


def _run(x, ps, acts, keep=True, N3=None):
    W1, b1, W2, b2, W3, b3 = ps
    M, K1 = x.shape
    N3 = W3.shape[0]
    h1 = torch.full((M, 256), float("nan"), device="cuda") if keep else None
    h2 = torch.full((M, 256), float("nan"), device="cuda") if keep else None
    y = torch.full((M, N3), float("nan"), device="cuda")
    N.check(N.lib().mh_mlp3_forward(N.ptr(x), M, K1, K1, *[N.ptr(t) for t in ps], 256, N3, *acts, N.ptr(h1), N.ptr(h2),
                                    256, N.ptr(y), N3, 1, None, N.stream_of()), "mh_mlp3_forward")
    torch.cuda.synchronize()
    return y, h1, h2


CASES = [("policy", 5120, 12, 8, (1, 1, 0)), ("critic", 5120, 16, 1, (1, 1, 0)), ("lyapunov", 10240, 12, 256, (2, 2, 0)),
         ("ragged", 1000, 12, 8, (1, 1, 0)), ("tiny", 17, 6, 2, (1, 1, 0)), ("k1", 300, 1, 4, (1, 2, 0)),
         ("k20", 777, 20, 16, (2, 1, 0)), ("k32", 2048, 32, 64, (1, 1, 2)), ("n128", 512, 14, 128, (2, 2, 1))]


@pytest.mark.parametrize("name,M,K1,N3,acts", CASES, ids=[c[0] for c in CASES])
def test_mlp3_forward_matches_float64_layers(name, M, K1, N3, acts):
    ps = _params(K1, N3, seed=M + K1)
    x = (torch.rand(M, K1, generator=torch.Generator().manual_seed(1)) * 4 - 2).cuda()
    y, h1, h2 = _run(x, ps, acts)
    W1, b1, W2, b2, W3, b3 = ps
    _check_layer(h1, x, W1, b1, acts[0], "layer 1")
    _check_layer(h2, h1, W2, b2, acts[1], "layer 2")
    _check_layer(y, h2, W3, b3, acts[2], "layer 3")
    # without the kept activations: the same output, bit for bit
    y2, _, _ = _run(x, ps, acts, keep=False)
    assert torch.equal(y, y2)


def test_mlp3_forward_grouped_equals_ungrouped():
    """Two networks of one shape in one launch (the twin critics' joint buffers: W1 [2H][K],
    W2 [2][H][H], W3 [2][H], h [M][2H]); each group equals its ungrouped launch bit for bit."""
    M, K, H = 5120, 16, 256
    a, b = _params(K, 1, seed=3), _params(K, 1, seed=4)
    W1 = torch.cat([a[0], b[0]]).contiguous()
    b1 = torch.cat([a[1], b[1]]).contiguous()
    W2 = torch.stack([a[2], b[2]]).contiguous()
    b2 = torch.stack([a[3], b[3]]).contiguous()
    W3 = torch.cat([a[4], b[4]]).contiguous()
    b3 = torch.cat([a[5], b[5]]).contiguous()
    x = torch.randn(M, K, device="cuda")
    h1 = torch.empty(M, 2 * H, device="cuda")
    h2 = torch.empty(M, 2 * H, device="cuda")
    q = torch.empty(2, M, device="cuda")
    gs = (ctypes.c_int64 * 9)(0, H * K, H, H * H, H, H, 1, H, M)
    N.check(N.lib().mh_mlp3_forward(N.ptr(x), M, K, K, N.ptr(W1), N.ptr(b1), N.ptr(W2), N.ptr(b2), N.ptr(W3), N.ptr(b3),
                                    H, 1, 1, 1, 0, N.ptr(h1), N.ptr(h2), 2 * H, N.ptr(q), 1, 2, gs, N.stream_of()),
            "grouped")
    for g, ps in enumerate((a, b)):
        y, k1, k2 = _run(x, ps, (1, 1, 0))
        assert torch.equal(q[g], y[:, 0]), g
        assert torch.equal(h1[:, g * H:(g + 1) * H], k1), g
        assert torch.equal(h2[:, g * H:(g + 1) * H], k2), g


def test_mlp3_rejects_unsupported_shapes():
    ps = _params(12, 8, seed=0)
    x = torch.zeros(64, 40, device="cuda")
    y = torch.empty(64, 8, device="cuda")
    assert N.lib().mh_mlp3_forward(N.ptr(x), 64, 40, 40, *[N.ptr(t) for t in ps], 256, 8, 1, 1, 0, None, None, 256,
                                   N.ptr(y), 8, 1, None, N.stream_of()) == -1  # K1 > 32
    assert N.lib().mh_mlp3_forward(N.ptr(x), 64, 12, 40, *[N.ptr(t) for t in ps], 256, 20, 1, 1, 0, None, None, 256,
                                   N.ptr(y), 20, 1, None, N.stream_of()) == -1  # N3 = 20


def _kink_margin_rows(x, mods, margin=1e-5):
    """Rows whose ReLU pre-activations (float64) all keep `margin` x the layer's max |z| from 0.
    Two correct f32 evaluations of a layer (different summation orders, or the split-f16 layer
    against the f32 one) differ by ~1e-7 of its scale; a unit that close to the kink can take
    either side of it, and its mask then differs between the two paths, moving every gradient of
    its row by a whole term: a comparison of two paths' gradients is only meaningful where both
    agree on every mask."""
    D = lambda t: t.detach().double().cpu()  # noqa: E731
    a, keep = D(x), torch.ones(x.shape[0], dtype=torch.bool)
    for lin in (mods[0], mods[2]):
        z = a @ D(lin.weight).T + D(lin.bias)
        keep &= (z.abs() > margin * float(z.abs().max())).all(1)
        a = z.clamp_min(0.0)
    return keep.to(x.device)


@pytest.mark.parametrize("acts", [(nn.ReLU, nn.ReLU, nn.Identity), (nn.Tanh, nn.Tanh, nn.Identity)])
def test_mlp_module_fused_forward_backward_matches_per_layer(acts):
    """The MLP module (apprfunc/_fused.py) through MLP3 vs through the per-layer LinearAct launches:
    outputs within the f32 summation-order bound, every gradient rtol 1e-4 / atol 1e-5 of its scale
    (ReLU: on rows clear of the kink, _kink_margin_rows)."""
    torch.manual_seed(0)
    mods = [nn.Linear(12, 256), acts[0](), nn.Linear(256, 256), acts[1](), nn.Linear(256, 8), acts[2]()]
    net = F.MLP(*mods).cuda()
    x = torch.randn(256 * 21, 12, device="cuda")
    if acts[0] is nn.ReLU:
        x = x[_kink_margin_rows(x, mods)]
    x = x[:256 * 20].reshape(256, 20, 12).requires_grad_(True)
    g = torch.randn(256, 20, 8, device="cuda")
    outs = []
    for on in (True, False):
        F._MLP3["on"] = on
        try:
            net.zero_grad()
            xx = x.detach().clone().requires_grad_(True)
            y = net(xx)
            y.backward(g)
            outs.append((y.detach(), xx.grad.clone(), [p.grad.clone() for p in net.parameters()]))
        finally:
            F._MLP3["on"] = True
    (ya, gxa, gpa), (yb, gxb, gpb) = outs
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5 * float(yb.abs().max()))
    for u, v in [(gxa, gxb)] + list(zip(gpa, gpb)):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-5 * float(v.abs().max()))


@pytest.mark.parametrize("K1,N3,acts", [(12, 8, (1, 1)), (16, 1, (1, 1)), (12, 256, (2, 2)), (20, 16, (2, 1)),
                                        (5, 64, (1, 2))])
def test_mlp3_backward_chain_matches_float64(K1, N3, acts):
    """mh_mlp3_backward: g2 = (dy W3) act2'(h2), g1 = (g2 W2) act1'(h1), dx = g1 W1, each checked on
    the kernel's own previous gradient against float64 (the forward's bound)."""
    M = 3000
    ps = _params(K1, N3, seed=K1 * N3)
    W1, b1, W2, b2, W3, b3 = ps
    x = torch.randn(M, K1, device="cuda")
    y, h1, h2 = _run(x, ps, acts + (0,))
    dy = torch.randn(M, N3, device="cuda")
    g2 = torch.empty(M, 256, device="cuda")
    g1 = torch.empty(M, 256, device="cuda")
    dx = torch.empty(M, K1, device="cuda")
    N.check(N.lib().mh_mlp3_backward(N.ptr(dy), N3, N.ptr(h1), N.ptr(h2), 256, N.ptr(W1), N.ptr(W2), N.ptr(W3), M,
                                     K1, 256, N3, acts[0], acts[1], N.ptr(g2), N.ptr(g1), 256, N.ptr(dx), K1, 1, None,
                                     N.stream_of()), "mh_mlp3_backward")
    torch.cuda.synchronize()
    D = lambda t: t.double().cpu().numpy()  # noqa: E731
    dact = {1: lambda h: (h > 0).astype(np.float64), 2: lambda h: 1.0 - h * h}

    def check(out, g, W, h, act, what):
        lin = D(g) @ D(W)
        mag = np.abs(D(g)) @ np.abs(D(W))
        ref = lin * (dact[act](D(h)) if act else 1.0)
        tol = (2e-6 * (g.shape[1] ** 0.5) * mag + 1e-6) * (np.abs(dact[act](D(h))) if act else 1.0) + 1e-7
        err = np.abs(D(out) - ref)
        assert np.all(err <= tol), f"{what}: max err {err.max():.3e}, worst ratio {(err / tol).max():.3f}"

    check(g2, dy, W3, h2, acts[1], "g2")
    check(g1, g2, W2, h1, acts[0], "g1")
    check(dx, g1, W1, None, 0, "dx")


def test_twin_input_grad_chain_equals_per_layer():
    """TwinCritic.input_grad through mh_mlp3_backward (both critics, the input gradients summed in
    one launch) vs the per-layer launches: equal to the f32 summation-order bound."""
    from msacl_amd.apprfunc._twin import TwinCritic
    from msacl_amd.apprfunc.mlp import ActionValue
    torch.manual_seed(1)
    kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu", output_activation="linear")
    q1, q2 = ActionValue(**kw).cuda(), ActionValue(**kw).cuda()
    tc = TwinCritic.build(q1, q2)
    M = 5120
    x = torch.randn(M, 16, device="cuda")
    q, h1, h2 = tc.forward(x)
    dq = torch.randn(2, M, device="cuda")
    outs = []
    for on in (True, False):
        F._MLP3["on"] = on
        try:
            outs.append(tc.input_grad(dq, h1, h2))
        finally:
            F._MLP3["on"] = True
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-5 * float(outs[1].abs().max()))


@pytest.mark.parametrize("M", [5120, 3001])
def test_twin_forward_pair_equals_two_forwards(M):
    """TwinCritic.forward_pair (mh_mlp3_forward_pair: the critics and the target critics as the two
    network sets of one launch) equals the two separate forwards bit for bit."""
    from msacl_amd.apprfunc._twin import TwinCritic
    from msacl_amd.apprfunc.mlp import ActionValue
    torch.manual_seed(2)
    kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu", output_activation="linear")
    nets = [ActionValue(**kw).cuda() for _ in range(4)]
    tc, tt = TwinCritic.build(nets[0], nets[1]), TwinCritic.build(nets[2], nets[3])
    x, xo = torch.randn(M, 16, device="cuda"), torch.randn(M, 16, device="cuda")
    q, h1, h2, qo = tc.forward_pair(x, tt, xo)
    q_ref, h1_ref, h2_ref = tc.forward(x)
    qo_ref, _, _ = tt.forward(xo, keep=False)
    for a, b in ((q, q_ref), (h1, h1_ref), (h2, h2_ref), (qo, qo_ref)):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("rows", [5120, 3001])
def test_weight_grads_multi_matches_float64(rows):
    """mh_weight_grads: the three layers' dW = g^T x and db = column sums of g of a policy-shaped MLP
    (a narrow output layer computed transposed, a 256 x 256 layer, a K1 = 12 input layer) in two
    launches, each element against float64 within 2e-6 sqrt(rows) sum|g x| + 1e-6."""
    from msacl_amd.apprfunc._fused import weight_grads
    torch.manual_seed(rows)
    dev = "cuda"
    g3, h2 = torch.randn(rows, 8, device=dev), torch.rand(rows, 256, device=dev)
    g2, h1 = torch.randn(rows, 256, device=dev), torch.rand(rows, 256, device=dev)
    g1, x = torch.randn(rows, 256, device=dev), torch.randn(rows, 12, device=dev)
    outs = [(torch.empty(8, 256, device=dev), torch.empty(8, device=dev)),
            (torch.empty(256, 256, device=dev), torch.empty(256, device=dev)),
            (torch.empty(256, 12, device=dev), None)]
    weight_grads([(g3, 8, h2, 256, 8, 256) + outs[0], (g2, 256, h1, 256, 256, 256) + outs[1],
                  (g1, 256, x, 12, 256, 12) + outs[2]], rows, torch.device(dev))
    torch.cuda.synchronize()
    D = lambda t: t.double().cpu().numpy()  # noqa: E731
    for (g, xin), (dw, db) in zip(((g3, h2), (g2, h1), (g1, x)), outs):
        ref = D(g).T @ D(xin)
        tol = 2e-6 * rows ** 0.5 * (np.abs(D(g)).T @ np.abs(D(xin))) + 1e-6
        assert np.all(np.abs(D(dw) - ref) <= tol), np.abs(D(dw) - ref).max()
        if db is not None:
            rb = D(g).sum(0)
            assert np.all(np.abs(D(db) - rb) <= 2e-6 * rows ** 0.5 * np.abs(D(g)).sum(0) + 1e-6)


def test_twin_weight_grads_fused_equals_per_layer():
    """TwinCritic.backward_weights through the chain + mh_weight_grads vs the per-layer launches:
    every gradient within rtol 1e-4 / atol 1e-5 of its scale. Both backward paths take the same
    kept activations (one forward): the forward's own paths are compared above, and the ReLU
    masks of two forwards can differ at units within rounding of the kink (_kink_margin_rows)."""
    from msacl_amd.apprfunc._twin import TwinCritic
    from msacl_amd.apprfunc.mlp import ActionValue
    torch.manual_seed(2)
    kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu", output_activation="linear")
    q1, q2 = ActionValue(**kw).cuda(), ActionValue(**kw).cuda()
    tc = TwinCritic.build(q1, q2)
    M = 5120
    x = torch.randn(M, 16, device="cuda")
    dq = torch.randn(2, M, device="cuda")
    res = []
    q, h1, h2 = tc.forward(x)
    for on in (True, False):
        F._MLP3["on"] = on
        try:
            tc.backward_weights(x, dq, h1, h2)
            res.append([t.clone() for t in (tc.gW1, tc.gb1, tc.gW2, tc.gb2, tc.gW3, tc.gb3)])
        finally:
            F._MLP3["on"] = True
    for u, v in zip(*res):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-5 * float(v.abs().max()))


@pytest.mark.parametrize("mode", [-1, 1, 3, 4])
def test_forward_row_tile_modes_equal_default(mode):
    """mh_mlp3_set_row_tiles changes only the grid (rows per workgroup), never the bits: the twin
    critics' forward (2 x 5,120 rows and a ragged 1,037) under each mode equals the default."""
    from msacl_amd.apprfunc._twin import TwinCritic
    from msacl_amd.apprfunc.mlp import ActionValue
    N = F._native()
    torch.manual_seed(11)
    kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu", output_activation="linear")
    tc = TwinCritic.build(ActionValue(**kw).cuda(), ActionValue(**kw).cuda())
    for M in (5120, 1037):
        x = torch.randn(M, 16, device="cuda")
        ref = [t.clone() for t in tc.forward(x)]
        N.check(N.lib().mh_mlp3_set_row_tiles(mode), "mh_mlp3_set_row_tiles")
        try:
            got = [t.clone() for t in tc.forward(x)]
        finally:
            N.lib().mh_mlp3_set_row_tiles(0)
        for a, b in zip(got, ref):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    assert N.lib().mh_mlp3_set_row_tiles(5) != 0


@pytest.mark.parametrize("M", [5120, 1037, 16400])
def test_twin_head_grads_folded_into_chain(M):
    """The q heads' dW3 / db3 formed inside the chain launch (mh_mlp3_backward_w3) equal the
    grouped head backward's bit for bit below 16,384 rows (same 16-row partials, same finish;
    1,037: a ragged last block), agree with float64 at any size, and leave g1 / g2 unchanged."""
    from msacl_amd.apprfunc import _twin as T
    from msacl_amd.apprfunc.mlp import ActionValue
    torch.manual_seed(M)
    kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu", output_activation="linear")
    tc = T.TwinCritic.build(ActionValue(**kw).cuda(), ActionValue(**kw).cuda())
    x = torch.randn(M, 16, device="cuda")
    dq = torch.randn(2, M, device="cuda")
    q, h1, h2 = tc.forward(x)
    res = []
    saved = T._FOLD_W3
    for fold in (True, False):
        T._FOLD_W3 = fold
        try:
            tc.backward_weights(x, dq, h1, h2)
            torch.cuda.synchronize()
            res.append([t.clone() for t in (tc.gW1, tc.gb1, tc.gW2, tc.gb2, tc.gW3, tc.gb3)])
        finally:
            T._FOLD_W3 = saved
    exact = M < 16384
    for u, v in zip(*res):
        if exact:
            torch.testing.assert_close(u, v, rtol=0, atol=0)
        else:
            torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6 * float(v.abs().max()))
    D = lambda t: t.double().cpu().numpy()  # noqa: E731
    gW3, gb3 = res[0][4], res[0][5]
    for qn in range(2):
        hq = D(h2[:, qn * 256:(qn + 1) * 256])
        ref = D(dq[qn]) @ hq
        tol = 2e-6 * M ** 0.5 * (np.abs(D(dq[qn])) @ np.abs(hq)) + 1e-6
        assert np.all(np.abs(D(gW3[qn]).reshape(-1) - ref) <= tol)
        assert abs(float(gb3[qn]) - D(dq[qn]).sum()) <= 2e-6 * M ** 0.5 * np.abs(D(dq[qn])).sum() + 1e-6


@pytest.mark.parametrize("M", [10240, 5376, 999])
def test_lyapunov_square_sum_fused_equals_separate(M):
    """LyapunovValue through MLP3SquareSum (mh_mlp3_forward_sqsum / mh_mlp3_backward_sqsum: the
    square sums and dy = dV 2y inside the MLP's launches) vs the MLP's launches + SquareSum: V and
    every gradient bit for bit."""
    from msacl_amd.apprfunc.mlp import LyapunovValue
    torch.manual_seed(5)
    lya = LyapunovValue(input_dim=12, hidden_sizes=[256, 256], hidden_activation="tanh", output_dim=256,
                        output_activation="linear").cuda()
    x = torch.randn(M, 12, device="cuda")
    dv = torch.randn(M, device="cuda")
    outs = []
    for fused in (True, False):
        F._MLP3["sqsum"] = fused  # off: the same fused MLP launches, then SquareSum's two launches
        try:
            lya.zero_grad()
            v = lya(x)
            v.backward(dv)
            outs.append([v.detach().clone()] + [p.grad.detach().clone() for p in lya.parameters()])
        finally:
            F._MLP3["sqsum"] = True
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_mlp3_forward_weights_past_the_split_range_and_nonfinite_rows():
    """The split-f16 hidden layers (csrc/mlp_fused.hip layer_cols_run_x3) scale weights by 2^10
    before the f16 split: a weight of 64 or more overflows its f16 hi. Such a row tile is recomputed
    by the f32 layer (x3_redo_nonfinite), so the results stay within the f32 bound. A non-finite
    input row gives non-finite outputs in that row only; the other row tiles keep their bits."""
    for K1, N3, acts in ((12, 256, (2, 2, 0)), (16, 1, (1, 1, 0))):
        ps = _params(K1, N3, seed=7)
        W1, b1, W2, b2, W3, b3 = ps
        W2[3, 5] = 100.0
        W2[200, 17] = -70.0
        if N3 > 16:
            W3[9, 250] = 65.0
        M = 1000
        x = (torch.rand(M, K1, generator=torch.Generator().manual_seed(3)) * 4 - 2).cuda()
        y, h1, h2 = _run(x, ps, acts)
        _check_layer(h2, h1, W2, b2, acts[1], "layer 2")
        _check_layer(y, h2, W3, b3, acts[2], "layer 3")
        xb = x.clone()
        xb[40, 0] = float("nan")
        yb, _, _ = _run(xb, ps, acts)
        assert torch.all(torch.isnan(yb[40]))
        tile = torch.arange(M, device="cuda") // 16 == 40 // 16
        assert torch.equal(yb[~tile], y[~tile])
        assert torch.all(torch.isfinite(yb[tile & (torch.arange(M, device="cuda") != 40)]))


@pytest.mark.parametrize("name,M,K1,N3,acts", CASES[:3], ids=[c[0] for c in CASES[:3]])
def test_mlp3_hidden_layer_error_near_f32_rounding(name, M, K1, N3, acts):
    """The hidden layer's error against float64 on the kernel's own input, in units of the f32
    dot-product scale 2^-24 sqrt(K) sum_k |a_k w_k|: the split-f16 form drops the lo.lo products
    (<= 2^-22 of each product) and keeps weights to 22 bits."""
    ps = _params(K1, N3, seed=M + K1)
    x = (torch.rand(M, K1, generator=torch.Generator().manual_seed(1)) * 4 - 2).cuda()
    y, h1, h2 = _run(x, ps, acts)
    W2, b2 = ps[2], ps[3]
    a, w = h1.double().cpu().numpy(), W2.double().cpu().numpy()
    lin = a @ w.T + b2.double().cpu().numpy()
    mag = np.abs(a) @ np.abs(w).T + np.abs(b2.double().cpu().numpy())
    ref = ACT[acts[1]](lin)
    ratio = np.abs(h2.double().cpu().numpy() - ref) / (2.0 ** -24 * 16 * mag + 1e-30)
    print(f"{name}: layer-2 error / (2^-24 sqrt(K) mag): max {ratio.max():.3f} mean {ratio.mean():.4f}")
    assert ratio.max() < 4.0
