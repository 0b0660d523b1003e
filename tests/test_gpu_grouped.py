"""GPU: grouped layer launches (mh_gemm_f32_grouped, mh_linear_backward_grouped,
mh_head_backward_grouped) and the twin-critic network built on them (apprfunc/_twin.py).

Each group of a grouped launch runs the ungrouped kernel's arithmetic on its own operands, so it
must equal the ungrouped entry point on that group's (contiguous copies of the) operands BIT FOR
BIT. The twin critics as a whole (layer-1 weight gradient over the joint 2H outputs, the summed
input gradient) are checked against float64 autograd of the two nn.Module critics."""
import ctypes

import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N

pytestmark = pytest.mark.gpu


def _rand(*s, g, scale=1.0):
    return (torch.randn(*s, device="cuda", generator=g) * scale).contiguous()


def _gemm(A, B, bias, M, Nn, K, lda, ldb, ta, tb, act):
    C = torch.empty(M, Nn, device="cuda")
    ws = ctypes.c_int64()
    N.check(N.lib().mh_gemm_workspace(M, Nn, K, ctypes.byref(ws)), "ws")
    w = torch.empty(max(1, ws.value), device="cuda")
    N.check(N.lib().mh_gemm_f32(N.ptr(A), N.ptr(B), N.ptr(bias), N.ptr(C), M, Nn, K, lda, ldb, Nn, ta, tb, act,
                                N.ptr(w), N.stream_of()), "gemm")
    return C


@pytest.mark.parametrize("M,H,act", [(5120, 256, 1), (2048, 64, 0), (4099, 128, 2)])
def test_grouped_tall_and_gemv_equal_ungrouped(M, H, act):
    g = torch.Generator(device="cuda").manual_seed(M + H)
    h1 = _rand(M, 2 * H, g=g)
    W2, b2 = _rand(2, H, H, g=g, scale=0.05), _rand(2, H, g=g)
    W3, b3 = _rand(2, H, g=g, scale=0.05), _rand(2, g=g)
    h2 = torch.full((M, 2 * H), float("nan"), device="cuda")
    q = torch.empty(2, M, device="cuda")
    st = N.stream_of()
    N.check(N.lib().mh_gemm_f32_grouped(N.ptr(h1), N.ptr(W2), N.ptr(b2), N.ptr(h2), M, H, H, 2 * H, H, 2 * H, 0, 1,
                                        act, 2, H, H * H, H, H, st), "grouped tall")
    N.check(N.lib().mh_gemm_f32_grouped(N.ptr(h2), N.ptr(W3), N.ptr(b3), N.ptr(q), M, 1, H, 2 * H, H, 1, 0, 1, 0, 2,
                                        H, H, 1, M, st), "grouped gemv")
    for k in range(2):
        x = h1[:, k * H:(k + 1) * H].contiguous()
        ref = _gemm(x, W2[k], b2[k], M, H, H, H, H, 0, 1, act)
        assert torch.equal(h2[:, k * H:(k + 1) * H], ref), k
        r3 = _gemm(ref, W3[k], b3[k:k + 1], M, 1, H, H, H, 0, 1, 0)
        assert torch.equal(q[k], r3[:, 0]), k


def test_grouped_gemm_rejects_unsupported_shape():
    x = torch.zeros(100, 32, device="cuda")
    w = torch.zeros(2, 16, 16, device="cuda")
    c = torch.zeros(100, 32, device="cuda")
    rc = N.lib().mh_gemm_f32_grouped(N.ptr(x), N.ptr(w), None, N.ptr(c), 100, 16, 16, 32, 16, 32, 0, 1, 0, 2, 16, 256,
                                     0, 16, N.stream_of())
    assert rc != 0


@pytest.mark.parametrize("M,H,want_w", [(5120, 256, True), (5120, 256, False), (3000, 128, True)])
def test_grouped_linear_and_head_backward_equal_ungrouped(M, H, want_w):
    g = torch.Generator(device="cuda").manual_seed(7 * M + H)
    h1 = torch.relu(_rand(M, 2 * H, g=g))
    h2 = torch.relu(_rand(M, 2 * H, g=g))
    W2, W3 = _rand(2, H, H, g=g, scale=0.05), _rand(2, H, g=g, scale=0.05)
    dq = _rand(2, M, g=g)
    st = N.stream_of()
    hw = ctypes.c_int64()
    N.check(N.lib().mh_head_backward_workspace(M, 1, H, ctypes.byref(hw)), "hw")
    wsh = torch.empty(2 * hw.value, device="cuda")
    dh2 = torch.empty(M, 2 * H, device="cuda")
    gW3, gb3 = torch.empty(2, H, device="cuda"), torch.empty(2, device="cuda")
    N.check(N.lib().mh_head_backward_grouped(N.ptr(dq), N.ptr(h2), N.ptr(W3), M, 1, H, 2 * H, 2 * H, 2, M, H, H, H, H,
                                             1, N.ptr(dh2), N.ptr(gW3) if want_w else None,
                                             N.ptr(gb3) if want_w else None, N.ptr(wsh) if want_w else None, st),
            "grouped head")
    ok, lw = ctypes.c_int32(), ctypes.c_int64()
    N.check(N.lib().mh_linear_backward_plan(M, H, H, 1, int(want_w), int(want_w), ctypes.byref(ok), ctypes.byref(lw)),
            "plan")
    assert ok.value
    wsl = torch.empty(max(1, 2 * lw.value), device="cuda")
    dh1 = torch.empty(M, 2 * H, device="cuda")
    gW2, gb2 = torch.empty(2, H, H, device="cuda"), torch.empty(2, H, device="cuda")
    N.check(N.lib().mh_linear_backward_grouped(N.ptr(dh2), N.ptr(h2), 1, N.ptr(h1), N.ptr(W2), M, H, H, 2 * H, 2 * H,
                                               2 * H, 2, H, H, H * H, H, H * H, H, N.ptr(dh1),
                                               N.ptr(gW2) if want_w else None, N.ptr(gb2) if want_w else None,
                                               N.ptr(wsl), st), "grouped linear backward")
    for k in range(2):
        sl = slice(k * H, (k + 1) * H)
        x2, x1 = h2[:, sl].contiguous(), h1[:, sl].contiguous()
        d2 = torch.empty(M, H, device="cuda")
        w3, b3 = torch.empty(1, H, device="cuda"), torch.empty(1, device="cuda")
        ws1 = torch.empty(hw.value, device="cuda")
        N.check(N.lib().mh_head_backward(N.ptr(dq[k]), N.ptr(x2), N.ptr(W3[k]), M, 1, H, N.ptr(d2),
                                         N.ptr(w3) if want_w else None, N.ptr(b3) if want_w else None,
                                         N.ptr(ws1) if want_w else None, st), "head")
        assert torch.equal(dh2[:, sl], d2), k
        if want_w:
            assert torch.equal(gW3[k], w3[0]) and torch.equal(gb3[k:k + 1], b3), k
        d1 = torch.empty(M, H, device="cuda")
        w2, bb2 = torch.empty(H, H, device="cuda"), torch.empty(H, device="cuda")
        ws2 = torch.empty(max(1, lw.value), device="cuda")
        N.check(N.lib().mh_linear_backward(N.ptr(d2), N.ptr(x2), 1, N.ptr(x1), N.ptr(W2[k]), M, H, H, N.ptr(d1),
                                           N.ptr(w2) if want_w else None, N.ptr(bb2) if want_w else None, N.ptr(ws2),
                                           st), "linear backward")
        assert torch.equal(dh1[:, sl], d1), k
        if want_w:
            assert torch.equal(gW2[k], w2) and torch.equal(gb2[k], bb2), k


def _critics(K, H, seed):
    from msacl_amd.apprfunc.mlp import ActionValue
    torch.manual_seed(seed)
    kw = dict(obs_dim=K - 4, act_dim=4, hidden_sizes=(H, H), hidden_activation="relu", output_activation="linear")
    return ActionValue(**kw).cuda(), ActionValue(**kw).cuda()


def _ref64(q1, q2, x):
    """float64 autograd of the two module critics (parameter gradients and input gradient)."""
    import copy
    out = []
    xd = x.double().detach().requires_grad_(True)
    for q in (q1, q2):
        qd = copy.deepcopy(q).double()
        out.append((qd, qd.q(xd).squeeze(-1)))
    return xd, out


def test_twin_critic_matches_float64_autograd():
    from msacl_amd.apprfunc._twin import TwinCritic, TwinQ
    K, H, M = 16, 256, 5120
    q1, q2 = _critics(K, H, 3)
    before = [p.detach().clone() for q in (q1, q2) for p in q.parameters()]
    tc = TwinCritic.build(q1, q2)
    assert tc is not None
    # joining kept the values and made every parameter a view of the joint buffers
    for p, b in zip([p for q in (q1, q2) for p in q.parameters()], before):
        assert torch.equal(p.detach(), b)
    assert q1.q[0].weight.data_ptr() == tc.W1.data_ptr() and q2.q[2].weight.data_ptr() == tc.W2[1].data_ptr()
    g = torch.Generator(device="cuda").manual_seed(11)
    x = _rand(M, K, g=g)
    dq = _rand(2, M, g=g)
    q, h1, h2 = tc.forward(x)
    xd, ref = _ref64(q1, q2, x)
    for k in range(2):
        r = ref[k][1]
        assert (q[k].double() - r).abs().max().item() <= 1e-5 * (1 + r.abs().max().item()), k
    # parameter gradients
    tc.backward_weights(x, dq, h1, h2)
    torch.autograd.backward([ref[0][1], ref[1][1]], [dq[0].double(), dq[1].double()])
    for k, q in enumerate((q1, q2)):
        for p, pd in zip(q.parameters(), ref[k][0].parameters()):
            scale = pd.grad.abs().max().item() + 1e-12
            assert (p.grad.double() - pd.grad).abs().max().item() <= 1e-5 * scale, (k, tuple(p.shape))
    # input gradient of the frozen pair under autograd (TwinQ): the sum of both critics'
    xg = x.clone().requires_grad_(True)
    a, b = TwinQ.apply(xg, tc)
    torch.autograd.backward([a, b], [dq[0], dq[1]])
    scale = xd.grad.abs().max().item()
    assert (xg.grad.double() - xd.grad).abs().max().item() <= 1e-5 * scale
    # the optimiser-facing view: a joint storage re-pointed away is detected and re-joined
    q1.q[0].weight.data = q1.q[0].weight.data.clone()
    assert tc.joined() and q1.q[0].weight.data_ptr() == tc.W1.data_ptr()


def test_msacl_update_grouped_equals_two_networks(tmp_path):
    """One MSACL even (policy) update and one odd update at the bench shapes through the grouped
    twin critics vs the two-network path from the same state and batch: losses within f32
    summation-order noise, parameters within Adam's step scale."""
    import copy
    from msacl_amd.algorithm.msacl import MSACL
    from msacl_amd.utils.config import default_msacl_args
    from oracle import envs as OE
    cls = OE.QuadTracking
    a = default_msacl_args(obs_dim=12, act_dim=4, action_type="continu", action_high_limit=cls.act_high.copy(),
                           action_low_limit=cls.act_low.copy(), replay_batch_size=256, n_step=20)
    algs = []
    for grouped in (True, False):
        torch.manual_seed(0)
        kw = dict(a, alg_twin_grouped=grouped, alg_use_graph=False, device=torch.device("cuda", 0))
        algs.append(MSACL(**kw))
    algs[1].networks.load_state_dict(algs[0].networks.state_dict())
    g = torch.Generator(device="cuda").manual_seed(5)
    B, n = 256, 20
    lo = torch.as_tensor(cls.act_low, dtype=torch.float32, device="cuda")
    hi = torch.as_tensor(cls.act_high, dtype=torch.float32, device="cuda")
    act = lo + (hi - lo) * torch.sigmoid(_rand(B, n, 4, g=g))  # inside the action box (TanhGauss log-prob)
    batch = {"obs": _rand(B, n, 12, g=g), "act": act.contiguous(), "rew": _rand(B, n, g=g),
             "cost": _rand(B, n, g=g).abs(), "obs2": _rand(B, n, 12, g=g),
             "done": (torch.rand(B, n, device="cuda", generator=g) < 0.05).float(), "logp": _rand(B, n, g=g)}
    for it in (0, 1):
        outs = []
        for alg in algs:
            torch.manual_seed(100 + it)  # the same rsample noise for both
            tb = alg.model_update(copy.copy(batch), it)
            outs.append(None if tb is None else dict(tb))
        if outs[0] is not None:
            for k, v in outs[0].items():
                if "time" in k:
                    continue
                assert v == v and abs(v - outs[1][k]) <= 1e-4 * (1 + abs(v)), (it, k, v, outs[1][k])
    # Adam's first steps are ~lr * sign(g): a gradient element at the summation-order noise level
    # may take the other sign (2 lr per step apart); every other element agrees to f32 noise
    for (k, p), (_, r) in zip(algs[0].networks.named_parameters(), algs[1].networks.named_parameters()):
        d = (p.detach() - r.detach()).abs()
        assert d.max().item() <= 2 * 2 * 1e-3 + 1e-6, k
        assert (d > 1e-5).float().mean().item() <= 2e-3, (k, (d > 1e-5).sum().item(), d.numel())
