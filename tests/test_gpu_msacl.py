"""GPU parity of the fused MSACL kernels against the NumPy oracle, and of one full
MSACL.model_update (networks + Adam + fused kernels) against the reference's own run
(tests/golden/msacl_update.npz, recorded rsample noise replayed)."""
import ctypes
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle import msacl as OM

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


_KEEP = []


def dev(a, dtype=torch.float32):
    """Device copy kept alive for the test's duration (a pointer into a freed temporary would
    let the caching allocator hand the same block to the next input)."""
    t = torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda").contiguous()
    _KEEP.append(t)
    return t


@pytest.mark.parametrize("B,n", [(256, 20), (64, 5), (7, 70)])
@pytest.mark.parametrize("weighted", [False, True])
def test_q_target_kernel(B, n, weighted):
    rng = np.random.default_rng(B + n)
    f = lambda *s: rng.standard_normal(s).astype(np.float32)  # noqa: E731
    q1, q2, q1t, q2t, nlp, rew = f(B, n), f(B, n), f(B, n), f(B, n), f(B, n), f(B, n) * 10
    done = (rng.uniform(size=(B, n)) < 0.1).astype(np.float32)
    la = np.float32(0.3)
    w = rng.uniform(0.2, 1.0, B).astype(np.float32) if weighted else None
    out = [torch.empty(B, n, device="cuda") for _ in range(3)] + [torch.empty(1, device="cuda"), torch.empty(B, device="cuda")]
    N.check(N.lib().mh_msacl_q_target(*[N.ptr(dev(a)) for a in (q1, q2, q1t, q2t, nlp, rew, done)], N.ptr(dev([la])),
                                      N.ptr(dev(w)) if weighted else None, 0.99, B, n, *[N.ptr(o) for o in out],
                                      N.stream_of()), "q")
    bk, loss, d1, d2, td = OM.q_target(q1, q2, q1t, q2t, nlp, rew, done, float(np.exp(la, dtype=np.float32)), 0.99, w)
    np.testing.assert_allclose(out[0].cpu().numpy(), bk, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out[1].cpu().numpy(), d1, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out[2].cpu().numpy(), d2, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out[3].item(), loss, rtol=1e-5)
    np.testing.assert_allclose(out[4].cpu().numpy(), td, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,n", [(256, 20), (7, 70)])
def test_q_target_stats_kernel(B, n):
    """mh_msacl_q_target_stats: the same backup / gradients / loss bits as mh_msacl_q_target, plus
    the logged critic means (msacl.py:211-222) from the same float64 reduction (rtol 1e-6 vs numpy
    float64 means rounded to float32)."""
    rng = np.random.default_rng(B * n)
    f = lambda *s: rng.standard_normal(s).astype(np.float32)  # noqa: E731
    q1, q2, q1t, q2t, nlp, rew = f(B, n) + 3, f(B, n) - 1, f(B, n), f(B, n), f(B, n), f(B, n)
    done = (rng.uniform(size=(B, n)) < 0.1).astype(np.float32)
    ins = [N.ptr(dev(a)) for a in (q1, q2, q1t, q2t, nlp, rew, done)] + [N.ptr(dev([np.float32(0.3)])), None]
    outs = [[torch.empty(B, n, device="cuda") for _ in range(3)] + [torch.empty(1, device="cuda"),
                                                                   torch.empty(B, device="cuda")] for _ in range(2)]
    means = torch.full((2,), float("nan"), device="cuda")
    N.check(N.lib().mh_msacl_q_target(*ins, 0.99, B, n, *[N.ptr(o) for o in outs[0]], N.stream_of()), "q")
    N.check(N.lib().mh_msacl_q_target_stats(*ins, 0.99, B, n, *[N.ptr(o) for o in outs[1]], N.ptr(means),
                                            N.stream_of()), "q stats")
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    np.testing.assert_allclose(means.cpu().numpy(), [np.float32(q1.astype(np.float64).mean()),
                                                     np.float32(q2.astype(np.float64).mean())], rtol=1e-6)


def test_kernel_noise_state_round_trip():
    """The update's in-kernel rsample noise (Philox keyed by (seed, row, a device counter)):
    each update advances the counter; restoring networks + optimisers + rng_state() replays an
    update bit for bit, and restoring everything BUT the rng state gives different noise and so a
    different update (the counter is part of the algorithm's saved state)."""
    import copy
    from msacl_amd.algorithm.msacl import MSACL
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=False)
    alg.networks.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")})
    nets = alg.networks
    opts = [nets.q1_optimizer, nets.q2_optimizer, nets.lyapunov_optimizer, nets.policy_optimizer, nets.alpha_optimizer]
    alg.model_update(data, 1)
    st = alg.rng_state()
    assert st["noise_ctr"] is not None, "the in-kernel noise path is off"
    sd = {k: v.detach().clone() for k, v in nets.state_dict().items()}
    osd = [copy.deepcopy(o.state_dict()) for o in opts]

    def update():
        tb = alg.model_update(data, 0)
        torch.cuda.synchronize()
        return {k: v for k, v in dict(tb).items() if "time" not in k.lower()}, \
            {k: v.detach().clone() for k, v in nets.state_dict().items()}

    def restore(rng):
        nets.load_state_dict(sd)
        for o, s in zip(opts, osd):
            o.load_state_dict(copy.deepcopy(s))
        if rng:
            alg.load_rng_state(st)
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)  # (library split-K GEMMs: no atomics)
    try:
        tb_a, p_a = update()
        assert not torch.equal(alg.rng_state()["noise_ctr"], st["noise_ctr"])  # the update advanced it
        restore(True)
        tb_b, p_b = update()
        restore(False)  # the counter keeps going: new noise
        tb_c, p_c = update()
    finally:
        torch.use_deterministic_algorithms(prev)
    assert tb_a == tb_b
    for k in p_a:
        assert torch.equal(p_a[k], p_b[k]), k
    assert any(not torch.equal(p_a[k], p_c[k]) for k in p_a)


def test_tb_ring_slots(monkeypatch):
    """The policy updates' logged scalars go to a device ring (mh_msacl_tb_pack_ring, no copy out
    of the replayed graph): a tb dict read within the ring's depth equals the eager update's, and
    one read after its slot was reused raises instead of returning another update's values."""
    import msacl_amd.algorithm.msacl as M
    monkeypatch.setattr(M, "_TB_SLOTS", 2)
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    tbs = {}
    for mode in (True, False):
        torch.manual_seed(0)
        alg = M.MSACL(**_msacl_kwargs(B, n), alg_use_graph=mode)
        alg.networks.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")})
        tbs[mode] = [alg.model_update(data, it) for it in range(8)][::2]
        assert alg._tb_ring.shape == (2, 8)
    for mode in (True, False):
        with pytest.raises(RuntimeError, match="reused its slot"):
            tbs[mode][0]["Loss/Critic loss-RL iter"]
    for k in tbs[False][-1]:
        if "time" not in k.lower():
            np.testing.assert_allclose(tbs[True][-1][k], tbs[False][-1][k], rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("B,n,D", [(256, 20, 12), (33, 5, 2), (5, 100, 6)])
def test_lyapunov_kernel(B, n, D):
    rng = np.random.default_rng(B * n)
    obs = (rng.standard_normal((B, n, D)) * 0.5).astype(np.float32)
    obs2 = (obs + rng.standard_normal((B, n, D)) * 0.1).astype(np.float32)
    V = (rng.uniform(0, 2, (B, n)) * (obs ** 2).sum(-1)).astype(np.float32)
    V2 = (rng.uniform(0, 2, (B, n)) * (obs2 ** 2).sum(-1)).astype(np.float32)
    logp = rng.standard_normal((B, n)).astype(np.float32)
    old = (logp + rng.standard_normal((B, n)) * 0.3).astype(np.float32)
    c, w, s = OM.coefficients(n)
    outs = [torch.empty(B, n, device="cuda"), torch.empty(B, n, device="cuda"), torch.empty(B, device="cuda"),
            torch.empty(1, device="cuda"), torch.empty(B, n, device="cuda"), torch.empty(B, n, device="cuda")]
    N.check(N.lib().mh_msacl_lyapunov(*[N.ptr(dev(a)) for a in (logp, old, V, V2, obs, obs2, c, w, s)], 1.0, 2.0, 1.0,
                                      10.0, B, n, D, *[N.ptr(o) for o in outs], N.stream_of()), "lya")
    ic, esl, ld, loss, dV, dV2 = OM.lyapunov(logp, old, V, V2, obs, obs2, c, w, s, 1.0, 2.0, 1.0, 10.0)
    np.testing.assert_allclose(outs[0].cpu().numpy(), ic, rtol=1e-5, atol=1e-6)
    e = outs[1].cpu().numpy()
    assert np.mean(e == esl) > 0.999  # ESL can flip only where the norm difference is ~0
    np.testing.assert_allclose(outs[2].cpu().numpy(), ld, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(outs[3].item(), loss, rtol=1e-4)
    np.testing.assert_allclose(outs[4].cpu().numpy(), dV, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(outs[5].cpu().numpy(), dV2, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("B,n", [(256, 20), (9, 3)])
def test_stability_advantage_and_ppo_clip(B, n):
    rng = np.random.default_rng(B)
    V0 = rng.uniform(0, 3, B).astype(np.float32)
    V2 = rng.uniform(0, 3, (B, n)).astype(np.float32)
    ratio = rng.uniform(0.7, 1.3, B).astype(np.float32)
    ratio[:3] = [np.float32(0.9), np.float32(1.1), np.float32(1.0)]
    c, w, s = OM.coefficients(n)
    adv_raw = torch.empty(B, device="cuda")
    stats = torch.empty(2, dtype=torch.float64, device="cuda")
    N.check(N.lib().mh_msacl_stability_adv(N.ptr(dev(V0)), N.ptr(dev(V2)), N.ptr(dev(w)), N.ptr(dev(s)), B, n,
                                           N.ptr(adv_raw), N.ptr(stats), N.stream_of()), "adv")
    adv, loss, dr = torch.empty(B, device="cuda"), torch.empty(1, device="cuda"), torch.empty(B, device="cuda")
    N.check(N.lib().mh_msacl_ppo_clip(N.ptr(dev(ratio)), N.ptr(adv_raw), N.ptr(stats), float(B), 0.1, B, N.ptr(adv),
                                      N.ptr(loss), N.ptr(dr), N.stream_of()), "ppo")
    a_raw, a, l, g = OM.stability(V0, V2, ratio, w, s, 0.1)
    np.testing.assert_allclose(adv_raw.cpu().numpy(), a_raw, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(adv.cpu().numpy(), a, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.item(), l, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dr.cpu().numpy(), g, rtol=1e-4, atol=1e-7)


# ------------------------------------------------------------------ full update vs reference
def _msacl_kwargs(B, n):
    from oracle import envs as OE
    cls = OE.QuadTracking
    return dict(env_name="QuadTracking", obs_dim=12, act_dim=4, action_type="continu",
                action_high_limit=cls.act_high.copy(), action_low_limit=cls.act_low.copy(),
                value_func_name="ActionValue", value_func_type="MLP", value_hidden_sizes=[64, 64],
                value_hidden_activation="relu", value_output_activation="linear",
                lyapunov_func_name="LyapunovValue", lyapunov_func_type="MLP", lyapunov_hidden_sizes=[64, 64],
                lyapunov_hidden_activation="tanh", lyapunov_output_dim=32, lyapunov_output_activation="linear",
                lyapunov_single_input_dim=False, policy_func_name="StochaPolicy", policy_func_type="MLP",
                policy_act_distribution="TanhGaussDistribution", policy_hidden_sizes=[64, 64],
                policy_hidden_activation="relu", policy_min_log_std=-20, policy_max_log_std=1,
                q_learning_rate=1e-3, lyapunov_learning_rate=1e-3, policy_learning_rate=3e-4, alpha_learning_rate=1e-3,
                lya_diff_scale=10.0, lya_zero_scale=1.0, lya_positive_scale=1.0, gamma=0.99, retrace_lambda=0.95,
                tau=0.005, disable_auto_alpha=False, alpha=1.0, set_alpha_bound=False, alpha_bound=2.0, n_step=n,
                policy_frequency=2, target_network_frequency=1, anneal_lr=False, alpha1=1, alpha2=2, lya_eta=0.15,
                clip_coef=0.1, replay_batch_size=B, max_iteration=1000, buffer_name="nstep_replay_buffer")


def test_full_model_update_matches_reference(monkeypatch):
    import torch.distributions.normal as tdn
    from msacl_amd.algorithm.msacl import MSACL
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    alg = MSACL(**_msacl_kwargs(B, n))
    sd = {k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")}
    alg.networks.load_state_dict(sd)
    eps = [g[f"eps{i}"] for i in range(4)]
    it = iter(eps)
    monkeypatch.setattr(tdn, "_standard_normal",
                        lambda shape, dtype, device: torch.as_tensor(next(it), dtype=dtype, device=device).reshape(shape))
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    tb = alg.model_update(data, 0)
    ref_tb = dict(zip([str(k) for k in g["tb_keys"]], g["tb_vals"]))
    for k, v in tb.items():
        if "time" in k.lower():
            continue
        np.testing.assert_allclose(v, ref_tb[k], rtol=2e-4, atol=1e-5, err_msg=k)
    _compare_params(alg, g, "after0/")
    assert alg.model_update(data, 1) is None
    _compare_params(alg, g, "after1/")


def _compare_params(alg, g, prefix):
    mine = alg.networks.state_dict()
    worst = []
    for k in g.files:
        if not k.startswith(prefix):
            continue
        ref = g[k]
        got = mine[k[len(prefix):]].detach().cpu().numpy()
        bad = ~np.isclose(got, ref, rtol=1e-4, atol=3e-5)
        worst.append(bad.mean())
        assert not bad.any(), (k, bad.sum(), np.abs(got - ref).max())  # every element (no outlier allowance)
    assert worst


def test_graph_replayed_update_trains():
    """The HIP-graph path (warm -> capture -> replay, both even/odd branches) runs, keeps the
    parameters finite and fits a fixed batch like the eager path."""
    from msacl_amd.algorithm.msacl import MSACL
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    losses = {}
    for mode in (True, False):
        torch.manual_seed(0)
        alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=mode)
        sd = {k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")}
        alg.networks.load_state_dict(sd)
        hist = []
        for it in range(12):
            tb = alg.model_update(data, it)
            if tb is not None:
                hist.append(tb["Loss/Critic loss-RL iter"])
        assert all(torch.isfinite(p).all() for p in alg.networks.parameters())
        if mode:
            assert len(alg._graphs) == 2
        losses[mode] = hist
    for mode, h in losses.items():
        assert h[-1] < h[0], (mode, h)
    np.testing.assert_allclose(losses[True][0], losses[False][0], rtol=1e-5)


def test_segmented_graph_update_equals_single_graph(monkeypatch):
    """Data-parallel capture (utils/dist.py GraphSegments: the update graph cut at every
    all-reduce, forced here on one GPU) replays the same kernels as the single-graph path and the
    eager path: parameters bit-identical after several updates (fixed rsample noise)."""
    import torch.distributions.normal as tdn
    from msacl_amd.algorithm.msacl import MSACL
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    noise = {}

    def fixed(shape, dtype, device):
        key = tuple(shape)
        if key not in noise:
            gen = torch.Generator(device="cuda").manual_seed(len(noise) + 1)
            noise[key] = torch.randn(key, dtype=dtype, device=device, generator=gen)
        return noise[key]

    monkeypatch.setattr(tdn, "_standard_normal", fixed)
    states = {}
    for mode in ("eager", "graph", "segments"):
        alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=(mode != "eager"),
                    alg_force_graph_segments=(mode == "segments"))
        sd = {k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")}
        alg.networks.load_state_dict(sd)
        for it in range(6):
            alg.model_update(data, it)
        if mode == "segments":
            seg = alg._graphs[(True, True)][0]
            assert len(seg.graphs) > 1 and len(seg.ops) == len(seg.graphs) - 1
        states[mode] = {k: v.detach().clone() for k, v in alg.networks.state_dict().items()}
    for mode in ("graph", "segments"):
        for k, v in states["eager"].items():
            assert torch.equal(v, states[mode][k]), (mode, k)


def test_segmented_graph_collectives_bind_the_captured_gradients(monkeypatch):
    """Data-parallel replay with a stand-in collective (world size 2 faked; all_reduce multiplies
    by 3, so every all-reduced gradient is scaled by 1.5 after the average): the graph chain of
    each update branch must all-reduce the gradient tensors ITS graphs write, although the
    other branch's capture re-points p.grad. Eager and segmented runs agree bit for bit."""
    import torch.distributions.normal as tdn
    from msacl_amd.algorithm.msacl import MSACL
    from msacl_amd.utils import dist as D
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    noise = {}

    def fixed(shape, dtype, device):
        key = tuple(shape)
        if key not in noise:
            gen = torch.Generator(device="cuda").manual_seed(len(noise) + 1)
            noise[key] = torch.randn(key, dtype=dtype, device=device, generator=gen)
        return noise[key]

    monkeypatch.setattr(tdn, "_standard_normal", fixed)
    monkeypatch.setattr(D, "world_size", lambda: 2)
    monkeypatch.setattr(D.dist, "all_reduce", lambda t, *a, **k: t.mul_(3.0))
    states = {}
    for mode in ("eager", "segments"):
        alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=(mode != "eager"))
        sd = {k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")}
        alg.networks.load_state_dict(sd)
        for it in range(8):
            alg.model_update(data, it)
        if mode == "segments":
            assert len(alg._graphs) == 2 and all(isinstance(v[0], D.GraphSegments) for v in alg._graphs.values())
        states[mode] = {k: v.detach().clone() for k, v in alg.networks.state_dict().items()}
    for k, v in states["eager"].items():
        assert torch.equal(v, states["segments"][k]), k


@pytest.mark.parametrize("mode", ["eager", "graph", "segments"])
def test_twin_stream_update_equals_serial(monkeypatch, mode):
    """The forked q1 / q2 branches (alg_twin_streams, and the critic || Lyapunov streams) give
    the same parameters bit for bit as the serial order (both streams off), under eager, single
    graph and segmented-graph execution (fixed rsample noise, several even/odd updates)."""
    import torch.distributions.normal as tdn
    from msacl_amd.algorithm.msacl import MSACL
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    noise = {}

    def fixed(shape, dtype, device):
        key = tuple(shape)
        if key not in noise:
            gen = torch.Generator(device="cuda").manual_seed(len(noise) + 1)
            noise[key] = torch.randn(key, dtype=dtype, device=device, generator=gen)
        return noise[key]

    monkeypatch.setattr(tdn, "_standard_normal", fixed)
    states = {}
    for streams in (True, False):
        alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=(mode != "eager"), alg_force_graph_segments=(mode == "segments"),
                    alg_twin_streams=streams, alg_concurrent_streams=streams)
        sd = {k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")}
        alg.networks.load_state_dict(sd)
        for it in range(6):
            alg.model_update(data, it)
        torch.cuda.synchronize()
        states[streams] = {k: v.detach().clone() for k, v in alg.networks.state_dict().items()}
    for k, v in states[False].items():
        assert torch.equal(v, states[True][k]), k


def test_rccl_collectives_in_the_update_graph_one_gpu(monkeypatch):
    """The data-parallel update with REAL RCCL all-reduces on one GPU (a world-size-1 nccl process
    group with the collectives forced, utils/dist.py force_collectives): as graph segments cut at
    the collectives (the default for world > 1) and as ONE captured graph with the all-reduces
    inside it (MSACL_GRAPH_COLLECTIVES=1: RCCL under stream capture). Parameters bit-identical to
    the eager update without collectives (an all-reduce over one rank is the identity)."""
    import socket
    import torch.distributed as dist
    import torch.distributions.normal as tdn
    from msacl_amd.algorithm.msacl import MSACL
    import msacl_amd.utils.dist as D
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    data = {k: torch.as_tensor(g["in_" + k], device="cuda") for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    noise = {}

    def fixed(shape, dtype, device):
        key = tuple(shape)
        if key not in noise:
            gen = torch.Generator(device="cuda").manual_seed(len(noise) + 1)
            noise[key] = torch.randn(key, dtype=dtype, device=device, generator=gen)
        return noise[key]

    monkeypatch.setattr(tdn, "_standard_normal", fixed)

    def run(mode):
        alg = MSACL(**_msacl_kwargs(B, n), alg_use_graph=(mode != "eager"))
        alg.networks.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")})
        for it in range(6):
            alg.model_update(data, it)
        kinds = {type(v[0]).__name__ for v in alg._graphs.values()}
        st = {k: v.detach().clone() for k, v in alg.networks.state_dict().items()}
        alg.close()
        return st, kinds

    ref, _ = run("eager")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        D.force_collectives(True)
        D.set_graph_collectives(False)
        seg, kinds_seg = run("graph")
        D.set_graph_collectives(True)
        assert D.collectives_in_graph() and not D.graph_segments_wanted()
        one, kinds_one = run("graph")
    finally:
        D.force_collectives(False)
        D.set_graph_collectives(False)
        dist.destroy_process_group()
    assert kinds_seg == {"GraphSegments"} and kinds_one == {"CUDAGraph"}, (kinds_seg, kinds_one)
    for k, v in ref.items():
        assert torch.equal(v, seg[k]), ("segments", k)
        assert torch.equal(v, one[k]), ("in-graph", k)
