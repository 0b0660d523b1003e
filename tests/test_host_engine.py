"""BASELINE.json config 1 ("VanderPol, 1 env, MSACL off_serial_trainer on CPU reference sampler
(plumbing, no GPU)"): the engine's CPU build (csrc/host_engine.hip -> libmsacl_host.so) and the
CPU deployment around it (HostVectorEnv, CpuNstepOffSampler, HostNstepReplayBuffer, MSACL on
device="cpu") against the reference's own fixtures and the oracle. No GPU needed."""
import os
import re

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.env.host_vector_env import HostVectorEnv
from msacl_amd.trainer.buffer.host_nstep_replay_buffer import KEYS, HostNstepReplayBuffer, HostWindowBatch
from oracle import envs as OE
from oracle import msacl as OM

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
TOL = dict(rtol=1e-5, atol=1e-5)
NAMES = list(OE.ENVS)


def _reset_pool(name, n, seed=0):
    rng = np.random.default_rng(seed)
    if name == "QuadTracking":
        return OE.QuadTracking.reset_draw(rng, n, gauss=lambda k: rng.standard_normal((k, 3)))
    return OE.ENVS[name].reset_draw(rng, n)


# ------------------------------------------------------------------ the C ABI
def test_host_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "msacl_host.h")).read()
    declared = set(re.findall(r"\b(mhh_\w+)\s*\(", hdr))
    assert len(declared) >= 16
    assert declared == set(N.host_exported_symbols())
    L = N.host_lib()
    for name in declared:
        assert getattr(L, name) is not None
    assert L.mhh_abi_version() == 1


def test_host_errors_are_reported():
    h = torch.zeros(1)
    rc = N.host_lib().mhh_env_create(99, 4, 0, None)
    assert rc != 0
    with pytest.raises(RuntimeError, match="mhh_msacl_ratio0"):
        N.host_check(N.host_lib().mhh_msacl_ratio0(None, None, 0, 0, N.hptr(h)), "mhh_msacl_ratio0")


# ------------------------------------------------------------------ env step vs reference fixtures
@pytest.mark.parametrize("name", NAMES)
def test_host_env_step_matches_reference_fixtures(name):
    g = np.load(os.path.join(G, f"env_{name}.npz"))
    E = g["state"].shape[0]
    env = HostVectorEnv(name, E, seed=3)
    env.reset()
    xstate = g["xstate"] if "xstate" in g else None
    env.set_state(g["state"], xstate, g["steps"])
    rs = _reset_pool(name, E)
    nxt, rew, term, trunc, info = env.step(g["act"], reset_states=rs)
    real = info["final_observation"].numpy()
    np.testing.assert_allclose(real, g["obs"], **TOL)
    np.testing.assert_allclose(rew.numpy(), g["reward"].astype(np.float32), **TOL)
    cls = OE.ENVS[name]
    near = np.any((np.abs(g["obs"] - cls.obs_low) < 1e-4) | (np.abs(g["obs"] - cls.obs_high) < 1e-4), axis=1)
    np.testing.assert_array_equal(term.numpy()[~near], g["terminated"][~near])
    np.testing.assert_array_equal(trunc.numpy(), g["truncated"])
    done = (term | trunc).numpy()
    st, xs, sp = env.get_state()
    np.testing.assert_allclose(st.numpy()[~done], g["state_out"][~done], **TOL)
    np.testing.assert_array_equal(sp.numpy(), np.where(done, 0, g["steps"] + 1))
    if done.any():
        _, _, robs = OE.env_reset_from(name, rs[done])
        np.testing.assert_allclose(nxt.numpy()[done], robs, **TOL)
    if name == "VanderPol":  # no transcendental: bit-exact with the reference
        np.testing.assert_array_equal(real, g["obs"])
    env.close()


def test_host_quad_reset_matches_reference():
    g = np.load(os.path.join(G, "reset_QuadTracking.npz"))
    env = HostVectorEnv("QuadTracking", g["reset_state"].shape[0])
    obs, _ = env.reset(reset_states=g["reset_state"])
    np.testing.assert_allclose(obs.numpy(), g["obs"], **TOL)
    _, xs, sp = env.get_state()
    np.testing.assert_allclose(xs.numpy(), g["rd_last"], rtol=0, atol=1e-12)
    assert int(sp.abs().sum()) == 0


@pytest.mark.parametrize("name", [n for n in NAMES if n != "QuadTracking"])
def test_host_multi_step_vs_oracle(name):
    """20 steps of random in-box actions at 256 envs, state re-injected each step."""
    E = 256
    rng = np.random.default_rng(4)
    cls = OE.ENVS[name]
    env = HostVectorEnv(name, E, seed=5)
    env.reset(reset_states=_reset_pool(name, E, seed=2))
    for t in range(20):
        lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
        act = ((lo + hi) / 2 + (hi - lo) / 4 * rng.uniform(-1, 1, size=(E, lo.size))).astype(np.float32)
        st, xs, sp = env.get_state()
        s_in, k_in = st.numpy(), sp.numpy().astype(np.int64)
        x_in = xs.numpy() if xs is not None else None
        _, _, _, _, info = env.step(act, reset_states=_reset_pool(name, E, seed=100 + t))
        s2, xs2, o2, r2, te2, tr2 = OE.env_step(name, s_in, act, x_in, k_in)
        np.testing.assert_allclose(info["final_observation"].numpy(), o2, **TOL)


def test_host_autoreset_draws_are_deterministic_per_seed():
    a, b = HostVectorEnv("Pendulum", 64, seed=9), HostVectorEnv("Pendulum", 64, seed=9)
    oa, _ = a.reset()
    ob, _ = b.reset()
    np.testing.assert_array_equal(oa.numpy(), ob.numpy())
    c = HostVectorEnv("Pendulum", 64, seed=10)
    oc, _ = c.reset()
    assert not np.array_equal(oa.numpy(), oc.numpy())
    lo, hi = OE.Pendulum.obs_low, OE.Pendulum.obs_high
    assert np.all(oa.numpy() >= lo) and np.all(oa.numpy() <= hi)


# ------------------------------------------------------------------ MSACL target math vs oracle
def _h(a):
    return torch.as_tensor(np.ascontiguousarray(a, np.float32))


@pytest.mark.parametrize("B,n,weighted", [(256, 20, False), (64, 5, True), (7, 70, False)])
def test_host_q_target(B, n, weighted):
    rng = np.random.default_rng(B + n)
    f = lambda *s: rng.standard_normal(s).astype(np.float32)  # noqa: E731
    q1, q2, q1t, q2t, nlp, rew = f(B, n), f(B, n), f(B, n), f(B, n), f(B, n), f(B, n) * 10
    done = (rng.uniform(size=(B, n)) < 0.1).astype(np.float32)
    la = np.float32(0.3)
    w = rng.uniform(0.2, 1.0, B).astype(np.float32) if weighted else None
    ins = [_h(a) for a in (q1, q2, q1t, q2t, nlp, rew, done, [la])]
    wt = _h(w) if weighted else None
    out = [torch.empty(B, n) for _ in range(3)] + [torch.empty(1), torch.empty(B)]
    N.host_check(N.host_lib().mhh_msacl_q_target(*[N.hptr(t) for t in ins], N.hptr(wt), 0.99, B, n,
                                                 *[N.hptr(o) for o in out]), "q")
    bk, loss, d1, d2, td = OM.q_target(q1, q2, q1t, q2t, nlp, rew, done, float(np.exp(la, dtype=np.float32)), 0.99, w)
    np.testing.assert_allclose(out[0].numpy(), bk, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(out[1].numpy(), d1, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out[2].numpy(), d2, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out[3].item(), loss, rtol=1e-5)
    np.testing.assert_allclose(out[4].numpy(), td, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,n,D", [(256, 20, 12), (33, 5, 2)])
def test_host_lyapunov(B, n, D):
    rng = np.random.default_rng(B * n)
    obs = (rng.standard_normal((B, n, D)) * 0.5).astype(np.float32)
    obs2 = (obs + rng.standard_normal((B, n, D)) * 0.1).astype(np.float32)
    V = (rng.uniform(0, 2, (B, n)) * (obs ** 2).sum(-1)).astype(np.float32)
    V2 = (rng.uniform(0, 2, (B, n)) * (obs2 ** 2).sum(-1)).astype(np.float32)
    logp = rng.standard_normal((B, n)).astype(np.float32)
    old = (logp + rng.standard_normal((B, n)) * 0.3).astype(np.float32)
    c, w, s = OM.coefficients(n)
    outs = [torch.empty(B, n), torch.empty(B, n), torch.empty(B), torch.empty(1), torch.empty(B, n), torch.empty(B, n)]
    ins = [_h(a) for a in (logp, old, V, V2, obs, obs2, c, w, s)]
    N.host_check(N.host_lib().mhh_msacl_lyapunov(*[N.hptr(t) for t in ins], 1.0, 2.0, 1.0, 10.0, B, n, D,
                                                 *[N.hptr(o) for o in outs]), "lya")
    ic, esl, ld, loss, dV, dV2 = OM.lyapunov(logp, old, V, V2, obs, obs2, c, w, s, 1.0, 2.0, 1.0, 10.0)
    np.testing.assert_allclose(outs[0].numpy(), ic, rtol=1e-5, atol=1e-6)
    assert np.mean(outs[1].numpy() == esl) > 0.999
    np.testing.assert_allclose(outs[2].numpy(), ld, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(outs[3].item(), loss, rtol=1e-4)
    np.testing.assert_allclose(outs[4].numpy(), dV, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(outs[5].numpy(), dV2, rtol=1e-4, atol=1e-7)


def test_host_stability_advantage_and_ppo_clip():
    B, n = 256, 20
    rng = np.random.default_rng(B)
    V0 = rng.uniform(0, 3, B).astype(np.float32)
    V2 = rng.uniform(0, 3, (B, n)).astype(np.float32)
    ratio = rng.uniform(0.7, 1.3, B).astype(np.float32)
    ratio[:3] = [np.float32(0.9), np.float32(1.1), np.float32(1.0)]
    c, w, s = OM.coefficients(n)
    adv_raw, stats = torch.empty(B), torch.empty(2, dtype=torch.float64)
    L = N.host_lib()
    N.host_check(L.mhh_msacl_stability_adv(*[N.hptr(_h(a)) for a in (V0, V2, w, s)], B, n, N.hptr(adv_raw),
                                           N.hptr(stats)), "adv")
    adv, loss, dr = torch.empty(B), torch.empty(1), torch.empty(B)
    N.host_check(L.mhh_msacl_ppo_clip(N.hptr(_h(ratio)), N.hptr(adv_raw), N.hptr(stats), float(B), 0.1, B, N.hptr(adv),
                                      N.hptr(loss), N.hptr(dr)), "ppo")
    a_raw, a, l, g = OM.stability(V0, V2, ratio, w, s, 0.1)
    np.testing.assert_allclose(adv_raw.numpy(), a_raw, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(adv.numpy(), a, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(loss.item(), l, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dr.numpy(), g, rtol=1e-4, atol=1e-7)


def test_cpu_model_update_matches_reference(monkeypatch):
    """One full MSACL.model_update on device="cpu" (torch CPU MLPs + Adam, mhh_msacl_* target
    math) vs the reference's own run (tests/golden/msacl_update.npz, recorded noise replayed)."""
    import torch.distributions.normal as tdn

    from msacl_amd.algorithm.msacl import MSACL
    from test_gpu_msacl import _compare_params, _msacl_kwargs
    g = np.load(os.path.join(G, "msacl_update.npz"))
    B, n = int(g["cfg_B"]), int(g["cfg_n"])
    alg = MSACL(device="cpu", **_msacl_kwargs(B, n))
    alg.networks.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")})
    it = iter([g[f"eps{i}"] for i in range(4)])
    monkeypatch.setattr(tdn, "_standard_normal",
                        lambda shape, dtype, device: torch.as_tensor(next(it), dtype=dtype, device=device).reshape(shape))
    data = {k: torch.as_tensor(g["in_" + k]) for k in KEYS}
    tb = alg.model_update(data, 0)
    ref_tb = dict(zip([str(k) for k in g["tb_keys"]], g["tb_vals"]))
    for k, v in tb.items():
        if "time" not in k.lower():
            np.testing.assert_allclose(v, ref_tb[k], rtol=2e-4, atol=1e-5, err_msg=k)
    _compare_params(alg, g, "after0/")
    assert alg.model_update(data, 1) is None
    _compare_params(alg, g, "after1/")


# ------------------------------------------------------------------ CPU sampler + buffer
def _sampler_kwargs(name, E, n, **kw):
    from msacl_amd.utils.config import default_msacl_args
    cls = OE.ENVS[name]
    a = default_msacl_args(env_name=name, env_num=E, n_step=n, device="cpu", obs_dim=cls.obs_dim, act_dim=cls.act_dim,
                           action_type="continu", action_high_limit=cls.act_high.astype(np.float32),
                           action_low_limit=cls.act_low.astype(np.float32), sample_batch_size=4,
                           policy_hidden_sizes=[32, 32], value_hidden_sizes=[32, 32], lyapunov_hidden_sizes=[32, 32],
                           lyapunov_output_dim=16)
    a.update(kw)
    return a


def _cpu_trace(path):
    from msacl_amd.trainer.sampler.nstep_off_sampler import NstepOffSampler
    g = np.load(path)
    name = os.path.basename(path)[6:-4].replace("_n20", "")
    E, T, n = g["init_reset"].shape[0], g["actions"].shape[0], int(g["n_step"])
    smp = NstepOffSampler(**_sampler_kwargs(name, E, n))
    assert type(smp).__name__ == "CpuNstepOffSampler"
    obs, _ = smp.envs.reset(reset_states=g["init_reset"])
    smp.envs.set_state(None, None, g["init_steps"])
    smp.obs = obs.numpy()
    anchor = name == "TwoLink" and n == 20  # open-loop unstable arm: see tests/test_gpu_nstep.py
    buf = HostNstepReplayBuffer(obs_dim=smp.envs.obs_dim, act_dim=smp.envs.act_dim,
                                buffer_max_size=int(g["counts"].sum()) + 3, n_step=n)
    for t in range(T):
        w = smp.step_injected(g["actions"][t], g["logp"][t], g["resets"][t])
        assert len(w) == g["counts"][t]
        buf.add_batch(w)
        np.testing.assert_allclose(smp.obs, g["obs_trace"][t + 1], **TOL)
        if anchor:
            smp.envs.set_state(g["obs_trace"][t + 1])
            smp.obs = g["obs_trace"][t + 1].astype(np.float32).copy()
    return g, buf


TRACES = sorted(f for f in os.listdir(G) if f.startswith("nstep_"))


@pytest.mark.parametrize("fname", TRACES)
def test_cpu_sampler_windows_match_reference(fname):
    g, buf = _cpu_trace(os.path.join(G, fname))
    total = int(g["counts"].sum())
    assert buf.size == total
    for k in KEYS:
        np.testing.assert_allclose(buf.n_step_buf[k][:total], g["w_" + k], **TOL, err_msg=k)
    if fname.startswith("nstep_VanderPol"):
        for k in KEYS:
            np.testing.assert_array_equal(buf.n_step_buf[k][:total], g["w_" + k], err_msg=k)
    assert not buf.n_step_buf["done"][:total, :-1].any()


def test_host_buffer_fifo_and_store_paths_agree():
    rng = np.random.default_rng(0)
    W, n, D, A, cap = 50, 4, 3, 2, 17
    arrays = {"obs": rng.standard_normal((W, n, D)), "act": rng.standard_normal((W, n, A)),
              "rew": rng.standard_normal((W, n)), "cost": rng.standard_normal((W, n)),
              "obs2": rng.standard_normal((W, n, D)), "done": np.zeros((W, n)), "logp": rng.standard_normal((W, n))}
    arrays = {k: v.astype(np.float32) for k, v in arrays.items()}
    a = HostNstepReplayBuffer(obs_dim=D, act_dim=A, buffer_max_size=cap, n_step=n)
    b = HostNstepReplayBuffer(obs_dim=D, act_dim=A, buffer_max_size=cap, n_step=n)
    for lo, hi in ((0, 5), (5, 5), (5, 31), (31, 50)):
        a.add_batch(HostWindowBatch({k: v[lo:hi] for k, v in arrays.items()}))
        b.add_batch(list(HostWindowBatch({k: v[lo:hi] for k, v in arrays.items()})))
    assert a.size == b.size == cap and a.ptr == b.ptr == W % cap
    for k in KEYS:
        np.testing.assert_array_equal(a.n_step_buf[k], b.n_step_buf[k])
    np.random.seed(1)
    s = a.sample_batch(8)
    assert s["obs"].shape == (8, n, D) and s["obs"].dtype == torch.float32
    per_row = 4 * n * (2 * D + A + 4)
    assert a.__get_RAM__() == round(per_row * cap / 2 ** 20, 2)


def test_cpu_sampler_policy_windows_are_consistent():
    """sample() with the policy: windows chain (obs2[k] == obs[k+1] inside a window), carry
    done only at the last position, and actions stay in the box."""
    from msacl_amd.trainer.sampler.nstep_off_sampler import NstepOffSampler
    torch.manual_seed(0)
    np.random.seed(0)
    smp = NstepOffSampler(**_sampler_kwargs("Pendulum", 8, 5, sample_batch_size=40,
                                            noise_params={"mean": 0.0, "std": 0.1}))
    data, tb = smp.sample()
    assert smp.get_total_sample_number() == 320 and len(tb) == 1
    a = data.arrays
    assert len(data) > 0 and a["obs"].shape[1:] == (5, OE.Pendulum.obs_dim)
    live = a["done"][:, :-1] == 0
    assert live.all()
    np.testing.assert_array_equal(a["obs2"][:, :-1], a["obs"][:, 1:])
    lo, hi = OE.Pendulum.act_low, OE.Pendulum.act_high
    assert np.all(a["act"] >= lo - 1e-7) and np.all(a["act"] <= hi + 1e-7)
    np.testing.assert_allclose(a["cost"], (a["obs2"] ** 2).sum(-1) * 100.0, rtol=1e-6)


def test_config1_pipeline_trains_on_cpu(tmp_path):
    """BASELINE.json config 1: VanderPol, 1 env, MSACL nstep_off_serial_trainer, device="cpu",
    through the reference's create_* -> trainer.train() sequence."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    args = default_msacl_args(env_name="VanderPol", env_num=1, device="cpu", buffer_warm_size=100,
                              buffer_max_size=5000, max_iteration=4, eval_interval=2, log_save_interval=2,
                              apprfunc_save_interval=4, save_folder=str(tmp_path), seed=0, num_eval_episode=2,
                              replay_batch_size=32, value_hidden_sizes=[64, 64], policy_hidden_sizes=[64, 64],
                              lyapunov_hidden_sizes=[64, 64], lyapunov_output_dim=32)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    assert type(sampler).__name__ == "CpuNstepOffSampler" and type(buffer).__name__ == "HostNstepReplayBuffer"
    assert evaluator.envs.device.type == "cpu" and alg.device.type == "cpu"
    assert buffer.size >= 100
    trainer.train()
    assert trainer.iteration == 5
    for p in alg.networks.parameters():
        assert p.device.type == "cpu" and torch.isfinite(p).all()
    assert os.path.exists(os.path.join(str(tmp_path), "apprfunc", "apprfunc_5.pkl"))


def test_sanitizer_build_of_the_cpu_engine_runs_clean():
    """tests/native/asan_driver: host_engine.hip + a driver of every mhh_* entry under
    AddressSanitizer + UBSan (SURVEY §5 sanitizer host build); exit 0 = no report."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "native", "build", "asan_driver")
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "native")], check=True, capture_output=True)
    syms = subprocess.run(["nm", exe], check=True, capture_output=True, text=True).stdout
    assert "__asan_init" in syms and "__ubsan_handle" in syms
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
