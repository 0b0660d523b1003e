"""GPU parity of the BENCHMARKED sampler instantiations against the oracle.

The headline runs the fused horizon sampler (csrc/sample_fused.hip, tests/test_gpu_fused_horizon.py
pins it bit for bit to the lockstep kernels) and the lockstep path runs `k_rollout<Env, true>`
(csrc/rollout.hip): in-kernel TanhGauss sampling and clip (RL/utils/act_distribution_cls.py:45-57,
RL/trainer/sampler/base.py:127-143), the env step, rew_plus_cost, in-kernel Philox resets
(gymnasium SyncVectorEnv autoreset) and the deferred n-step window emission (base.py:178-217). The
other parity tests drive the injected-action instantiation `k_rollout<Env, false>`. Here the
sampler itself runs, lockstep by lockstep, eagerly (HipNstepOffSampler.step_traced: the same policy
forward + lockstep launch as one iteration of the sampler's graph-captured horizon) at the configs'
65,536 envs with n = 20, writing its own sampled actions / log-probs and the env step's outputs
(mh_rollout_set_trace). Before each lockstep the env state and the per-env Philox counters are
snapshotted, and the oracle recomputes from the seed alone:

* the action and its log-prob: oracle/rng.py's float64 TanhGauss of (the policy kernel's logits,
  the eps the env draws at its counter) at rtol = atol = 1e-5, every row (no atanh recovery, no
  exclusion of saturated actions);
* next observation (final_observation), raw reward, terminated, truncated at rtol = atol = 1e-5
  (QuadTracking against the float64-polar path, and the as-is path within 1e-5 plus the
  reference's own float32-SVD deviation: see tests/test_gpu_env.py);
* the next state of every continuing env, its steps counter (k + 1, or 0 after a reset), and its
  Philox counter (+1);
* every reset row: the stored state is the oracle's reset draw at that env's counter (bit-exact;
  QuadTracking's rotation block within 2e-7) and the returned observation (and QuadTracking's
  Rd_last) equals oracle.env_reset_from(state);
* the replay store filled by the deferred emitter waves (+ the final flush) equals the windows
  oracle.sampler.NStepWindows assembles from the oracle's per-step records — actions and log-probs
  included — row for row.

1/16 of the envs start 985-999 steps into their episode so truncation happens inside the run.
The fused horizon's sampled actions and log-probs (mh_sample_horizon's act_out / logp_out, its
logits trace) are checked against the oracle the same way for a whole 20-lockstep horizon.
"""
import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
from msacl_amd.create_pkg.create_buffer import create_buffer
from msacl_amd.create_pkg.create_envs import create_envs
from msacl_amd.create_pkg.create_sampler import create_sampler
from msacl_amd.trainer.buffer.device_nstep_replay_buffer import KEYS
from msacl_amd.utils.config import default_msacl_args
from msacl_amd.utils.init_args import init_args
from oracle import envs as OE
from oracle import rng as OR
from oracle import sampler as OS
import msacl_amd._native as N

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-5, atol=1e-5)
E, NSTEP = 65536, 20
# locksteps per env: windows need 20 consecutive steps; QuadTracking's oracle (batched 3x3 SVDs
# twice per substep) is the slow one
STEPS = {"QuadTracking": 27}


def _near_bound(cls, obs, eps=1e-4):
    return np.any((np.abs(obs - cls.obs_low) < eps) | (np.abs(obs - cls.obs_high) < eps), axis=1)


def _reset_box_ok(name, st):
    if name == "VanderPol":
        return np.abs(st).max(initial=0) <= 5.0
    if name == "Pendulum":
        return np.all(st >= OE.Pendulum.obs_low) and np.all(st <= OE.Pendulum.obs_high)
    if name == "QuadTracking":
        n = st.shape[0]
        R = st[:, 6:15].reshape(n, 3, 3).astype(np.float64)
        orth = np.abs(np.matmul(R, np.transpose(R, (0, 2, 1))) - np.eye(3)).max(initial=0) < 1e-6
        return np.abs(st[:, np.r_[0:6, 15:18]]).max(initial=0) <= 0.01 and orth
    return np.abs(st).max(initial=0) <= 0.5


def _quad_obs_of_state(s2, xs, k):
    """The reference's observation map (QuadTracking.py:229-246: desired states at step k + 1,
    cal_eR / cal_eOmega) applied to a given post-step state [x, v, R, Omega]."""
    n = s2.shape[0]
    Q = OE.QuadTracking
    ex, ev, Rd, Od = Q.desired(s2[:, 0:3].copy(), s2[:, 3:6].copy(), k + 1, xs.reshape(n, 3, 3))
    return Q.errors(s2[:, 6:15].reshape(n, 3, 3).copy(), s2[:, 15:18].copy(), ex, ev, Rd, Od)


def _quad_allowance(xs, k, got, o2, st_post):
    """QuadTracking rows whose observation is beyond 1e-5 of the float64-polar oracle's.

    The observation is a function of the post-step state, and e_Omega = Omega - R^T R_d Omega_d
    (obs components 9-11) multiplies last-bit differences of that state (the rotation R leaves
    the polar factorisation rounded to float32) by |Omega_d|: a row measured on the MI355X was
    3.6e-5 / 2.3e-5 off on e_Omega x / z with |Omega| ~ 2 rad/s. Such a row passes when
    (a) the kernel's post-step state is within 1e-5 of the oracle's (asserted for EVERY row by
        the caller, terminal rows included: the kernel exports each env's post-step state before
        the autoreset overwrites it, mh_rollout_set_trace_state), and
    (b) the kernel's observation is within 1e-5 of the reference's observation map applied to
        the kernel's OWN post-step state (_quad_obs_of_state),
    i.e. both halves of the step are within 1e-5 and only their composition amplifies a
    rounding difference. Terminal and continuing rows get the same check; there is no other
    allowance. Returns the rows that needed it (a handful: 1 in 1.77 M env-steps measured).
    """
    far = ~np.isclose(got, o2, **TOL)
    rows = np.nonzero(far.any(axis=1))[0]
    if rows.size:
        mine = _quad_obs_of_state(st_post[rows], xs[rows], k[rows])
        np.testing.assert_allclose(got[rows], mine, **TOL, err_msg=f"rows {rows}: obs of the kernel's own state")
    return rows


def _sampler(name, tmp_path, noise=None):
    # the store holds every window of the run (VanderPol emits 1.34 M in 40 locksteps)
    args = default_msacl_args(env_name=name, env_num=E, n_step=NSTEP, seed=0, env_seed=5, buffer_max_size=2_000_000,
                              buffer_warm_size=0, save_folder=str(tmp_path), noise_params=noise)
    args = init_args(create_envs(**args), **args)
    sampler, buffer = create_sampler(**args), create_buffer(**args)
    sampler.bind_store(buffer)
    return sampler, buffer


@pytest.mark.parametrize("name,noise", [(n, None) for n in OE.ENVS] + [("DuctedFan", {"mean": 0.0, "std": 0.2})],
                         ids=list(OE.ENVS) + ["DuctedFan-gauss-noise"])
def test_sampled_lockstep_kernel_matches_oracle(name, noise, tmp_path):
    cls = OE.ENVS[name]
    quad = name == "QuadTracking"
    sampler, buffer = _sampler(name, tmp_path, noise)
    env, dev = sampler.envs, sampler.device
    D, A = env.obs_dim, env.act_dim
    rng = np.random.default_rng(3)
    k0 = np.zeros(E, np.int32)
    late = rng.choice(E, E // 16, replace=False)
    k0[late] = rng.integers(985, 1000, size=late.size)
    env.set_state(None, None, k0)
    lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
    act, logp = torch.empty(E, A, device=dev), torch.empty(E, device=dev)
    real, rew = torch.empty(E, D, device=dev), torch.empty(E, device=dev)
    term, trunc = torch.empty(E, dtype=torch.uint8, device=dev), torch.empty(E, dtype=torch.uint8, device=dev)
    # the post-step state before the autoreset of the envs that reset (mh_rollout_set_trace_state)
    t_st = torch.empty(env.state_dim, E, device=dev)
    t_xs = torch.empty(max(env.xstate_dim, 1), E, dtype=torch.float64, device=dev)
    windows = OS.NStepWindows(E, NSTEP, D, A)
    expect = {k: [] for k in KEYS}

    st, xs, k = env.get_state()
    st = st.cpu().numpy()
    xs = xs.cpu().numpy() if xs is not None else None
    k = k.cpu().numpy().astype(np.int64)
    assert _reset_box_ok(name, st)
    _, xs_r, obs_o = OE.env_reset_from(name, st)  # the oracle's view of the current observation
    np.testing.assert_allclose(sampler.obs.cpu().numpy(), obs_o, **TOL)
    if quad:
        np.testing.assert_allclose(xs, xs_r, rtol=0, atol=1e-12)
    n_reset = n_trunc = n_lp = n_quad_allow = n_rd_allow = 0
    seed, idx = env.seed, np.arange(E)
    pol = sampler.networks.policy
    ls_lo, ls_hi = float(getattr(pol, "min_log_std", -20.0)), float(getattr(pol, "max_log_std", 1.0))
    for t in range(STEPS.get(name, 40)):
        ctr = env.get_counters().cpu().numpy()
        logits = sampler.step_traced(act, logp, trace=(real, rew, term, trunc), state_trace=(t_st, t_xs))
        a_np, lp_np, lg32 = act.cpu().numpy(), logp.cpu().numpy(), logits.cpu().numpy()
        noise_t = float(sampler._noise[0]) if noise is not None else 0.0
        got_real, got_rew = real.cpu().numpy(), rew.cpu().numpy()
        got_term, got_trunc = term.cpu().numpy().astype(bool), trunc.cpu().numpy().astype(bool)
        st2, xs2, k2 = env.get_state()
        st2, k2 = st2.cpu().numpy(), k2.cpu().numpy().astype(np.int64)
        xs2 = xs2.cpu().numpy() if xs2 is not None else None
        obs_next = sampler.obs.cpu().numpy()
        # the post-step state of every env before its reset: the trace holds it for the envs that
        # reset this lockstep, the env state itself for the others
        rs_k = got_term | got_trunc
        st_post = np.where(rs_k[:, None], t_st.cpu().numpy().T, st2)
        xs_post = np.where(rs_k[:, None], t_xs.cpu().numpy().T, xs2) if quad else None

        # ---- the action and its log-prob: the oracle's TanhGauss of (logits, the env's eps)
        assert np.all((a_np >= cls.act_low) & (a_np <= cls.act_high))
        eps = OR.action_normals(seed, idx, ctr)
        a_o, lp_o = OR.tanh_gauss_sample(lg32, eps, lo, hi, ls_lo, ls_hi, noise=noise_t)
        np.testing.assert_allclose(a_np, a_o, **TOL, err_msg="sampled action")
        np.testing.assert_allclose(lp_np, lp_o, **TOL, err_msg="sampled log-prob")
        n_lp += E
        np.testing.assert_array_equal(env.get_counters().cpu().numpy(), (ctr + 1) & 0xFFFFFFFF)

        # ---- the env step from the snapshot, with the kernel's own actions
        s_o, xs_o, o2, r2, te, tr = OE.env_step(name, st, a_np, xs, k, polar64=quad)
        # ---- the post-step state of EVERY env (terminal rows too, before their reset overwrites it)
        np.testing.assert_allclose(st_post, s_o, **TOL, err_msg="post-step state (pre-reset)")
        if quad:
            # Rd_last = R_d(x, v) of the post-step state (QuadTracking.py:122-149): rows beyond
            # (1e-5, 1e-6) of the oracle's must be R_d of the kernel's OWN post-step x, v (float64
            # arithmetic on the same float32 inputs): the two halves again, as for e_Omega below
            far = np.nonzero(~np.isclose(xs_post, xs_o, rtol=1e-5, atol=1e-6).all(axis=1))[0]
            if far.size:
                _, _, rd_mine, _ = OE.QuadTracking.desired(st_post[far, 0:3].copy(), st_post[far, 3:6].copy(),
                                                           k[far] + 1, xs[far].reshape(-1, 3, 3))
                np.testing.assert_allclose(xs_post[far], rd_mine.reshape(-1, 9), rtol=0, atol=1e-10,
                                           err_msg=f"rows {far}: R_d of the kernel's own state")
            n_rd_allow += far.size
        if quad:  # rows beyond 1e-5 of the float64-polar path: see _quad_allowance
            bad = _quad_allowance(xs, k, got_real, o2, st_post)
            n_quad_allow += bad.size
            o2[bad] = got_real[bad]
        np.testing.assert_allclose(got_real, o2, **TOL)
        np.testing.assert_allclose(got_rew, r2, **TOL)
        if quad:  # the reference as-is (float32 SVD) on a slice: within 1e-5 + its own SVD noise
            sl = slice(0, 4096)
            _, _, o32, _, _, _ = OE.env_step(name, st[sl], a_np[sl], xs[sl], k[sl])
            dev32 = np.abs(o32.astype(np.float64) - o2[sl])
            assert np.all(np.abs(got_real[sl] - o32) <= 1e-5 + 1e-5 * np.abs(o32) + dev32)
        nb = _near_bound(cls, o2)
        np.testing.assert_array_equal(got_term[~nb], te[~nb])
        np.testing.assert_array_equal(got_trunc, tr)
        done = got_term | got_trunc  # the kernel's flags (they differ from te only at the bound)
        n_reset += int(done.sum())
        n_trunc += int(got_trunc.sum())

        # ---- continuing envs: counter, observation (their next state is checked above)
        np.testing.assert_array_equal(k2, np.where(done, 0, k + 1))
        np.testing.assert_allclose(obs_next[~done], o2[~done], **TOL)
        # ---- reset rows: a reset-distribution draw, and obs / Rd_last = env_reset_from(state)
        obs_new = o2.copy()
        if done.any():
            assert _reset_box_ok(name, st2[done])
            want = OR.reset_draw(name, seed, idx[done], ctr[done])
            if quad:
                uni = np.r_[0:6, 15:18]
                np.testing.assert_array_equal(st2[done][:, uni], want[:, uni])
                np.testing.assert_allclose(st2[done][:, 6:15], want[:, 6:15], rtol=0, atol=2e-7)
            else:
                np.testing.assert_array_equal(st2[done], want)
            _, xr, orr = OE.env_reset_from(name, st2[done])
            np.testing.assert_allclose(obs_next[done], orr, **TOL)
            if quad:
                np.testing.assert_allclose(xs2[done], xr, rtol=0, atol=1e-12)
            obs_new[done] = orr

        # ---- the oracle's n-step records (rew_plus_cost.py:18-21 with the reference's scales)
        r_s, c_s = OS.rew_plus_cost(o2, r2.astype(np.float32), 100.0, 100.0)
        rec = windows.push(obs_o, a_o.astype(np.float32), r_s, c_s, o2, done, lp_o.astype(np.float32))
        for key, w in zip(KEYS, rec):
            expect[key].append(w)
        st, xs, k, obs_o = st2, xs2, k2, obs_new

    sampler.flush()
    torch.cuda.synchronize()
    exp = {key: np.concatenate(v) for key, v in expect.items()}
    total = exp["obs"].shape[0]
    assert total > 500 and n_reset > 0 and n_trunc > 0, (total, n_reset, n_trunc)
    assert n_quad_allow <= 1e-5 * E * STEPS.get(name, 40), n_quad_allow  # a handful of 1.77 M env-steps
    assert n_rd_allow <= 1e-5 * E * STEPS.get(name, 40), n_rd_allow
    print(f"{name}: {n_reset} resets, rows checked against their own state: obs {n_quad_allow}, Rd_last {n_rd_allow}")
    assert n_lp > 1000
    assert int(buffer.cursor[2]) == total and total < buffer.max_size
    for key in KEYS:
        np.testing.assert_allclose(buffer.n_step_buf[key][:total].cpu().numpy(), exp[key], **TOL, err_msg=key)
    assert not buffer.n_step_buf["done"][:total, :-1].any()


@pytest.mark.parametrize("name", list(OE.ENVS))
def test_fused_horizon_samples_match_oracle(name, tmp_path):
    """The benchmarked kernel (mh_sample_horizon): every lockstep's sampled actions and log-probs of
    a 20-lockstep horizon at 65,536 envs equal the oracle's TanhGauss of (the logits the kernel
    sampled from, the eps env e draws at counter c0[e] + t) at rtol = atol = 1e-5, and every
    counter advances by the horizon."""
    sampler, buffer = _sampler(name, tmp_path)
    assert sampler.fused_horizon
    env, dev = sampler.envs, sampler.device
    D, A, H = env.obs_dim, env.act_dim, sampler.horizon
    cls = OE.ENVS[name]
    lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
    pol = sampler.networks.policy
    ls_lo, ls_hi = float(getattr(pol, "min_log_std", -20.0)), float(getattr(pol, "max_log_std", 1.0))
    sampler.sample()  # the envs move off their initial draws
    lg = torch.empty(H, E, 2 * A, device=dev)
    ob = torch.empty(H, E, D, device=dev)
    act, logp = torch.empty(H, E, A, device=dev), torch.empty(H, E, device=dev)
    N.check(N.lib().mh_sample_horizon_debug_logits(sampler._h, N.ptr(lg), N.ptr(ob)), "debug logits")
    try:
        c0 = env.get_counters().cpu().numpy()
        with torch.no_grad():
            sampler._horizon(buffer, act_out=act, logp_out=logp)
        torch.cuda.synchronize()
    finally:
        N.check(N.lib().mh_sample_horizon_debug_logits(sampler._h, None, None), "debug logits off")
    sampler.check_errors()
    np.testing.assert_array_equal(env.get_counters().cpu().numpy(), (c0 + H) & 0xFFFFFFFF)
    lg, act, logp = lg.cpu().numpy(), act.cpu().numpy(), logp.cpu().numpy()
    for t in range(H):
        eps = OR.action_normals(env.seed, np.arange(E), (c0 + t) & 0xFFFFFFFF)
        a_o, lp_o = OR.tanh_gauss_sample(lg[t], eps, lo, hi, ls_lo, ls_hi)
        np.testing.assert_allclose(act[t], a_o, **TOL, err_msg=f"lockstep {t} action")
        np.testing.assert_allclose(logp[t], lp_o, **TOL, err_msg=f"lockstep {t} log-prob")
