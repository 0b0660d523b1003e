#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by EXECUTING the reference's own code.

Runs only in the build container (the reference is not on the GPU box); the fixtures it writes
are data (inputs + reference outputs) and are committed. Nothing here is imported by the
product package.

  env_<Name>.npz     512 (state, action) -> (obs, reward, terminated, truncated, state') pairs
                     per env, from the reference env.step (RL/env/<Name>.py) run on injected
                     states (tools/refload.py: methods compiled from the reference source;
                     gymnasium absent and not stood in for), incl. near-bound states and
                     steps 998/999 (truncation).
  reset_QuadTracking.npz  reset observation from injected (x, v, R, W) via the reference reset
                     tail (QuadTracking.py:161-202, the RNG draws replaced by the injected state).
  nstep_<Name>.npz   BaseSampler._n_step (RL/trainer/sampler/base.py:118-222, compiled from the
                     reference source) over a vector env of reference env objects with the
                     gymnasium 0.28.1 SyncVectorEnv autoreset restated, the reference
                     StochaPolicy/TanhGaussDistribution sampling actions (torch CPU RNG, seeded);
                     records actions, log-probs, injected resets and every emitted window.
  msacl_update.npz   two MSACL.model_update calls (RL/algorithm/msacl.py:174-224) on a fixed
                     batch with fixed weights; the Normal.rsample noise is recorded so the
                     device implementation can replay it. `.cuda()` is made a no-op in this
                     process only (no GPU in the build container).
Usage: python tools/gen_golden.py
"""
from __future__ import annotations

import ast
import os
import sys
import types
from collections import deque

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import envs as OE  # noqa: E402
from tools.refload import REF, RefModule, load_env  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
F32 = np.float32


# ---------------------------------------------------------------------- env step pairs
def _rollout_states(name, n_keep, rng, horizon=60):
    """Realistic input states: oracle rollouts from reset draws with random in-box actions."""
    cls = OE.ENVS[name]
    E = max(n_keep, 64)
    if name == "QuadTracking":
        rs = cls.reset_draw(rng, E, gauss=lambda k: rng.standard_normal((k, 3)))
    else:
        rs = cls.reset_draw(rng, E)
    st, xs, _ = OE.env_reset_from(name, rs)
    steps = np.zeros(E, np.int64)
    pool = []
    for t in range(horizon):
        act = _actions(name, rng, E, gentle=True)
        s2, xs2, obs, rew, te, tr = OE.env_step(name, st, act, xs, steps)
        done = te | tr
        steps = steps + 1
        st, xs = s2, xs2
        if done.any():
            idx = np.nonzero(done)[0]
            if name == "QuadTracking":
                r2 = cls.reset_draw(rng, idx.size, gauss=lambda k: rng.standard_normal((k, 3)))
            else:
                r2 = cls.reset_draw(rng, idx.size)
            a, b, _ = OE.env_reset_from(name, r2)
            st[idx] = a
            if xs is not None:
                xs[idx] = b
            steps[idx] = 0
        pool.append((st.copy(), None if xs is None else xs.copy(), steps.copy()))
    S = np.concatenate([p[0] for p in pool])
    X = None if pool[0][1] is None else np.concatenate([p[1] for p in pool])
    K = np.concatenate([p[2] for p in pool])
    pick = rng.choice(S.shape[0], n_keep, replace=False)
    return S[pick], (None if X is None else X[pick]), K[pick]


def _actions(name, rng, n, gentle=False):
    cls = OE.ENVS[name]
    lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
    if name == "QuadTracking" and gentle:
        mg = 4.34 * 9.8
        a = np.stack([rng.normal(mg, 3.0, n), rng.normal(0, 0.3, n), rng.normal(0, 0.3, n), rng.normal(0, 0.3, n)], 1)
        return np.clip(a, lo, hi).astype(F32)
    if gentle:
        return rng.uniform(lo * 0.3, hi * 0.3, size=(n, lo.size)).astype(F32)
    return rng.uniform(lo, hi, size=(n, lo.size)).astype(F32)


def gen_env_pairs(name, N=512, seed=0):
    rng = np.random.default_rng(1000 + seed + OE.ENV_IDS[name])
    mod = load_env(name)
    env = mod.make()
    cls = OE.ENVS[name]
    S, X, K = _rollout_states(name, N, rng)
    A = np.concatenate([_actions(name, rng, N // 2, gentle=True), _actions(name, rng, N - N // 2)])
    # edge cases: truncation boundary and near-bound states
    K[0:8] = 999
    K[8:16] = 998
    if name != "QuadTracking":
        lo, hi = cls.obs_low.astype(np.float64), cls.obs_high.astype(np.float64)
        for j in range(16, 48):
            d = j % cls.obs_dim
            S[j, d] = F32((hi[d] if j % 2 else lo[d]) * (1.0 - 1e-4 * (j % 5)))
    else:
        S[16:24, 0:3] += F32(9.5)  # position error near the +-10 bound
    obs_out = np.zeros((N, cls.obs_dim), F32)
    state_out = np.zeros_like(S)
    xstate_out = None if X is None else np.zeros_like(X)
    rew = np.zeros(N, np.float64)
    term = np.zeros(N, bool)
    trunc = np.zeros(N, bool)
    T = OE.QuadTracking.T
    for i in range(N):
        k = int(K[i])
        if name == "QuadTracking":
            env.x = S[i, 0:3].copy()
            env.v = S[i, 3:6].copy()
            env.R = S[i, 6:15].reshape(3, 3).copy()
            env.Omega = S[i, 15:18].copy()
            env.Rd_last = X[i].reshape(3, 3).astype(np.float64).copy()
            env.Omega_d_last = np.zeros(3, F32)
            env.current_step = k
            env.current_time = float(T[k])
            env.t_last = np.array([T[k], T[k - 1] if k > 0 else 0.0])
        else:
            env.obs = S[i].copy()
            env.current_step = k
        o, r, te, tr, _ = env.step(A[i].copy())
        obs_out[i] = o
        rew[i] = r
        term[i] = bool(te)
        trunc[i] = bool(tr)
        if name == "QuadTracking":
            state_out[i] = np.concatenate([env.x, env.v, env.R.reshape(9), env.Omega])
            xstate_out[i] = env.Rd_last.reshape(9)
        else:
            state_out[i] = env.obs
    d = dict(state=S, steps=K.astype(np.int32), act=A, obs=obs_out, reward=rew, terminated=term,
             truncated=trunc, state_out=state_out)
    if X is not None:
        d["xstate"] = X.astype(np.float64)
        d["xstate_out"] = xstate_out
    np.savez_compressed(os.path.join(OUT, f"env_{name}.npz"), **d)
    print(f"env_{name}: {N} pairs, term={term.sum()} trunc={trunc.sum()}")


# ---------------------------------------------------------------------- reset helpers
_RESET_SKIP = ("seed", "np_random", "super()", "random_rot_vec")


def ref_reset(mod, env, name, rs):
    """Reference reset() with its RNG draws replaced by the injected state rs."""
    if name == "QuadTracking":
        env.x = rs[0:3].copy()
        env.v = rs[3:6].copy()
        env.R = rs[6:15].reshape(3, 3).copy()
        env.Omega = rs[15:18].copy()
    else:
        env.obs = rs.astype(F32).copy()
    out = mod.run_statements("reset", env, lambda s: any(t in s for t in _RESET_SKIP))
    return np.asarray(out[0], F32).copy()


def gen_quad_reset(N=256, seed=7):
    rng = np.random.default_rng(seed)
    mod = load_env("QuadTracking")
    env = mod.make()
    rs = OE.QuadTracking.reset_draw(rng, N, gauss=lambda k: rng.standard_normal((k, 3)))
    rs[: N // 4, 0:6] *= 300.0  # larger position/velocity offsets as well
    obs, rdl = [], []
    for i in range(N):
        obs.append(ref_reset(mod, env, "QuadTracking", rs[i]))
        rdl.append(np.asarray(env.Rd_last, np.float64).reshape(9).copy())
    np.savez_compressed(os.path.join(OUT, "reset_QuadTracking.npz"), reset_state=rs, obs=np.stack(obs),
                        rd_last=np.stack(rdl))
    print(f"reset_QuadTracking: {N}")


# ---------------------------------------------------------------------- QuadTracking: polar-factor precision
def _normalize_orient_f64(mat):
    """NormalizeOrientMatrix (QuadTracking.py:308-315) with the SVD in float64 (dgesdd on the
    float32 input) instead of float32 sgesdd; same det < 0 flip, same final float32 cast. Used
    ONLY here, to measure how much of the reference's own output is float32-SVD rounding."""
    U, s, Vh = np.linalg.svd(np.asarray(mat, np.float64))
    R = U @ Vh
    if np.linalg.det(R) < 0:
        U[:, -1] *= -1
        R = U @ Vh
    return R.astype(np.float32)


def _quad_fields(env):
    return {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in vars(env).items() if not callable(v)}


def _quad_step_both(mod, env, twin, act):
    """Step `env` with the reference as-is and `twin` (a copy of env's state) with the float64
    polar factor; returns both (obs, reward, terminated, truncated, state')."""
    for k, v in _quad_fields(env).items():
        setattr(twin, k, v)
    out32 = env.step(act.copy())
    st32 = np.concatenate([env.x, env.v, env.R.reshape(9), env.Omega]).astype(F32)
    orig = mod.ns["NormalizeOrientMatrix"]
    mod.ns["NormalizeOrientMatrix"] = _normalize_orient_f64
    try:
        out64 = twin.step(act.copy())
    finally:
        mod.ns["NormalizeOrientMatrix"] = orig
    st64 = np.concatenate([twin.x, twin.v, twin.R.reshape(9), twin.Omega]).astype(F32)
    return out32, st32, out64, st64


def gen_quad_polar64(E=256, T=20, seed=11):
    """quad_polar64.npz — the reference's self-noise from its float32 SVD:
      pairs/*   the 512 env_QuadTracking.npz inputs stepped with the float64 polar factor;
      traj/*    E envs x T lockstep steps of the reference under random in-box torques (the
                action distribution of tests/test_gpu_env.py::test_multi_step_rollout_vs_oracle:
                box centre +- 20 % of the half range), autoreset from drawn reset states; per step
                the input state and BOTH outputs (reference as-is; float64 polar factor)."""
    mod = load_env("QuadTracking")
    cls = OE.QuadTracking
    g = np.load(os.path.join(OUT, "env_QuadTracking.npz"))
    env, twin = mod.make(), mod.make()
    Tt = cls.T
    p_obs, p_rew, p_state = [], [], []
    for i in range(g["state"].shape[0]):
        k = int(g["steps"][i])
        S, X = g["state"][i], g["xstate"][i]
        env.x, env.v, env.R, env.Omega = S[0:3].copy(), S[3:6].copy(), S[6:15].reshape(3, 3).copy(), S[15:18].copy()
        env.Rd_last = X.reshape(3, 3).astype(np.float64).copy()
        env.Omega_d_last = np.zeros(3, F32)
        env.current_step = k
        env.current_time = float(Tt[k])
        env.t_last = np.array([Tt[k], Tt[k - 1] if k > 0 else 0.0])
        out32, st32, out64, st64 = _quad_step_both(mod, env, twin, g["act"][i])
        assert np.array_equal(np.asarray(out32[0], F32), g["obs"][i])  # the as-is run IS the fixture
        p_obs.append(np.asarray(out64[0], F32))
        p_rew.append(float(out64[1]))
        p_state.append(st64)
    rng = np.random.default_rng(seed)
    envs = [mod.make() for _ in range(E)]
    twins = [mod.make() for _ in range(E)]
    rs0 = cls.reset_draw(rng, E, gauss=lambda m: rng.standard_normal((m, 3)))
    for i, e in enumerate(envs):
        ref_reset(mod, e, "QuadTracking", rs0[i])
    lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
    rec = {k: [] for k in ("state", "xstate", "steps", "act", "obs32", "obs64", "rew32", "rew64", "term32", "term64",
                           "state32", "state64", "reset")}
    for t in range(T):
        act = ((lo + hi) / 2 + (hi - lo) / 2 * 0.2 * rng.uniform(-1, 1, size=(E, lo.size))).astype(F32)
        pool = cls.reset_draw(rng, E, gauss=lambda m: rng.standard_normal((m, 3)))
        row = {k: [] for k in rec}
        for i, e in enumerate(envs):
            row["state"].append(np.concatenate([e.x, e.v, e.R.reshape(9), e.Omega]).astype(F32))
            row["xstate"].append(np.asarray(e.Rd_last, np.float64).reshape(9).copy())
            row["steps"].append(int(e.current_step))
            row["act"].append(act[i])
            out32, st32, out64, st64 = _quad_step_both(mod, e, twins[i], act[i])
            row["obs32"].append(np.asarray(out32[0], F32))
            row["obs64"].append(np.asarray(out64[0], F32))
            row["rew32"].append(float(out32[1]))
            row["rew64"].append(float(out64[1]))
            row["term32"].append(bool(out32[2]))
            row["term64"].append(bool(out64[2]))
            row["state32"].append(st32)
            row["state64"].append(st64)
            row["reset"].append(pool[i])
            if out32[2] or out32[3]:
                ref_reset(mod, e, "QuadTracking", pool[i])
        for k in rec:
            rec[k].append(np.asarray(row[k]))
    d = {"pairs/obs64": np.stack(p_obs), "pairs/reward64": np.array(p_rew), "pairs/state64": np.stack(p_state)}
    for k, v in rec.items():
        d["traj/" + k] = np.stack(v)
    noise = np.abs(d["traj/obs32"].astype(np.float64) - d["traj/obs64"])
    np.savez_compressed(os.path.join(OUT, "quad_polar64.npz"), **d)
    print("quad_polar64: max |obs32 - obs64| per component over the trajectories:",
          np.array2string(noise.reshape(-1, 12).max(0), precision=2),
          "pairs:", np.array2string(np.abs(d["pairs/obs64"] - g["obs"]).max(0), precision=2),
          "terminations:", int(d["traj/term32"].sum()))


# ---------------------------------------------------------------------- n-step sampler traces
class RefVectorEnv:
    """gymnasium 0.28.1 SyncVectorEnv.step autoreset (restated) over reference env objects."""

    def __init__(self, mod, name, E, init_resets, init_steps, reset_pool):
        self.mod, self.name, self.E = mod, name, E
        self.envs = [mod.make() for _ in range(E)]
        cls = OE.ENVS[name]
        self.action_space = types.SimpleNamespace(low=np.tile(cls.act_low, (E, 1)), high=np.tile(cls.act_high, (E, 1)))
        self.pool = reset_pool
        self.pool_i = 0
        self.obs0 = np.stack([ref_reset(mod, e, name, init_resets[i]) for i, e in enumerate(self.envs)])
        for i, e in enumerate(self.envs):
            e.current_step = int(init_steps[i])
        self.log_actions, self.log_resets = [], []

    def step(self, actions):
        self.log_actions.append(np.asarray(actions, F32).copy())
        rs_used = np.zeros((self.E, self.pool.shape[1]), F32)
        obs, finals = [], np.empty(self.E, dtype=object)
        rewards = np.zeros(self.E, np.float64)
        terms = np.zeros(self.E, bool)
        truncs = np.zeros(self.E, bool)
        for i, env in enumerate(self.envs):
            o, r, te, tr, info = env.step(actions[i])
            rewards[i], terms[i], truncs[i] = r, te, tr
            o = np.asarray(o, F32).copy()
            if te or tr:
                finals[i] = o
                rs = self.pool[self.pool_i]
                self.pool_i += 1
                rs_used[i] = rs
                o = ref_reset(self.mod, env, self.name, rs)
            obs.append(o)
        self.log_resets.append(rs_used)
        return np.stack(obs).astype(F32), rewards, terms, truncs, {"final_observation": finals}


def load_n_step():
    """Compile BaseSampler._n_step and nStepExperience from RL/trainer/sampler/base.py."""
    path = f"{REF}/RL/trainer/sampler/base.py"
    tree = ast.parse(open(path).read())
    if REF not in sys.path:
        sys.path.insert(0, REF)
    ns = {"__name__": "ref_base"}
    fn = None
    for node in tree.body:
        if isinstance(node, ast.ImportFrom) and node.module == "RL.create_pkg.create_envs":
            continue  # imports gymnasium (absent)
        if isinstance(node, ast.ClassDef) and node.name == "BaseSampler":
            for item in node.body:
                if isinstance(item, ast.FunctionDef) and item.name == "_n_step":
                    fn = item
            continue
        exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
    return ns["_n_step"]


def gen_nstep_trace(name, E=24, T=40, n_step=5, seed=3, tag="", log_std=-1.5, gentle_policy=("QuadTracking",),
                    pd_gain=None):
    import torch
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from RL.apprfunc.mlp import StochaPolicy
    from RL.utils.act_distribution_cls import TanhGaussDistribution

    rng = np.random.default_rng(seed + 17 * OE.ENV_IDS[name])
    torch.manual_seed(seed)
    mod = load_env(name)
    cls = OE.ENVS[name]

    def draw(k):
        if name == "QuadTracking":
            return cls.reset_draw(rng, k, gauss=lambda m: rng.standard_normal((m, 3)))
        return cls.reset_draw(rng, k)

    init_resets = draw(E)
    init_steps = np.zeros(E, np.int64)
    if name != "QuadTracking":
        init_steps[: E // 4] = 1000 - 7  # exercise truncation (and deque clears) inside the trace
    pool = draw(E * T)
    venv = RefVectorEnv(mod, name, E, init_resets, init_steps, pool)
    policy = StochaPolicy(obs_dim=cls.obs_dim, act_dim=cls.act_dim, hidden_sizes=[64, 64], hidden_activation="relu",
                          output_activation="linear", min_log_std=-20, max_log_std=1,
                          act_high_lim=cls.act_high.copy(), act_low_lim=cls.act_low.copy(),
                          action_distribution_cls=TanhGaussDistribution)
    if pd_gain is not None:
        # the reference StochaPolicy with weights set to a linear state feedback, so TwoLink
        # episodes outlive n = 20 (its default-init policy drops the arm within a few steps):
        # layer 1 = [x, -x] (ReLU keeps both halves), layer 2 passes them on, the mean row of
        # joint j = -(kp q_j + kd qdot_j) / a_high (tanh squashing ~ identity at small torques)
        D, A = cls.obs_dim, cls.act_dim
        kp, kd = pd_gain
        with torch.no_grad():
            l1, l2, l3 = policy.policy[0], policy.policy[2], policy.policy[-2]
            for l in (l1, l2, l3):
                l.weight.zero_()
                l.bias.zero_()
            l1.weight[:D, :] = torch.eye(D)
            l1.weight[D:2 * D, :] = -torch.eye(D)
            l2.weight[:2 * D, :2 * D] = torch.eye(2 * D)
            for j in range(A):
                for col, k in ((j, kp), (A + j, kd)):
                    l3.weight[j, col] = -k / float(cls.act_high[j])
                    l3.weight[j, D + col] = k / float(cls.act_high[j])
            l3.bias[A:] = log_std
    if name in gentle_policy:  # keep episodes alive past n: box-centre mean, small std
        with torch.no_grad():
            last = policy.policy[-2]
            last.weight.mul_(0.01)
            last.bias.zero_()
            last.bias[cls.act_dim:] = log_std
    logps = []

    class Net:
        def __init__(self):
            self.policy = policy

        def create_action_distributions(self, logits):
            dist = policy.get_act_dist_cls(logits)
            orig = dist.sample

            def sample():
                a, lp = orig()
                logps.append(lp.detach().numpy().astype(F32).copy())
                return a, lp
            dist.sample = sample
            return dist

    smp = types.SimpleNamespace(env_id=name, num_envs=E, envs=venv, networks=Net(), noise_params=None,
                                action_type="continu", reward_scale=100.0, cost_scale=100.0, target_value=0.0,
                                n_step=n_step, n_step_buffers=[deque(maxlen=n_step) for _ in range(E)],
                                obs=venv.obs0.astype(F32).copy())
    _n_step = types.MethodType(load_n_step(), smp)
    counts, windows = [], {k: [] for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    obs_trace = [smp.obs.copy()]
    with torch.no_grad():
        for t in range(T):
            exps = _n_step()
            counts.append(len(exps))
            for ex in exps:
                for k, v in zip(windows.keys(), ex):
                    windows[k].append(np.asarray(v, F32))
            obs_trace.append(np.asarray(smp.obs, F32).copy())
    d = dict(init_reset=init_resets, init_steps=init_steps.astype(np.int32), actions=np.stack(venv.log_actions),
             logp=np.stack(logps), resets=np.stack(venv.log_resets), counts=np.array(counts, np.int64),
             obs_trace=np.stack(obs_trace), n_step=np.int64(n_step))
    for k, v in windows.items():
        d["w_" + k] = np.stack(v) if v else np.zeros((0,), F32)
    fn = f"nstep_{name}{tag}.npz"
    np.savez_compressed(os.path.join(OUT, fn), **d)
    print(f"{fn}: E={E} T={T} n={n_step} windows={sum(counts)} resets={int((np.abs(d['resets']).sum(-1) > 0).sum())}")


# ---------------------------------------------------------------------- 1-step / on-policy traces
def load_ref_methods(relpath, cls_name, names, skip_modules=(), extra_ns=None):
    """Compile methods `names` of class `cls_name` from a reference source file (module-level
    statements executed, imports of `skip_modules` skipped)."""
    path = f"{REF}/{relpath}"
    tree = ast.parse(open(path).read())
    if REF not in sys.path:
        sys.path.insert(0, REF)
    ns = {"__name__": "ref_" + cls_name}
    ns.update(extra_ns or {})
    found = {}
    for node in tree.body:
        if isinstance(node, ast.ImportFrom) and node.module in skip_modules:
            continue
        if isinstance(node, ast.ClassDef) and node.name == cls_name:
            for item in node.body:
                if isinstance(item, ast.FunctionDef) and item.name in names:
                    found[item.name] = item
            continue
        exec(compile(ast.Module(body=[node], type_ignores=[]), path, "exec"), ns)
    out = {}
    for nm in names:
        exec(compile(ast.Module(body=[found[nm]], type_ignores=[]), path, "exec"), ns)
        out[nm] = ns.pop(nm)
    return out, ns


def _ref_policy_and_recorder(name, hidden=64):
    import torch
    from RL.apprfunc.mlp import StochaPolicy
    from RL.utils.act_distribution_cls import TanhGaussDistribution
    cls = OE.ENVS[name]
    policy = StochaPolicy(obs_dim=cls.obs_dim, act_dim=cls.act_dim, hidden_sizes=[hidden, hidden],
                          hidden_activation="relu", output_activation="linear", min_log_std=-20, max_log_std=1,
                          act_high_lim=cls.act_high.copy(), act_low_lim=cls.act_low.copy(),
                          action_distribution_cls=TanhGaussDistribution)
    if name == "QuadTracking":
        with torch.no_grad():
            last = policy.policy[-2]
            last.weight.mul_(0.01)
            last.bias.zero_()
            last.bias[cls.act_dim:] = log_std
    logps = []

    def make_dist(logits):
        dist = policy.get_act_dist_cls(logits)
        orig = dist.sample

        def sample():
            a, lp = orig()
            logps.append(lp.detach().numpy().astype(F32).copy())
            return a, lp
        dist.sample = sample
        return dist
    return policy, make_dist, logps


def _trace_env(name, E, T, seed, trunc_frac=4):
    rng = np.random.default_rng(seed + 17 * OE.ENV_IDS[name])
    mod = load_env(name)
    cls = OE.ENVS[name]

    def draw(k):
        if name == "QuadTracking":
            return cls.reset_draw(rng, k, gauss=lambda m: rng.standard_normal((m, 3)))
        return cls.reset_draw(rng, k)
    init_resets = draw(E)
    init_steps = np.zeros(E, np.int64)
    if name != "QuadTracking":
        init_steps[: E // trunc_frac] = 1000 - 7
    venv = RefVectorEnv(mod, name, E, init_resets, init_steps, draw(E * T))
    return venv, init_resets, init_steps


def gen_step_trace(name, E=24, T=30, seed=4):
    """BaseSampler._step (base.py:225-298), the OffSampler's per-step path, with recorded
    actions/resets; every step's Experience list is stored as [T][E] arrays."""
    import torch
    torch.manual_seed(seed)
    base, _ = load_ref_methods("RL/trainer/sampler/base.py", "BaseSampler", ["_step"],
                               skip_modules=("RL.create_pkg.create_envs",))
    venv, init_resets, init_steps = _trace_env(name, E, T, seed)
    policy, make_dist, logps = _ref_policy_and_recorder(name)
    net = types.SimpleNamespace(policy=policy, create_action_distributions=make_dist)
    smp = types.SimpleNamespace(env_id=name, num_envs=E, envs=venv, networks=net, noise_params=None,
                                action_type="continu", reward_scale=100.0, cost_scale=100.0, target_value=0.0,
                                obs=venv.obs0.astype(F32).copy())
    _step = types.MethodType(base["_step"], smp)
    keys = ("obs", "act", "rew", "cost", "obs2", "done", "logp")
    rec = {k: [] for k in keys}
    with torch.no_grad():
        for t in range(T):
            exps = _step()
            assert len(exps) == E
            for k, j in zip(keys, range(7)):
                rec[k].append(np.stack([np.asarray(ex[j], F32) for ex in exps]))
    d = dict(init_reset=init_resets, init_steps=init_steps.astype(np.int32), actions=np.stack(venv.log_actions),
             logp=np.stack(logps), resets=np.stack(venv.log_resets))
    for k in keys:
        d["x_" + k] = np.stack(rec[k])
    np.savez_compressed(os.path.join(OUT, f"step_{name}.npz"), **d)
    print(f"step_{name}: E={E} T={T} dones={int(d['x_done'].sum())}")


def gen_onpolicy_trace(name, E=16, H=40, seed=6):
    """OnSampler._sample (on_sampler.py:44-79) incl. _process_experiences/_finish_trajs (GAE),
    compiled from the reference source, over reference envs with a reference StateValue net."""
    import torch
    from RL.apprfunc.mlp import StateValue
    torch.manual_seed(seed)
    base, bns = load_ref_methods("RL/trainer/sampler/base.py", "BaseSampler", ["_step"],
                                 skip_modules=("RL.create_pkg.create_envs",))
    on, _ = load_ref_methods("RL/trainer/sampler/on_sampler.py", "OnSampler",
                             ["_sample", "_process_experiences", "_finish_trajs"],
                             skip_modules=("RL.trainer.sampler.base",), extra_ns={"Experience": bns["Experience"]})
    cls = OE.ENVS[name]
    venv, init_resets, init_steps = _trace_env(name, E, H, seed, trunc_frac=3)
    policy, make_dist, logps = _ref_policy_and_recorder(name)
    value = StateValue(obs_dim=cls.obs_dim, hidden_sizes=[64, 64], hidden_activation="relu",
                       output_activation="linear")
    vcalls = []

    def value_fn(x):
        out = value(x)
        vcalls.append(out.detach().numpy().astype(F32).copy())
        return out
    net = types.SimpleNamespace(policy=policy, value=value_fn, create_action_distributions=make_dist)
    D, A = cls.obs_dim, cls.act_dim
    z = lambda *s, dt=F32: np.zeros(s, dtype=dt)  # noqa: E731
    smp = types.SimpleNamespace(env_id=name, num_envs=E, envs=venv, networks=net, noise_params=None,
                                action_type="continu", reward_scale=100.0, cost_scale=100.0, target_value=0.0,
                                obs=venv.obs0.astype(F32).copy(), horizon=H, gamma=0.99, gae_lambda=0.95,
                                obs_dim=(D,), act_dim=(A,), mb_obs=z(E, H, D), mb_obs2=z(E, H, D), mb_act=z(E, H, A),
                                mb_rew=z(E, H), mb_cost=z(E, H), mb_logp=z(E, H), mb_done=z(E, H, dt=np.bool_),
                                mb_val=z(E, H), mb_adv=z(E, H), mb_ret=z(E, H))
    for nm, fn in list(base.items()) + list(on.items()):
        setattr(smp, nm, types.MethodType(fn, smp))
    with torch.no_grad():
        out = smp._sample()
    out = {k: v.numpy() for k, v in out.items()}
    # bootstrap values V(real_next_obs) of the single-row calls, in call order (t-major, env order)
    done = out["done"].reshape(E, H)
    v2 = np.full((E, H), np.nan, F32)
    it = iter(c for c in vcalls if c.shape == (1,))
    for t in range(H):
        for i in range(E):
            if done[i, t] or t == H - 1:
                v2[i, t] = next(it)[0]
    d = dict(init_reset=init_resets, init_steps=init_steps.astype(np.int32), actions=np.stack(venv.log_actions),
             logp_sampled=np.stack(logps), resets=np.stack(venv.log_resets), val2=v2, H=np.int64(H),
             gamma=np.float64(0.99), gae_lambda=np.float64(0.95))
    for k, v in out.items():
        d["mb_" + k] = v
    for k, v in value.state_dict().items():
        d["value/" + k] = v.numpy().copy()
    np.savez_compressed(os.path.join(OUT, f"onpolicy_{name}.npz"), **d)
    print(f"onpolicy_{name}: E={E} H={H} dones={int(done.sum())}")


def gen_evaluator(name, E=8, seed=9):
    """Evaluator.run_parallel_episodes and run_an_episode (RL/trainer/evaluator.py:59-204),
    compiled from the reference source, with a reference StochaPolicy (mode() actions) and
    injected initial states (resets after an episode's end do not enter the metric)."""
    import torch
    torch.manual_seed(seed)
    ev, _ = load_ref_methods("RL/trainer/evaluator.py", "Evaluator", ["run_parallel_episodes", "run_an_episode",
                                                                      "run_n_episodes"],
                             skip_modules=("RL.create_pkg.create_envs",))
    cls = OE.ENVS[name]
    rng = np.random.default_rng(seed)

    def draw(k):
        if name == "QuadTracking":
            return cls.reset_draw(rng, k, gauss=lambda m: rng.standard_normal((m, 3)))
        return cls.reset_draw(rng, k)
    init = draw(E)
    seq_init = draw(3)
    policy, make_dist, _ = _ref_policy_and_recorder(name)
    net = types.SimpleNamespace(policy=policy, create_action_distributions=lambda lg: policy.get_act_dist_cls(lg))
    mod = load_env(name)

    class EvalEnvs(RefVectorEnv):
        def __init__(self, inits):
            self.inits = list(inits)
            super().__init__(mod, name, len(self.inits[0]), self.inits[0], np.zeros(len(self.inits[0]), np.int64),
                             draw(4096))
            self.k = 0

        def reset(self, seed=None):
            rs = self.inits[self.k]
            self.k += 1
            for i, e in enumerate(self.envs):
                e.current_step = 0
            return np.stack([ref_reset(self.mod, e, self.name, rs[i]) for i, e in enumerate(self.envs)]), {}

    def make_self(envs, n):
        smp = types.SimpleNamespace(env_id=name, envs=envs, networks=net, target_value=0.0, cost_scale=100.0,
                                    reward_scale=100.0, num_eval_episode=n, render=False)
        for nm, fn in ev.items():
            setattr(smp, nm, types.MethodType(fn, smp))
        return smp
    with torch.no_grad():
        par = make_self(EvalEnvs([init]), E).run_parallel_episodes()
        seq = make_self(EvalEnvs([seq_init[i:i + 1] for i in range(3)]), 1).run_n_episodes(3, 0)
        # per-episode lengths of the parallel run, for the test's diagnostics
    np.savez_compressed(os.path.join(OUT, f"eval_{name}.npz"), init=init, seq_init=seq_init,
                        parallel=np.array(par, np.float64), sequential=np.array(seq, np.float64),
                        **{"policy/" + k: v.numpy().copy() for k, v in policy.state_dict().items()})
    print(f"eval_{name}: parallel={np.round(par, 4)} sequential={np.round(seq, 4)}")


# ---------------------------------------------------------------------- MSACL update
def gen_msacl(B=64, n=20, seed=11):
    import torch
    import torch.distributions.normal as tdn

    torch.Tensor.cuda = lambda self, *a, **k: self   # build container has no GPU (this process only)
    torch.nn.Module.cuda = lambda self, *a, **k: self
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from RL.algorithm.msacl import MSACL

    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    cls = OE.QuadTracking
    D, A = cls.obs_dim, cls.act_dim
    kw = dict(env_name="QuadTracking", obs_dim=D, act_dim=A, action_type="continu",
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
              clip_coef=0.1, replay_batch_size=B, max_iteration=1000)
    alg = MSACL(**kw)
    init_sd = {k: v.detach().numpy().copy() for k, v in alg.networks.state_dict().items()}
    # a synthetic but well-formed batch: old log-probs from the current policy plus noise
    obs = (rng.standard_normal((B, n, D)) * 0.3).astype(F32)
    obs2 = (obs + rng.standard_normal((B, n, D)).astype(F32) * 0.05).astype(F32)
    lo, hi = cls.act_low, cls.act_high
    act = (lo + (hi - lo) * rng.uniform(0.05, 0.95, size=(B, n, A))).astype(F32)
    with torch.no_grad():
        dist = alg.networks.create_action_distributions(alg.networks.policy(torch.from_numpy(obs)))
        lp = dist.log_prob(torch.from_numpy(act)).numpy()
    logp = (lp + rng.normal(0, 0.5, size=lp.shape)).astype(F32)
    rew = (rng.standard_normal((B, n)) * 10).astype(F32)
    cost = (rng.uniform(0, 5, size=(B, n))).astype(F32)
    done = np.zeros((B, n), F32)
    done[rng.choice(B, B // 8, replace=False), n - 1] = 1.0
    data_np = dict(obs=obs, act=act, rew=rew, cost=cost, obs2=obs2, done=done, logp=logp)
    eps_log = []
    orig = tdn._standard_normal

    def rec(shape, dtype, device):
        e = orig(shape, dtype=dtype, device=device)
        eps_log.append(e.detach().numpy().copy())
        return e
    tdn._standard_normal = rec
    outs = []
    for it in range(2):
        data = {k: torch.from_numpy(v.copy()) for k, v in data_np.items()}
        tb = alg.model_update(data, it)
        outs.append(tb)
        sd = {k: v.detach().numpy().copy() for k, v in alg.networks.state_dict().items()}
        if it == 0:
            sd0 = sd
    tdn._standard_normal = orig
    tb0 = outs[0]
    d = {"in_" + k: v for k, v in data_np.items()}
    for k, v in init_sd.items():
        d["init/" + k] = v
    for k, v in sd0.items():
        d["after0/" + k] = v
    for k, v in sd.items():
        d["after1/" + k] = v
    for i, e in enumerate(eps_log):
        d[f"eps{i}"] = e
    d["tb_keys"] = np.array(list(tb0.keys()))
    d["tb_vals"] = np.array([float(v) for v in tb0.values()])
    d["cfg_B"], d["cfg_n"] = np.int64(B), np.int64(n)
    np.savez_compressed(os.path.join(OUT, "msacl_update.npz"), **d)
    print("msacl_update:", {k: round(float(v), 6) for k, v in tb0.items()}, "eps draws:", len(eps_log))


_INTERMEDIATES = {
    "_q_update": ("q1", "q2", "next_q", "next_logp", "backup"),
    "_lyapunov_update": ("logp", "ratio", "is_clip_ratio", "lya_obs", "lya_obs2", "ESL", "lya_diff", "loss_lya2",
                         "loss_lya3"),
    "_policy_update": ("new_act_logp", "is_ratio", "start_lya", "lya_obs2", "mb_stability_adv", "loss_policy_q",
                       "loss_policy_lya"),
}


def gen_msacl_bench(B=256, n=20, seed=13):
    """msacl_update_bench.npz: two MSACL.model_update calls at the benchmark configuration
    (example/msacl_train.py defaults: QuadTracking dims, 256-wide critics / Lyapunov (output 256) /
    policy, B = 256 windows of n = 20) with every per-window intermediate of the reference's
    update functions (locals at return of _q_update / _lyapunov_update / _policy_update, read by a
    profile hook: backup, ratio, is_clip_ratio, ESL, lya_diff, normalised stability advantage, ...)
    and the Adam moments after each call (the parameter gradients: exp_avg = (1 - b1) g on the
    first step). Windows are chained like the sampler's (obs[k+1] = obs2[k] unless done)."""
    import torch
    import torch.distributions.normal as tdn

    torch.Tensor.cuda = lambda self, *a, **k: self   # build container has no GPU (this process only)
    torch.nn.Module.cuda = lambda self, *a, **k: self
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from RL.algorithm.msacl import MSACL

    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    cls = OE.QuadTracking
    D, A = cls.obs_dim, cls.act_dim
    kw = dict(env_name="QuadTracking", obs_dim=D, act_dim=A, action_type="continu",
              action_high_limit=cls.act_high.copy(), action_low_limit=cls.act_low.copy(),
              value_func_name="ActionValue", value_func_type="MLP", value_hidden_sizes=[256, 256],
              value_hidden_activation="relu", value_output_activation="linear",
              lyapunov_func_name="LyapunovValue", lyapunov_func_type="MLP", lyapunov_hidden_sizes=[256, 256],
              lyapunov_hidden_activation="tanh", lyapunov_output_dim=256, lyapunov_output_activation="linear",
              lyapunov_single_input_dim=False, policy_func_name="StochaPolicy", policy_func_type="MLP",
              policy_act_distribution="TanhGaussDistribution", policy_hidden_sizes=[256, 256],
              policy_hidden_activation="relu", policy_min_log_std=-20, policy_max_log_std=1,
              q_learning_rate=1e-3, lyapunov_learning_rate=1e-3, policy_learning_rate=3e-4, alpha_learning_rate=1e-3,
              lya_diff_scale=10.0, lya_zero_scale=1.0, lya_positive_scale=1.0, gamma=0.99, retrace_lambda=0.95,
              tau=0.005, disable_auto_alpha=False, alpha=1.0, set_alpha_bound=False, alpha_bound=2.0, n_step=n,
              policy_frequency=2, target_network_frequency=1, anneal_lr=False, alpha1=1, alpha2=2, lya_eta=0.15,
              clip_coef=0.1, replay_batch_size=B, max_iteration=1000000)
    alg = MSACL(**kw)
    init_sd = {k: v.detach().numpy().copy() for k, v in alg.networks.state_dict().items()}
    # chained windows: a contracting random walk in the 12-d error space, episode ends at slot n-1
    x = np.zeros((B, n + 1, D), np.float64)
    x[:, 0] = rng.standard_normal((B, D)) * 0.2
    for k in range(n):
        x[:, k + 1] = 0.93 * x[:, k] + rng.standard_normal((B, D)) * 0.03
    obs, obs2 = x[:, :n].astype(F32), x[:, 1:].astype(F32)
    lo, hi = cls.act_low, cls.act_high
    act = (lo + (hi - lo) * rng.uniform(0.05, 0.95, size=(B, n, A))).astype(F32)
    with torch.no_grad():
        dist = alg.networks.create_action_distributions(alg.networks.policy(torch.from_numpy(obs)))
        lp = dist.log_prob(torch.from_numpy(act)).numpy()
    logp = (lp + rng.normal(0, 0.5, size=lp.shape)).astype(F32)
    rew = (-(obs2.astype(np.float64) ** 2).sum(-1) * 100 + rng.standard_normal((B, n))).astype(F32)
    cost = ((obs2.astype(np.float64) ** 2).sum(-1) * 100).astype(F32)
    done = np.zeros((B, n), F32)
    done[rng.choice(B, B // 8, replace=False), n - 1] = 1.0
    data_np = dict(obs=obs, act=act, rew=rew, cost=cost, obs2=obs2, done=done, logp=logp)

    eps_log, inter = [], []
    orig = tdn._standard_normal

    def rec(shape, dtype, device):
        e = orig(shape, dtype=dtype, device=device)
        eps_log.append(e.detach().numpy().copy())
        return e

    def prof(frame, event, arg):
        if event == "return" and frame.f_code.co_name in _INTERMEDIATES and "self" in frame.f_locals \
                and isinstance(frame.f_locals["self"], MSACL):
            loc = frame.f_locals
            vals = {k: loc[k].detach().numpy().copy() for k in _INTERMEDIATES[frame.f_code.co_name] if k in loc}
            if frame.f_code.co_name == "_policy_update":  # Adam moments after each policy step
                st = loc["self"].networks.policy_optimizer.state_dict()["state"]
                for i, (pn, _) in enumerate(loc["self"].networks.policy.named_parameters()):
                    vals[f"adam/{pn}/exp_avg"] = st[i]["exp_avg"].numpy().copy()
            inter.append((frame.f_code.co_name, vals))

    nets = alg.networks
    opts = {"q1": (nets.q1, nets.q1_optimizer), "q2": (nets.q2, nets.q2_optimizer),
            "lyapunov": (nets.lyapunov, nets.lyapunov_optimizer), "policy": (nets.policy, nets.policy_optimizer)}
    d = {"in_" + k: v for k, v in data_np.items()}
    for k, v in init_sd.items():
        d["init/" + k] = v
    tdn._standard_normal = rec
    try:
        for it in range(2):
            data = {k: torch.from_numpy(v.copy()) for k, v in data_np.items()}
            inter.clear()
            sys.setprofile(prof)
            try:
                tb = alg.model_update(data, it)
            finally:
                sys.setprofile(None)
            if it == 0:
                d["tb_keys"] = np.array(list(tb.keys()))
                d["tb_vals"] = np.array([float(v) for v in tb.values()])
            else:
                assert tb is None
            counts = {}
            for fn, vals in inter:
                c = counts.get(fn, 0)
                counts[fn] = c + 1
                for k, v in vals.items():
                    d[f"it{it}/{fn[1:]}{c}/{k}"] = v
            for k, v in alg.networks.state_dict().items():
                d[f"after{it}/" + k] = v.detach().numpy().copy()
            for name, (net, opt) in opts.items():
                st = opt.state_dict()["state"]
                for i, (pn, _) in enumerate(net.named_parameters()):
                    d[f"adam{it}/{name}.{pn}/exp_avg"] = st[i]["exp_avg"].numpy().copy()
                    d[f"adam{it}/{name}.{pn}/exp_avg_sq"] = st[i]["exp_avg_sq"].numpy().copy()
    finally:
        tdn._standard_normal = orig
        sys.setprofile(None)
    for i, e in enumerate(eps_log):
        d[f"eps{i}"] = e
    d["n_eps"] = np.int64(len(eps_log))
    d["cfg_B"], d["cfg_n"] = np.int64(B), np.int64(n)
    np.savez_compressed(os.path.join(OUT, "msacl_update_bench.npz"), **d)
    print("msacl_update_bench:", {k: round(float(v), 6) for k, v in zip(d["tb_keys"], d["tb_vals"])},
          "eps draws:", len(eps_log), "intermediates:", sorted({k.split("/")[1] for k in d if k.startswith("it")}))


# ---------------------------------------------------------------------- SAC / LAC / PPO / POLYC updates
def _alg_kwargs(env="QuadTracking", hidden=64):
    cls = OE.ENVS[env]
    return dict(env_name=env, obs_dim=cls.obs_dim, act_dim=cls.act_dim, action_type="continu",
                action_high_limit=cls.act_high.copy(), action_low_limit=cls.act_low.copy(),
                value_func_type="MLP", value_hidden_sizes=[hidden, hidden], value_hidden_activation="relu",
                value_output_activation="linear", policy_func_name="StochaPolicy", policy_func_type="MLP",
                policy_act_distribution="TanhGaussDistribution", policy_hidden_sizes=[hidden, hidden],
                policy_hidden_activation="relu", policy_min_log_std=-20, policy_max_log_std=1, target_value=0.0)


def _off_batch(rng, env, B):
    cls = OE.ENVS[env]
    D, A = cls.obs_dim, cls.act_dim
    obs = (rng.standard_normal((B, D)) * 0.3).astype(F32)
    obs2 = (obs + rng.standard_normal((B, D)).astype(F32) * 0.05).astype(F32)
    act = (cls.act_low + (cls.act_high - cls.act_low) * rng.uniform(0.05, 0.95, size=(B, A))).astype(F32)
    done = np.zeros(B, F32)
    done[rng.choice(B, B // 8, replace=False)] = 1.0
    return dict(obs=obs, act=act, rew=(rng.standard_normal(B) * 10).astype(F32),
                cost=rng.uniform(0, 5, size=B).astype(F32), obs2=obs2, done=done,
                logp=(rng.standard_normal(B)).astype(F32))


def _record_updates(alg, data_np, calls, tag, extra_fn=None):
    """Run `calls` (list of callables taking a fresh torch data dict) with the Normal.rsample
    noise recorded; store inputs, weights before/after each call, tb values of the first."""
    import torch
    import torch.distributions.normal as tdn
    init_sd = {k: v.detach().numpy().copy() for k, v in alg.networks.state_dict().items()}
    eps_log = []
    orig = tdn._standard_normal

    def rec(shape, dtype, device):
        e = orig(shape, dtype=dtype, device=device)
        eps_log.append(e.detach().numpy().copy())
        return e
    tdn._standard_normal = rec
    d = {"in_" + k: v for k, v in data_np.items()}
    for k, v in init_sd.items():
        d["init/" + k] = v
    try:
        for i, call in enumerate(calls):
            data = {k: torch.from_numpy(v.copy()) for k, v in data_np.items()}
            out = call(data)
            tb = out[0] if isinstance(out, tuple) else out
            if tb is not None and "tb_keys" not in d:
                d["tb_keys"] = np.array(list(tb.keys()))
                d["tb_vals"] = np.array([float(v) for v in tb.values()])
            for k, v in alg.networks.state_dict().items():
                d[f"after{i}/" + k] = v.detach().numpy().copy()
    finally:
        tdn._standard_normal = orig
    for i, e in enumerate(eps_log):
        d[f"eps{i}"] = e
    d["n_eps"] = np.int64(len(eps_log))
    d.update(extra_fn() if extra_fn else {})
    np.savez_compressed(os.path.join(OUT, f"{tag}_update.npz"), **d)
    print(f"{tag}_update:", {k: round(float(v), 5) for k, v in zip(d.get("tb_keys", []), d.get("tb_vals", []))},
          "eps draws:", len(eps_log))


def gen_algs(seed=21):
    import torch
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from RL.algorithm.lac import LAC
    from RL.algorithm.polyc import POLYC
    from RL.algorithm.ppo import PPO
    from RL.algorithm.sac import SAC

    # SAC: two model_update calls (iteration 0: Q + target + 2 policy/alpha steps; 1: Q + target)
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    kw = _alg_kwargs()
    kw.update(value_func_name="ActionValue", q_learning_rate=1e-3, policy_learning_rate=3e-4, alpha_learning_rate=1e-3,
              gamma=0.99, tau=0.005, alpha=1.0, auto_alpha=True, policy_frequency=2, target_network_frequency=1)
    alg = SAC(**kw)
    data = _off_batch(rng, "QuadTracking", 64)
    _record_updates(alg, data, [lambda d: alg.model_update(d, 0), lambda d: alg.model_update(d, 1)], "sac")

    torch.manual_seed(seed + 1)
    rng = np.random.default_rng(seed + 1)
    kw = _alg_kwargs("Pendulum")
    kw.update(value_func_name="ActionValue", l_learning_rate=1e-3, policy_learning_rate=3e-4, alpha_learning_rate=1e-3,
              beta_learning_rate=1e-3, gamma=0.99, tau=0.005, alpha=1.0, beta=1.0, auto_alpha=True, alpha3=0.01,
              policy_frequency=2, target_network_frequency=1)
    alg = LAC(**kw)
    data = _off_batch(rng, "Pendulum", 64)
    _record_updates(alg, data, [lambda d: alg.model_update(d, 0), lambda d: alg.model_update(d, 1)], "lac")

    # PPO / POLYC: one model_update on a synthetic on-policy batch; np.random drives the shuffles
    for tag, Alg in (("ppo", PPO), ("polyc", POLYC)):
        torch.manual_seed(seed + 2)
        rng = np.random.default_rng(seed + 2)
        env = "DuctedFan"
        kw = _alg_kwargs(env)
        cls = OE.ENVS[env]
        kw.update(value_func_name="StateValue", lyapunov_func_name="LyapunovValue", lyapunov_func_type="MLP",
                  lyapunov_hidden_sizes=[64, 64], lyapunov_hidden_activation="tanh", lyapunov_output_dim=32,
                  lyapunov_output_activation="linear", lyapunov_single_input_dim=False, learning_rate=1e-3,
                  policy_learning_rate=3e-4, loss_coefficient_value=1.0, loss_coefficient_entropy=0.01,
                  loss_coefficient_kl=0.2, loss_value_clip=True, value_clip=0.5, beta=0.3, gamma=0.99,
                  schedule_adam="linear", schedule_clip="linear", clip=0.1, max_iteration=100, num_repeat=2,
                  num_mini_batch=4, mini_batch_size=16, sample_batch_size=64, env_num=2)
        if tag == "polyc":  # polyc.py:36 builds the Lyapunov net from the TOP-LEVEL kwargs
            kw.update(apprfunc="MLP", name="LyapunovValue", input_dim=cls.obs_dim, output_dim=32, hidden_sizes=[64, 64],
                      hidden_activation="tanh", output_activation="linear")
        alg = Alg(**kw)
        N = 128
        D, A = cls.obs_dim, cls.act_dim
        obs = (rng.standard_normal((N, D)) * 0.3).astype(F32)
        act = (cls.act_low + (cls.act_high - cls.act_low) * rng.uniform(0.05, 0.95, size=(N, A))).astype(F32)
        with torch.no_grad():
            dist = alg.networks.create_action_distributions(alg.networks.policy(torch.from_numpy(obs)))
            lp = dist.log_prob(torch.from_numpy(act)).numpy()
        data = dict(obs=obs, obs2=(obs + rng.standard_normal((N, D)).astype(F32) * 0.05).astype(F32), act=act,
                    rew=(rng.standard_normal(N)).astype(F32), cost=rng.uniform(0, 5, N).astype(F32),
                    done=np.zeros(N, np.bool_), logp=(lp + rng.normal(0, 0.3, N)).astype(F32),
                    adv=(rng.standard_normal(N) * 2).astype(F32), ret=(rng.standard_normal(N) * 3).astype(F32),
                    val=(rng.standard_normal(N) * 3).astype(F32))
        np.random.seed(seed + 3)
        _record_updates(alg, data, [lambda d: alg.model_update(d)], tag,
                        extra_fn=lambda: dict(np_seed=np.int64(seed + 3), indices_after=alg.indices.copy()))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["env", "reset", "nstep", "msacl", "step", "onpolicy", "algs", "eval"]
    if "env" in which:
        for nm in OE.ENVS:
            gen_env_pairs(nm)
    if "reset" in which:
        gen_quad_reset()
    if "polar64" in which or "env" in which:
        gen_quad_polar64()
    if "nstep" in which:
        for nm in OE.ENVS:
            gen_nstep_trace(nm)
        gen_nstep_trace("VanderPol", E=16, T=60, n_step=20, seed=5, tag="_n20")
    if "nstep" in which or "nstep20" in which:
        # the benchmark's n = 20 for the envs of configs 3 and 4
        gen_nstep_trace("QuadTracking", E=16, T=60, n_step=20, seed=5, tag="_n20", log_std=-4.0)
        gen_nstep_trace("TwoLink", E=16, T=60, n_step=20, seed=5, tag="_n20", log_std=-3.0, gentle_policy=(),
                        pd_gain=(60.0, 12.0))
        gen_nstep_trace("DuctedFan", E=16, T=60, n_step=20, seed=5, tag="_n20")
    if "msacl" in which:
        gen_msacl()
    if "msacl_bench" in which or "msacl" in which:
        gen_msacl_bench()
    if "step" in which:
        for nm in ("VanderPol", "TwoLink", "QuadTracking"):
            gen_step_trace(nm)
    if "eval" in which:
        for nm in ("VanderPol", "DuctedFan", "QuadTracking"):
            gen_evaluator(nm)
    if "algs" in which:
        gen_algs()
    if "onpolicy" in which:
        for nm in ("Pendulum", "DuctedFan", "QuadTracking"):
            gen_onpolicy_trace(nm)
