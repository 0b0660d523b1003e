"""CPU ORACLE — test infrastructure only.

Restatement of the rollout path around the envs:
  * gymnasium 0.28.1 SyncVectorEnv.step autoreset semantics (third-party, pinned in the
    reference's requirements/requirements.txt:24, absent from this image). Published algorithm:
    for each sub-env i in order: (obs, rew, term, trunc, info) = env.step(a_i); if term or
    trunc: info["final_observation"] = obs; obs = env.reset(); rewards go into a float64
    buffer; observations are stacked float32.
  * RL/utils/rew_plus_cost.py:6-23 (reward * reward_scale, sum(real_next_obs^2) * cost_scale).
  * RL/trainer/sampler/base.py:118-222 (`_n_step`): per-env deque(maxlen=n), window emitted when
    the deque is full, deque cleared when the newest item is done, env-index emission order.
  * RL/trainer/buffer/nstep_replay_buffer.py:91-150 ring storage.
Also the CPU baseline leg of bench.py (a faithful per-env Python loop, like the reference).
"""
from __future__ import annotations

from collections import deque

import numpy as np

from oracle import envs as E

F32 = np.float32


class VectorEnv:
    """Batch of one env id with SyncVectorEnv autoreset. Reset states come from `reset_fn(idx)`
    (returns [len(idx), reset_dim] float32) so parity tests can inject them."""

    def __init__(self, name, num_envs, reset_fn):
        self.name = name
        self.cls = E.ENVS[name]
        self.n = num_envs
        self.reset_fn = reset_fn
        self.state = None
        self.xstate = None
        self.steps = np.zeros(num_envs, np.int64)

    def reset(self):
        rs = self.reset_fn(np.arange(self.n))
        self.state, self.xstate, obs = E.env_reset_from(self.name, rs)
        self.steps[:] = 0
        return obs

    def step(self, actions):
        s2, xs2, obs, rew, term, trunc = E.env_step(self.name, self.state, actions, self.xstate, self.steps)
        rewards = rew.astype(np.float64)          # SyncVectorEnv._rewards buffer (float64)
        done = term | trunc
        final_obs = obs.copy()
        next_obs = obs.copy()
        self.state = s2
        self.xstate = xs2
        self.steps = self.steps + 1
        idx = np.nonzero(done)[0]
        if idx.size:
            rs = self.reset_fn(idx)
            st, xs, o = E.env_reset_from(self.name, rs)
            self.state[idx] = st
            if self.xstate is not None:
                self.xstate[idx] = xs
            next_obs[idx] = o
            self.steps[idx] = 0
        return next_obs, rewards, term, trunc, final_obs


def rew_plus_cost(real_next_obs, original_rewards, reward_scale, cost_scale):
    """RL/utils/rew_plus_cost.py:18-21."""
    rewards = original_rewards * reward_scale
    costs = (real_next_obs ** 2).sum(axis=1) * cost_scale
    return rewards, costs


class NStepRollout:
    """BaseSampler._n_step with injected actions (the policy's torch RNG cannot be replayed on
    the device, so parity mode feeds the sampled+clipped actions and their log-probs)."""

    def __init__(self, venv: VectorEnv, n_step, reward_scale=100.0, cost_scale=100.0):
        self.venv = venv
        self.n = n_step
        self.reward_scale = reward_scale
        self.cost_scale = cost_scale
        self.deques = [deque(maxlen=n_step) for _ in range(venv.n)]
        self.obs = venv.reset()

    def step(self, actions_clip, logp):
        next_obs, rewards, term, trunc, final_obs = self.venv.step(actions_clip)
        next_obs = np.float32(next_obs)
        original_rewards = np.float32(rewards)
        obs = np.float32(self.obs)
        dones = np.logical_or(term, trunc)
        real_next_obs = next_obs.copy()
        real_next_obs[dones] = final_obs[dones]
        rew, cost = rew_plus_cost(real_next_obs, original_rewards, self.reward_scale, self.cost_scale)
        windows = []
        for i in range(self.venv.n):
            dq = self.deques[i]
            dq.append((obs[i], actions_clip[i], rew[i], cost[i], real_next_obs[i], dones[i], logp[i]))
            if len(dq) == self.n:
                windows.append(tuple(np.array([it[j] for it in dq], dtype=F32) for j in range(7)))
            if dq and dq[-1][5]:
                dq.clear()
        self.obs = next_obs
        return windows, dict(real_next_obs=real_next_obs, rew=rew, cost=cost, done=dones, next_obs=next_obs)


class NStepWindows:
    """The `_n_step` deque bookkeeping of NStepRollout (base.py:178-217: per env a
    deque(maxlen=n); append the step's record; a full deque is emitted oldest-first; the deque is
    cleared when the newest record is done; emission in env-index order) restated over arrays
    for 65,536-env parity tests: each env's deque is a ring of n records with a length and a
    write position. Records are given as the 7 per-step arrays (obs[E,D], act[E,A], rew[E],
    cost[E], obs2[E,D], done[E], logp[E]); `push` returns the step's windows as 7 arrays
    [W, n, ...] (W = emitting envs) in WindowStore.KEYS order. tests/test_oracle_windows.py pins
    it to NStepRollout."""

    def __init__(self, num_envs, n_step, obs_dim, act_dim):
        self.E, self.n, self.D, self.A = num_envs, n_step, obs_dim, act_dim
        self.F = 2 * obs_dim + act_dim + 4
        self.ring = np.zeros((num_envs, n_step, self.F), F32)
        self.len = np.zeros(num_envs, np.int64)
        self.pos = np.zeros(num_envs, np.int64)

    def push(self, obs, act, rew, cost, obs2, done, logp):
        E, n, D, A = self.E, self.n, self.D, self.A
        rec = np.concatenate([np.asarray(obs, F32).reshape(E, D), np.asarray(act, F32).reshape(E, A),
                              np.asarray(obs2, F32).reshape(E, D), np.asarray(rew, F32).reshape(E, 1),
                              np.asarray(cost, F32).reshape(E, 1), np.asarray(done, F32).reshape(E, 1),
                              np.asarray(logp, F32).reshape(E, 1)], axis=1)
        env = np.arange(E)
        self.ring[env, self.pos] = rec
        self.pos = (self.pos + 1) % n
        self.len = np.minimum(self.len + 1, n)
        em = np.nonzero(self.len == n)[0]                   # env-index order
        slots = (self.pos[em, None] + np.arange(n)[None, :]) % n  # oldest first
        w = self.ring[em[:, None], slots]                    # [W, n, F]
        self.len[np.asarray(done, bool).reshape(E)] = 0      # deque.clear()
        s = 2 * D + A
        return (w[:, :, :D], w[:, :, D:D + A], w[:, :, s], w[:, :, s + 1], w[:, :, D + A:s], w[:, :, s + 2],
                w[:, :, s + 3])  # KEYS order: obs, act, rew, cost, obs2, done, logp


class WindowStore:
    """NstepReplayBuffer storage (nstep_replay_buffer.py:52-125)."""

    KEYS = ("obs", "act", "rew", "cost", "obs2", "done", "logp")

    def __init__(self, max_size, n_step, obs_dim, act_dim):
        self.max_size = max_size
        self.buf = {
            "obs": np.zeros((max_size, n_step, obs_dim), F32),
            "act": np.zeros((max_size, n_step, act_dim), F32),
            "rew": np.zeros((max_size, n_step), F32),
            "cost": np.zeros((max_size, n_step), F32),
            "obs2": np.zeros((max_size, n_step, obs_dim), F32),
            "done": np.zeros((max_size, n_step), F32),
            "logp": np.zeros((max_size, n_step), F32),
        }
        self.ptr = 0
        self.size = 0
        self.total = 0

    def add_batch(self, windows):
        for w in windows:
            for k, v in zip(self.KEYS, w):
                self.buf[k][self.ptr] = v
            self.ptr = (self.ptr + 1) % self.max_size
            self.size = min(self.size + 1, self.max_size)
            self.total += 1

    def gather(self, idx):
        return {k: v[idx] for k, v in self.buf.items()}


# ------------------------------------------------------------------------ CPU baseline
class CpuPolicy:
    """StochaPolicy forward (RL/apprfunc/mlp.py:111-136) in NumPy for the CPU baseline:
    obs -> Linear/ReLU x2 -> Linear -> (mean, clamp(log_std).exp())."""

    def __init__(self, weights):
        self.w = [(np.asarray(W, F32), np.asarray(b, F32)) for W, b in weights]

    def __call__(self, obs):
        h = obs
        for i, (W, b) in enumerate(self.w):
            h = h @ W.T + b
            if i < len(self.w) - 1:
                h = np.maximum(h, 0)
        a = h.shape[1] // 2
        return h[:, :a], np.exp(np.clip(h[:, a:], -20, 1))


def tanh_gauss_sample(rng, mean, std, low, high):
    """TanhGaussDistribution.sample (RL/utils/act_distribution_cls.py:45-57) + clip."""
    z = mean + std * rng.standard_normal(mean.shape).astype(F32)
    th = np.tanh(z)
    half = (high - low) / 2
    act = half * th + (high + low) / 2
    lp = (-((z - mean) ** 2) / (2 * std ** 2) - np.log(std) - np.float32(0.5 * np.log(2 * np.pi))).sum(-1)
    lp = lp - np.log(1 + 1e-6 - th ** 2).sum(-1) - np.log(half).sum(-1)
    return np.clip(act, low, high).astype(F32), lp.astype(F32)


class PerEnvCpuSampler:
    """CPU baseline with the reference's structure: per-env Python objects stepped one at a
    time (SyncVectorEnv loop), per-env deques, NumPy policy — one process, 1 thread."""

    def __init__(self, name, num_envs, n_step, policy, seed=0):
        self.name = name
        self.cls = E.ENVS[name]
        self.rng = np.random.default_rng(seed)
        self.n = num_envs
        self.policy = policy
        self.nstep = n_step
        self.deques = [deque(maxlen=n_step) for _ in range(num_envs)]
        self.state, self.xstate, self.steps, obs = [], [], [], []
        for _ in range(num_envs):
            s, xs, o = self._reset_one()
            self.state.append(s); self.xstate.append(xs); self.steps.append(0); obs.append(o)
        self.obs = np.stack(obs)

    def _reset_one(self):
        if self.name == "QuadTracking":
            rs = self.cls.reset_draw(self.rng, 1, gauss=lambda k: self.rng.standard_normal((k, 3)))
        else:
            rs = self.cls.reset_draw(self.rng, 1)
        s, xs, o = E.env_reset_from(self.name, rs)
        return s, xs, o[0]

    def step(self):
        mean, std = self.policy(self.obs)
        act, lp = tanh_gauss_sample(self.rng, mean, std, self.cls.act_low, self.cls.act_high)
        next_obs = np.empty_like(self.obs)
        real = np.empty_like(self.obs)
        rews = np.zeros(self.n, np.float64)
        dones = np.zeros(self.n, bool)
        for i in range(self.n):  # the SyncVectorEnv per-env loop
            s2, xs2, o, r, te, tr = E.env_step(self.name, self.state[i], act[i:i + 1], self.xstate[i],
                                               np.array([self.steps[i]]))
            rews[i] = r[0]
            real[i] = o[0]
            self.state[i], self.xstate[i] = s2, xs2
            self.steps[i] += 1
            if te[0] or tr[0]:
                dones[i] = True
                s, xs, o0 = self._reset_one()
                self.state[i], self.xstate[i], self.steps[i] = s, xs, 0
                next_obs[i] = o0
            else:
                next_obs[i] = o[0]
        rew, cost = rew_plus_cost(real, np.float32(rews), 100.0, 100.0)
        emitted = 0
        for i in range(self.n):
            dq = self.deques[i]
            dq.append((self.obs[i], act[i], rew[i], cost[i], real[i], dones[i], lp[i]))
            if len(dq) == self.nstep:
                _ = [np.array([it[j] for it in dq], dtype=F32) for j in range(7)]
                emitted += 1
            if dones[i]:
                dq.clear()
        self.obs = next_obs
        return emitted
