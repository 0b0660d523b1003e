"""CPU n-step off-policy sampler: BASELINE.json config 1 ("VanderPol, 1 env, MSACL
off_serial_trainer on CPU reference sampler").

The reference's BaseSampler._n_step / NstepOffSampler._sample (RL/trainer/sampler/base.py:118-222,
nstep_off_sampler.py:15-30) on the CPU, with the env batch stepped by the engine's CPU build
(env/host_vector_env.py -> libmsacl_host.so, the gfx950 kernels' env math compiled for the host):

  per lockstep step   logits = policy(obs) -> TanhGauss sample() -> (+ one scalar
                      np.random.normal(mean, std), explore_noise.py:8-9) -> clip to the action box
                      -> envs.step -> real_next_obs (final_observation on done rows) ->
                      rew_plus_cost (reward * reward_scale, sum(real_next_obs^2) * cost_scale,
                      rew_plus_cost.py:16-23) -> append to each env's n-step ring -> emit the full
                      rings in env-index order -> clear the rings whose last entry is done.

The per-env deques are a ring array [E][n] per field (one vectorised shift per step instead of E
Python deques); windows come out in the reference's order. sample() returns a HostWindowBatch:
a sequence of nStepExperience-ordered 7-tuples (obs, act, rew, cost, obs2, done, logp), also
carrying the stacked [W, n, ...] arrays so HostNstepReplayBuffer.add_batch writes them in one go.
Selected only by an explicit device="cpu"; the GPU path never routes here.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ...create_pkg.create_alg import create_approx_contrainer
from ...env.host_vector_env import HostVectorEnv
from ...utils.tensorboard_setup import tb_tags
from ..buffer.host_nstep_replay_buffer import KEYS, HostWindowBatch


class CpuNstepOffSampler:
    def __init__(self, **kwargs):
        self.env_id = kwargs["env_name"]
        self.num_envs = int(kwargs["env_num"])
        self.device = torch.device("cpu")
        self.envs = HostVectorEnv(self.env_id, self.num_envs, seed=int(kwargs.get("env_seed") or 0) +
                                  int(kwargs.get("sampler_seed_offset", 0)))
        self.obs_dim = self.envs.single_observation_space.shape
        self.act_dim = self.envs.single_action_space.shape
        self.networks = create_approx_contrainer(**kwargs)
        self.sample_batch_size = int(kwargs["sample_batch_size"]) * self.num_envs
        self.action_type = kwargs["action_type"]
        if self.action_type != "continu":
            raise RuntimeError("Only continuous action space is supported!")
        self.reward_scale = kwargs["reward_scale"]
        self.cost_scale = kwargs["cost_scale"]
        self.noise_params = kwargs.get("noise_params")
        self.target_value = kwargs.get("target_value", 0.0)
        self.total_sample_number = 0
        self.horizon = self.sample_batch_size // self.num_envs
        self.n_step = int(kwargs.get("n_step", 1))
        self.gamma = kwargs.get("gamma", 0.99)
        self.td_lambda = kwargs.get("retrace_lambda", 0.95)
        E, n, D, A = self.num_envs, self.n_step, self.envs.obs_dim, self.envs.act_dim
        self._low = np.asarray(self.envs.single_action_space.low, np.float32)
        self._high = np.asarray(self.envs.single_action_space.high, np.float32)
        self._ring = {"obs": np.zeros((E, n, D), np.float32), "act": np.zeros((E, n, A), np.float32),
                      "rew": np.zeros((E, n), np.float32), "cost": np.zeros((E, n), np.float32),
                      "obs2": np.zeros((E, n, D), np.float32), "done": np.zeros((E, n), np.float32),
                      "logp": np.zeros((E, n), np.float32)}
        self._len = np.zeros(E, np.int64)
        obs, _ = self.envs.reset(seed=None)
        self.obs = obs.numpy().astype(np.float32)

    # ------------------------------------------------------------------ reference API
    def get_total_sample_num(self) -> int:
        return self.total_sample_number

    def get_total_sample_number(self) -> int:
        return self.total_sample_number

    def load_state_dict(self, state_dict):
        self.networks.load_state_dict(state_dict)

    # ------------------------------------------------------------------ one lockstep step
    def _policy_actions(self):
        """policy -> distribution sample -> noise -> clip (base.py:126-147)."""
        with torch.no_grad():
            logits = self.networks.policy(torch.from_numpy(self.obs))
            dist = self.networks.create_action_distributions(logits)
            actions, log_probs = dist.sample()
        actions = actions.numpy().astype(np.float32)
        log_probs = log_probs.numpy().astype(np.float32)
        if self.noise_params is not None:  # GaussNoise: one scalar per step, added to every action
            actions = actions + np.random.normal(self.noise_params["mean"], self.noise_params["std"])
        return actions.clip(self._low, self._high), log_probs

    def _push(self, obs, act, rew, cost, obs2, done, logp):
        """Append one step to every env's ring; returns the full windows in env-index order and
        clears the rings whose newest entry is done (base.py:176-216)."""
        n = self.n_step
        full = self._len == n
        rows = np.arange(self.num_envs)
        pos = np.where(full, n - 1, self._len)
        for k, v in zip(KEYS, (obs, act, rew, cost, obs2, done, logp)):
            r = self._ring[k]
            if full.any():
                r[full, :-1] = r[full, 1:]
            r[rows, pos] = v
        self._len = np.minimum(self._len + 1, n)
        emit = np.nonzero(self._len == n)[0]
        out = {k: self._ring[k][emit].copy() for k in KEYS}
        self._len[done.astype(bool)] = 0
        return out

    def _finish(self, actions_clip, log_probs, reset_states=None):
        obs = self.obs
        next_obs, rew, term, trunc, info = self.envs.step(actions_clip, reset_states=reset_states)
        next_obs = next_obs.numpy().astype(np.float32)
        real = info["final_observation"].numpy().astype(np.float32)  # == next_obs on live rows
        dones = np.logical_or(term.numpy(), trunc.numpy())
        rewards = rew.numpy().astype(np.float32) * self.reward_scale       # rew_plus_cost.py:16-23
        costs = (real ** 2).sum(axis=1) * self.cost_scale
        out = self._push(obs, actions_clip, rewards, costs, real, dones.astype(np.float32), log_probs)
        self.obs = next_obs
        return out

    def _n_step(self):
        actions_clip, log_probs = self._policy_actions()
        return self._finish(actions_clip, log_probs)

    def _sample(self):
        parts = [self._n_step() for _ in range(self.horizon)]
        return HostWindowBatch({k: np.concatenate([p[k] for p in parts]) for k in KEYS})

    def sample(self):
        """-> (HostWindowBatch, {sampler_time ms}) (base.py:308-323)."""
        self.total_sample_number += self.sample_batch_size
        t0 = time.perf_counter()
        data = self._sample()
        return data, {tb_tags["sampler_time"]: (time.perf_counter() - t0) * 1000}

    # ------------------------------------------------------------------ parity mode
    def step_injected(self, actions, logp, reset_states=None):
        """One lockstep step with injected (already clipped) actions, log-probs and the states
        of any autoreset; returns that step's windows as a HostWindowBatch."""
        act = np.ascontiguousarray(actions, np.float32).reshape(self.num_envs, self.envs.act_dim)
        lp = np.ascontiguousarray(logp, np.float32).reshape(self.num_envs)
        return HostWindowBatch(self._finish(act, lp, reset_states))
