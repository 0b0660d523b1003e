"""Device on-policy sampler for PPO / POLYC (drop-in for RL/trainer/sampler/on_sampler.py:11-154).

`_sample()` runs `horizon` lockstep steps of BaseSampler._step (base.py:225-298) over all envs:
per step the policy MLP (PyTorch-ROCm) and ONE fused gfx950 rollout kernel that samples the
TanhGauss action, clips, integrates the env, autoresets, applies rew_plus_cost and writes
column t of the env-major [E][H] trajectory arrays (the reference's mb_* buffers). After the
horizon, V(obs) and V(real_next_obs) are two batched value-MLP passes over all E*H rows
(the reference evaluates V per step and per finished env, on_sampler.py:115,125-129 — same
values, batched), and the GAE kernel (csrc/gae.hip) computes advantages and discounted
returns per trajectory segment (segments end at done or at the horizon, bootstrap
V(real_next_obs) * (1 - done); _finish_trajs, :134-154). After the first call the whole
sample (rollout + values + GAE) replays as one HIP graph.

Returns the reference's dict of flattened [E*H, ...] tensors (obs, obs2, act, rew, cost, done
(bool), logp, adv, ret, val), env-major, as device views of the sampler's buffers (the
reference's torch.from_numpy views alias its mb arrays the same way).
"""
from __future__ import annotations

import ctypes

import torch

from ... import _native as N
from ...utils import dist as D
from .hip_nstep_off_sampler import HipNstepOffSampler

__all__ = ["OnSampler"]


class OnSampler(HipNstepOffSampler):
    def __init__(self, **kwargs):
        kw = dict(kwargs)
        kw["n_step"] = 1  # no n-step deques on this path (the rings stay unused)
        kw["sampler_fused_horizon"] = False  # trajectory columns, not windows: its own horizon loop
        super().__init__(**kw)
        self.gamma = kwargs["gamma"]
        self.gae_lambda = kwargs["gae_lambda"]
        E, H = self.num_envs, self.horizon
        D, A = self.envs.obs_dim, self.envs.act_dim
        f = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        self.mb_obs, self.mb_obs2, self.mb_act = f(E, H, D), f(E, H, D), f(E, H, A)
        self.mb_rew, self.mb_cost, self.mb_logp = f(E, H), f(E, H), f(E, H)
        self.mb_done = torch.zeros(E, H, dtype=torch.uint8, device=self.device)
        self.mb_val, self.mb_val2, self.mb_adv, self.mb_ret = f(E, H), f(E, H), f(E, H), f(E, H)
        self.traj = N.TrajStore(*[ctypes.c_void_p(t.data_ptr()) for t in
                                  (self.mb_obs, self.mb_act, self.mb_rew, self.mb_cost, self.mb_obs2, self.mb_done,
                                   self.mb_logp)], H)

    # ------------------------------------------------------------------ device work
    def _traj_step(self, t, logits=None, act_in=None, logp_in=None, reset_states=None):
        N.check(N.lib().mh_rollout_traj_step(self._h, N.ptr(logits), N.ptr(act_in), N.ptr(logp_in),
                                             N.ptr(reset_states), N.ptr(self.obs), ctypes.byref(self.traj), int(t),
                                             None, None, N.stream_of(self.device)), "mh_rollout_traj_step")

    def _values_and_gae(self):
        E, H, D = self.num_envs, self.horizon, self.envs.obs_dim
        value = self.networks.value
        self.mb_val.view(-1).copy_(value(self.mb_obs.view(E * H, D)))
        self.mb_val2.view(-1).copy_(value(self.mb_obs2.view(E * H, D)))
        N.check(N.lib().mh_gae(N.ptr(self.mb_val), N.ptr(self.mb_val2), N.ptr(self.mb_rew), N.ptr(self.mb_done), E, H,
                               float(self.gamma), float(self.gae_lambda), N.ptr(self.mb_adv), N.ptr(self.mb_ret),
                               N.stream_of(self.device)), "mh_gae")

    def _horizon(self, store):
        pol = self.networks.policy
        fused = self._pack_policy()
        for t in range(self.horizon):
            self._draw_noise()
            logits, raw = self._policy_fused() if fused else self._policy_raw()
            N.check(N.lib().mh_nstep_set_log_std_clamp(self._h, int(raw), float(getattr(pol, "min_log_std", -20.0)),
                                                       float(getattr(pol, "max_log_std", 1.0))), "log_std clamp")
            self._traj_step(t, logits=logits)
        self._values_and_gae()

    def _graph_for(self, store):
        key = (id(self.networks.policy), id(self.networks.value),
               tuple(p.data_ptr() for p in self.networks.policy.parameters()),
               tuple(p.data_ptr() for p in self.networks.value.parameters()), self.obs.data_ptr())
        if self._graph is None or self._graph_key != key:
            g = torch.cuda.CUDAGraph()
            with D.cuda_graph(g):
                self._horizon(None)
            self._graph, self._graph_key = g, key
        return self._graph

    def _batch(self):
        E, H, D, A = self.num_envs, self.horizon, self.envs.obs_dim, self.envs.act_dim
        return {"obs": self.mb_obs.view(E * H, D), "obs2": self.mb_obs2.view(E * H, D),
                "act": self.mb_act.view(E * H, A), "rew": self.mb_rew.view(-1), "cost": self.mb_cost.view(-1),
                "done": self.mb_done.view(-1).view(torch.bool), "logp": self.mb_logp.view(-1),
                "adv": self.mb_adv.view(-1), "ret": self.mb_ret.view(-1), "val": self.mb_val.view(-1)}

    def _sample(self):
        with torch.no_grad():
            if self.use_graph and self._eager_calls >= 1:
                self._graph_for(None).replay()
            else:
                self._horizon(None)
                self._eager_calls += 1
        return self._batch()

    def sample_with_replay_format(self):
        """(data, tb) exactly as sample() (on_sampler.py:82-84)."""
        return self.sample()

    # ------------------------------------------------------------------ parity mode
    def sample_injected(self, actions, logp, resets):
        """One _sample() with injected per-step actions [H][E][A], log-probs [H][E] and reset
        states [H][E][reset_dim] (parity with the reference's traces)."""
        dev = self.device
        with torch.no_grad():
            for t in range(self.horizon):
                a = torch.as_tensor(actions[t], dtype=torch.float32, device=dev).contiguous()
                lp = torch.as_tensor(logp[t], dtype=torch.float32, device=dev).contiguous()
                rs = torch.as_tensor(resets[t], dtype=torch.float32, device=dev).contiguous()
                N.require_device(a, "actions", torch.float32, self.num_envs * self.envs.act_dim, dev)
                N.require_device(rs, "resets", torch.float32, self.num_envs * self.envs.reset_dim, dev)
                self._traj_step(t, act_in=a, logp_in=lp, reset_states=rs)
            self._values_and_gae()
        return self._batch()
