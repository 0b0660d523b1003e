"""CPU lockstep vector env (BASELINE.json config 1: the CPU sampler plumbing, no GPU).

The same gymnasium SyncVectorEnv contract as HipVectorEnv (RL/create_pkg/create_envs.py:24-32,
RL/env/make_env.py:10-41; autoreset + final_observation), stepped by the engine's CPU build
(csrc/host_engine.hip -> libmsacl_host.so): the gfx950 kernels' own env math (env_math.h) and
reset draws (reset_draw.h) compiled for the host. Tensors are CPU tensors. Selected explicitly
with device="cpu"; the GPU path never routes here.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native as N
from .hip_vector_env import HipVectorEnv


class HostVectorEnv(HipVectorEnv):
    def __init__(self, env_id: str, num_envs: int, seed: int = 0, device=None):
        super().__init__(env_id, num_envs, seed=seed, device=torch.device("cpu"))

    @staticmethod
    def _env_info(env_id):
        return N.host_env_info(env_id)  # the CPU build answers for itself (no HIP library load)

    @property
    def device(self):
        return torch.device("cpu")

    def handle(self):
        if self._h is None:
            h = ctypes.c_void_p()
            N.host_check(N.host_lib().mhh_env_create(N.ENV_IDS[self.env_id], self.num_envs, self.seed, ctypes.byref(h)),
                         "mhh_env_create")
            self._h = h
        return self._h

    def close(self):
        if self._h is not None:
            N.host_lib().mhh_env_destroy(self._h)
            self._h = None

    def _host(self, x, cols, name):
        if x is None:
            return None
        t = torch.as_tensor(np.asarray(x.cpu() if torch.is_tensor(x) else x, np.float32)).contiguous()
        if t.numel() != self.num_envs * cols:
            raise ValueError(f"{name} must have {self.num_envs * cols} elements (got {t.numel()})")
        return t

    def reset(self, seed=None, options=None, reset_states=None):
        obs = torch.empty(self.num_envs, self.obs_dim)
        rs = self._host(reset_states, self.reset_dim, "reset_states")
        N.host_check(N.host_lib().mhh_env_reset(self.handle(), N.hptr(rs), N.hptr(obs)), "mhh_env_reset")
        return obs, {}

    def step(self, actions, reset_states=None):
        act = self._host(actions, self.act_dim, "actions")
        rs = self._host(reset_states, self.reset_dim, "reset_states")
        E, D = self.num_envs, self.obs_dim
        next_obs, real, rew = torch.empty(E, D), torch.empty(E, D), torch.empty(E)
        term, trunc = torch.empty(E, dtype=torch.uint8), torch.empty(E, dtype=torch.uint8)
        N.host_check(N.host_lib().mhh_env_step(self.handle(), N.hptr(act), N.hptr(rs), N.hptr(next_obs), N.hptr(real),
                                               N.hptr(rew), N.hptr(term), N.hptr(trunc)), "mhh_env_step")
        return next_obs, rew, term.bool(), trunc.bool(), {"final_observation": real}

    def get_state(self):
        st = torch.empty(self.num_envs, self.state_dim)
        xs = torch.empty(self.num_envs, max(self.xstate_dim, 1), dtype=torch.float64)
        steps = torch.empty(self.num_envs, dtype=torch.int32)
        N.host_check(N.host_lib().mhh_env_get_state(self.handle(), N.hptr(st), N.hptr(xs) if self.xstate_dim else None,
                                                    N.hptr(steps)), "mhh_env_get_state")
        return st, (xs if self.xstate_dim else None), steps

    def set_state(self, state, xstate=None, steps=None):
        st = self._host(state, self.state_dim, "state")
        xs = None
        if xstate is not None and self.xstate_dim:
            xs = torch.as_tensor(np.asarray(xstate.cpu() if torch.is_tensor(xstate) else xstate, np.float64)).contiguous()
        sp = None
        if steps is not None:
            sp = torch.as_tensor(np.asarray(steps.cpu() if torch.is_tensor(steps) else steps, np.int32)).contiguous()
        N.host_check(N.host_lib().mhh_env_set_state(self.handle(), N.hptr(st), N.hptr(xs), N.hptr(sp)),
                     "mhh_env_set_state")


def make_vector_env(env_id, num_envs, seed=0, device=None):
    """HostVectorEnv for device="cpu", else the device env."""
    if device is not None and torch.device(device).type == "cpu":
        return HostVectorEnv(env_id, num_envs, seed=seed)
    return HipVectorEnv(env_id, num_envs, seed=seed, device=device)
