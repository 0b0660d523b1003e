"""Device-resident lockstep vector env over the six MSACL envs.

Replaces `gym.vector.SyncVectorEnv([make_env(...)])` (RL/create_pkg/create_envs.py:24-32,
RL/env/make_env.py:10-41): the same reset/step/autoreset contract, but every env of the batch
advances in one gfx950 kernel launch (csrc/rollout.hip) and all tensors stay in HBM.
Spaces are host-side and need no GPU (init_args only reads dims and limits).
"""
from __future__ import annotations

import atexit

import numpy as np
import torch

from .. import _native as N

ENV_NAMES = tuple(N.ENV_IDS)


class Box:
    """float32 box with the attributes init_args / the samplers read (low, high, shape, dtype)."""

    def __init__(self, low, high):
        self.low = np.asarray(low, np.float32)
        self.high = np.asarray(high, np.float32)
        self.shape = self.low.shape
        self.dtype = np.dtype(np.float32)

    def __repr__(self):
        return f"Box({self.low.tolist()}, {self.high.tolist()})"


class HipVectorEnv:
    """`num_envs` copies of env `env_id` stepped in lockstep on `device`.

    reset(seed=None, reset_states=None) -> (obs[E, D], {})
    step(actions[E, A], reset_states=None) -> (next_obs, reward, terminated, truncated, infos)
      with infos["final_observation"] = pre-reset observation of every env (rows of finished
      envs are what SyncVectorEnv puts in info["final_observation"]); reward is float32 (the
      reference's float64 reward buffer holds float32 values, base.py:152 casts back).
    reset_states injects the state a finishing env restarts from (parity mode); without it
    the kernel draws from the env's reset distribution with a counter-based Philox stream.
    """

    def __init__(self, env_id: str, num_envs: int, seed: int = 0, device=None):
        if env_id not in N.ENV_IDS:
            raise ValueError(f"Unknown custom env: {env_id}")
        self.env_id = env_id
        self.num_envs = int(num_envs)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.info = self._env_info(env_id)
        D, A = self.info.obs_dim, self.info.act_dim
        self.obs_dim, self.act_dim = D, A
        self.state_dim, self.xstate_dim = self.info.state_dim, self.info.xstate_dim
        self.reset_dim = self.info.reset_dim
        self.single_observation_space = Box(list(self.info.obs_low)[:D], list(self.info.obs_high)[:D])
        self.single_action_space = Box(list(self.info.act_low)[:A], list(self.info.act_high)[:A])
        self.observation_space = Box(np.tile(self.single_observation_space.low, (self.num_envs, 1)),
                                     np.tile(self.single_observation_space.high, (self.num_envs, 1)))
        self.action_space = Box(np.tile(self.single_action_space.low, (self.num_envs, 1)),
                                np.tile(self.single_action_space.high, (self.num_envs, 1)))
        self._device = device
        self._h = None

    @staticmethod
    def _env_info(env_id):
        return N.env_info(env_id)

    # ------------------------------------------------------------------ device handle
    @property
    def device(self):
        if self._device is None:
            self._device = torch.device("cuda", torch.cuda.current_device())
        return torch.device(self._device)

    def handle(self):
        if self._h is None:
            if not torch.cuda.is_available():
                raise RuntimeError("HipVectorEnv needs a HIP device (MI355X); no CPU fallback exists")
            import ctypes
            h = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                N.check(N.lib().mh_env_create(N.ENV_IDS[self.env_id], self.num_envs, self.seed, ctypes.byref(h)),
                        "mh_env_create")
            self._h = h
        return self._h

    def close(self):
        if self._h is not None:
            h, self._h = self._h, None
            _destroy_when_safe(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _f32(self, x, cols, name):
        if x is None:
            return None
        t = torch.as_tensor(x, dtype=torch.float32, device=self.device).contiguous()
        N.require_device(t, name, torch.float32, self.num_envs * cols, self.device)
        return t

    # ------------------------------------------------------------------ gym-like API
    def reset(self, seed=None, options=None, reset_states=None):
        h = self.handle()
        obs = torch.empty(self.num_envs, self.obs_dim, device=self.device)
        rs = self._f32(reset_states, self.reset_dim, "reset_states")
        N.check(N.lib().mh_env_reset(h, N.ptr(rs), N.ptr(obs), N.stream_of(self.device)), "mh_env_reset")
        return obs, {}

    def step(self, actions, reset_states=None):
        h = self.handle()
        act = self._f32(actions, self.act_dim, "actions")
        rs = self._f32(reset_states, self.reset_dim, "reset_states")
        E, D, dev = self.num_envs, self.obs_dim, self.device
        next_obs = torch.empty(E, D, device=dev)
        real = torch.empty(E, D, device=dev)
        rew = torch.empty(E, device=dev)
        term = torch.empty(E, dtype=torch.uint8, device=dev)
        trunc = torch.empty(E, dtype=torch.uint8, device=dev)
        N.check(N.lib().mh_env_step(h, N.ptr(act), N.ptr(rs), N.ptr(next_obs), N.ptr(real), N.ptr(rew), N.ptr(term),
                                    N.ptr(trunc), N.stream_of(dev)), "mh_env_step")
        return next_obs, rew, term.bool(), trunc.bool(), {"final_observation": real}

    # ------------------------------------------------------------------ state access
    def get_state(self):
        h = self.handle()
        dev = self.device
        st = torch.empty(self.num_envs, self.state_dim, device=dev)
        xs = torch.empty(self.num_envs, max(self.xstate_dim, 1), dtype=torch.float64, device=dev)
        steps = torch.empty(self.num_envs, dtype=torch.int32, device=dev)
        N.check(N.lib().mh_env_get_state(h, N.ptr(st), N.ptr(xs) if self.xstate_dim else None, N.ptr(steps),
                                         N.stream_of(dev)), "mh_env_get_state")
        return st, (xs if self.xstate_dim else None), steps

    def get_counters(self):
        """The per-env Philox counters [E] (int64 copy of the uint32 words, mh_env_get_counters):
        with `seed` they key every in-kernel draw (oracle/rng.py replays them)."""
        c = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        N.check(N.lib().mh_env_get_counters(self.handle(), N.ptr(c), N.stream_of(self.device)), "mh_env_get_counters")
        return c.to(torch.int64) & 0xFFFFFFFF

    def set_counters(self, counters):
        c = torch.as_tensor(counters, device=self.device).to(torch.int64).to(torch.int32).contiguous()
        N.require_device(c, "counters", torch.int32, self.num_envs, self.device)
        N.check(N.lib().mh_env_set_counters(self.handle(), N.ptr(c), N.stream_of(self.device)), "mh_env_set_counters")

    def set_state(self, state, xstate=None, steps=None):
        h = self.handle()
        dev = self.device
        st = self._f32(state, self.state_dim, "state")
        xs = None
        if xstate is not None and self.xstate_dim:
            xs = torch.as_tensor(xstate, dtype=torch.float64, device=dev).contiguous()
            N.require_device(xs, "xstate", torch.float64, self.num_envs * self.xstate_dim, dev)
        sp = None
        if steps is not None:
            sp = torch.as_tensor(steps, dtype=torch.int32, device=dev).contiguous()
            N.require_device(sp, "steps", torch.int32, self.num_envs, dev)
        N.check(N.lib().mh_env_set_state(h, N.ptr(st), N.ptr(xs), N.ptr(sp), N.stream_of(dev)), "mh_env_set_state")


# Handles released while a HIP graph is being captured (a finaliser run by the garbage collector
# inside someone else's capture): hipFree is illegal there, so their destruction waits for the
# next release outside a capture.
_PENDING = []


def _destroy_when_safe(h):
    _PENDING.append(h)
    drain_pending_handles()


def drain_pending_handles():
    """Destroy the handles whose release was deferred by a capture, unless one is in progress now
    (called by every release, after the samplers' graph captures and at interpreter exit)."""
    if not _PENDING:
        return
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return
    while _PENDING:
        N.lib().mh_env_destroy(_PENDING.pop())


atexit.register(drain_pending_handles)


def make_env(env_id, seed, idx, capture_video=False, run_name=""):
    """Thunk factory with the RL/env/make_env.py:10-41 signature; builds a 1-env batch."""
    def thunk():
        return HipVectorEnv(env_id, 1, seed=seed)
    return thunk
