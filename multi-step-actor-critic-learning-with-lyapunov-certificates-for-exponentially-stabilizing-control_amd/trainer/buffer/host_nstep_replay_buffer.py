"""Host n-step replay buffer for the CPU deployment (BASELINE.json config 1): the reference's
NstepReplayBuffer (RL/trainer/buffer/nstep_replay_buffer.py:20-150) — seven float32 arrays
[max_size, n_step, ...], FIFO ptr/size, `np.random.randint(0, size, B)` uniform draws, batches
as float32 CPU tensors. add_batch() writes a HostWindowBatch's stacked arrays in one slice
assignment per field (with wrap) instead of one store() per window.
"""
from __future__ import annotations

import numpy as np
import torch

KEYS = ("obs", "act", "rew", "cost", "obs2", "done", "logp")


class HostWindowBatch:
    """Windows of one sample() call: a sequence of (obs, act, rew, cost, obs2, done, logp)
    tuples (the reference's nStepExperience field order) over stacked [W, n, ...] arrays."""

    def __init__(self, arrays):
        self.arrays = arrays

    def __len__(self):
        return int(self.arrays["obs"].shape[0])

    def __getitem__(self, i):
        return tuple(self.arrays[k][i] for k in KEYS)

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class HostNstepReplayBuffer:
    def __init__(self, **kwargs):
        self.obsv_dim = int(kwargs["obs_dim"])
        self.act_dim = int(kwargs["act_dim"])
        self.max_size = int(kwargs["buffer_max_size"])
        self.n_step = int(kwargs["n_step"])
        self.device = torch.device("cpu")
        M, n, D, A = self.max_size, self.n_step, self.obsv_dim, self.act_dim
        z = lambda *s: np.zeros(s, dtype=np.float32)  # noqa: E731
        self.n_step_buf = {"obs": z(M, n, D), "act": z(M, n, A), "rew": z(M, n), "cost": z(M, n),
                           "obs2": z(M, n, D), "done": z(M, n), "logp": z(M, n)}
        self.ptr, self.size = 0, 0

    def __len__(self):
        return self.size

    def __get_RAM__(self):
        """MB held by the valid windows (nstep_replay_buffer.py:76-88)."""
        if self.size == 0:
            return 0.0
        per_row = sum(v[0].nbytes for v in self.n_step_buf.values())
        return round(per_row * self.size / (1024 * 1024), 2)

    def store(self, obs, act, rew, cost, next_obs, done, logp):
        for k, v in zip(KEYS, (obs, act, rew, cost, next_obs, done, logp)):
            self.n_step_buf[k][self.ptr] = v
        self.ptr = (self.ptr + 1) % self.max_size
        self.size = min(self.size + 1, self.max_size)

    def add_batch(self, samples):
        if not isinstance(samples, HostWindowBatch):
            for s in samples:
                self.store(*s)
            return
        W = len(samples)
        if W == 0:
            return
        keep = min(W, self.max_size)  # FIFO: a batch larger than the store keeps its newest rows
        dst = (self.ptr + (W - keep) + np.arange(keep)) % self.max_size
        for k in KEYS:
            self.n_step_buf[k][dst] = samples.arrays[k][W - keep:]
        self.ptr = (self.ptr + W) % self.max_size
        self.size = min(self.size + W, self.max_size)

    def sample_batch(self, batch_size: int) -> dict:
        idx = np.random.randint(0, self.size, size=batch_size)
        return {k: torch.as_tensor(v[idx], dtype=torch.float32) for k, v in self.n_step_buf.items()}
