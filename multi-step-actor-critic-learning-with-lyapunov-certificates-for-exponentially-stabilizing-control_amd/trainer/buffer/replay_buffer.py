"""HBM-resident 1-step replay buffer (drop-in for RL/trainer/buffer/replay_buffer.py:34-137).

Storage is the reference's dict of seven float32 arrays `[max_size, ...]` (`self.buf`), held on
the device and written in place by the rollout kernel's emission stage: a 1-step transition is
an n-step window with n = 1, so the same device store, FIFO cursor and gather kernels serve it
(the arrays are allocated `[max_size, 1, ...]`; `buf` exposes them as `[max_size, ...]` views).

API: add_batch(samples), sample_batch(batch_size) -> {obs[B, D], act[B, A], rew[B], cost[B],
obs2[B, D], done[B], logp[B]} float32 device tensors (replay_buffer.py:122-137), store(...),
.size, __len__, __get_RAM__(). The uniform index draw of `np.random.randint(0, size, B)`
(:131) is a device Philox draw. Unlike the reference (whose __get_RAM__ reads a
`n_step_buf` attribute the class never defines, replay_buffer.py:66-80), __get_RAM__ works.
"""
from __future__ import annotations

from .device_nstep_replay_buffer import DeviceNstepReplayBuffer

__all__ = ["ReplayBuffer"]


class ReplayBuffer(DeviceNstepReplayBuffer):
    graph_draw = False  # 1-step transitions: the trainers draw and gather eagerly

    def __init__(self, **kwargs):
        kw = dict(kwargs)
        kw["n_step"] = 1
        super().__init__(**kw)
        M = self.max_size
        self.buf = {k: v.view(M, *v.shape[2:]) for k, v in self.n_step_buf.items()}

    def gather(self, idx):
        out = super().gather(idx)
        B = int(idx.numel())
        return {k: v.view(B, *v.shape[2:]) for k, v in out.items()}
