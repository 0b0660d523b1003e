"""Prioritized n-step replay over the device window store (NEW: the reference trainer calls
`buffer.update_batch(idx, new_priority)` when buffer_name == "prioritized_replay_buffer",
RL/trainer/nstep_off_serial_trainer.py:30,93-95, and the README advertises PER, but the
reference ships no such buffer — so this component is parity-unpinned by construction).

Proportional prioritisation (Schaul et al., 2016): P(i) ~ p_i, p_i = (|delta_i| + eps)^alpha
with delta_i the window's mean |TD| from the fused Q-target kernel; new windows enter with the
running max priority; importance weights w_i = (N P(i))^-beta / max_batch w. The float64
sum-tree lives in HBM and is rebuilt by blocked kernels (csrc/per.hip).
"""
import torch

from ... import _native as N
from .device_nstep_replay_buffer import DeviceNstepReplayBuffer


class PrioritizedReplayBuffer(DeviceNstepReplayBuffer):
    graph_draw = False  # the proportional draw (host draw counter) and the tree stay outside the graph

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.alpha = float(kwargs.get("per_alpha", 0.6))
        self.beta = float(kwargs.get("per_beta", 0.4))
        self.eps = float(kwargs.get("per_eps", 1e-6))
        pow2 = 1
        while pow2 < self.max_size:
            pow2 <<= 1
        self.pow2 = pow2
        self.tree = torch.zeros(2 * pow2, dtype=torch.float64, device=self.device)
        self.max_prio = torch.ones(1, dtype=torch.float64, device=self.device)
        self._seen = self.cursor.clone()
        self._per_draws = 0

    def _on_windows_added(self):
        N.check(N.lib().mh_per_set_new(N.ptr(self.tree), self.pow2, N.ptr(self._seen), N.ptr(self.cursor),
                                       self.max_size, N.ptr(self.max_prio), N.stream_of(self.device)), "mh_per_set_new")
        self._seen.copy_(self.cursor)

    def sample_batch(self, batch_size: int, out=None, joint=False) -> dict:
        """Proportional draw + IS weights, then the window gather (into `out` when it fits,
        DeviceNstepReplayBuffer.gather; its "idx" / "weight" too; joint: the update's joint layouts)."""
        fits = self._fits(out, batch_size)
        idx = out.get("idx") if fits else None
        w = out.get("weight") if fits else None
        if idx is None or idx.shape != (batch_size,) or idx.dtype != torch.int64:
            idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        if w is None or w.shape != (batch_size,) or w.dtype != torch.float32:
            w = torch.empty(batch_size, dtype=torch.float32, device=self.device)
        N.check(N.lib().mh_per_sample(N.ptr(self.tree), self.pow2, N.ptr(self.cursor), self.seed, self._per_draws,
                                      batch_size, self.beta, N.ptr(idx), N.ptr(w), N.stream_of(self.device)),
                "mh_per_sample")
        self._per_draws += 1
        out = self.gather(idx, out, joint)
        out["idx"] = idx
        out["weight"] = w
        return out

    def update_batch(self, idx, priority):
        idx = torch.as_tensor(idx, dtype=torch.int64, device=self.device).contiguous()
        pr = torch.as_tensor(priority, dtype=torch.float32, device=self.device).contiguous()
        N.check(N.lib().mh_per_update(N.ptr(self.tree), self.pow2, N.ptr(idx), N.ptr(pr), int(idx.numel()), self.alpha,
                                      self.eps, N.ptr(self.max_prio), N.stream_of(self.device)), "mh_per_update")
