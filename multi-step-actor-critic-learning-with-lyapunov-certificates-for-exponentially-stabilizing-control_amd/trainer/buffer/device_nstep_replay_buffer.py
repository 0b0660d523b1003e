"""HBM-resident n-step replay buffer (drop-in for RL/trainer/buffer/nstep_replay_buffer.py).

Storage is the reference's dict of seven float32 arrays `[max_size, n_step, ...]`, held as
device tensors and written directly by the rollout kernel's window-emission stage (the HIP
sampler binds to this store on the first add_batch, after which add_batch is bookkeeping only:
no host copy, no per-window Python loop). The FIFO cursor {ptr, size, total, last} lives on
the device so the whole rollout can run without a host sync.

API: add_batch(samples), sample_batch(batch_size) -> dict of [B, n, ...] tensors, .size,
__len__, __get_RAM__(), store(...) (single window, host path). The uniform index draw of
`np.random.randint(0, size, B)` (nstep_replay_buffer.py:138) is a device Philox draw.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ... import _native as N

KEYS = ("obs", "act", "rew", "cost", "obs2", "done", "logp")


class DeviceWindowBatch:
    """What the HIP sampler's sample() returns: windows already emitted into `store_owner`
    (when bound) or into the sampler's staging store. `count` is a device int64 scalar, or None
    with `count_fn` given: the count is then read on demand (the fused horizon's header holds it
    until the sampler's next horizon, which first calls resolve() on a batch still unresolved)."""

    def __init__(self, sampler, store_owner, count, first_total=None, count_fn=None):
        self.sampler = sampler
        self.store_owner = store_owner
        self.count = count
        self.first_total = first_total
        self._count_fn = count_fn

    def resolve(self):
        if self.count is None:
            self.count = self._count_fn()
            self._count_fn = None
        return self.count

    def __len__(self):
        return int(self.resolve().item())


class DeviceNstepReplayBuffer:
    def __init__(self, **kwargs):
        self.obsv_dim = int(kwargs["obs_dim"])
        self.act_dim = int(kwargs["act_dim"])
        self.max_size = int(kwargs["buffer_max_size"])
        self.n_step = int(kwargs["n_step"])
        dev = kwargs.get("device")
        self.device = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
        self.seed = int(kwargs.get("buffer_seed", kwargs.get("seed", 0) or 0)) & ((1 << 63) - 1)
        M, n, D, A = self.max_size, self.n_step, self.obsv_dim, self.act_dim
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        self.n_step_buf = {"obs": z(M, n, D), "act": z(M, n, A), "rew": z(M, n), "cost": z(M, n),
                           "obs2": z(M, n, D), "done": z(M, n), "logp": z(M, n)}
        self.cursor = torch.zeros(4, dtype=torch.int64, device=self.device)  # ptr, size, total, last
        self.ws = N.WindowStore(*[ctypes.c_void_p(self.n_step_buf[k].data_ptr()) for k in KEYS],
                                M, ctypes.c_void_p(self.cursor.data_ptr()))
        # the replay draw counter lives on the device ([counter, arrival ticket]): a draw can then
        # be captured in the update's graph and replayed (mh_replay_draw_gather)
        self._draw_state = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._idx = None

    graph_draw = True  # sample_batch(B, out=...) is one capturable launch (the trainer's drawn update)

    @property
    def draws(self):
        """Replay draws made so far (reads the device counter: a host sync)."""
        return int(self._draw_state[0].item())

    # ------------------------------------------------------------------ size / memory
    @property
    def ptr(self):
        return int(self.cursor[0].item())

    @property
    def size(self):
        return int(self.cursor[1].item())

    def __len__(self):
        return self.size

    def __get_RAM__(self):
        """MB held by valid windows (nstep_replay_buffer.py:76-88 semantics)."""
        size = self.size
        if size == 0:
            return 0.0
        per_row = sum(v[0].numel() * v.element_size() for v in self.n_step_buf.values())
        return round(per_row * size / (1024 * 1024), 2)

    # ------------------------------------------------------------------ writes
    def store(self, obs, act, rew, cost, next_obs, done, logp):
        """Single window from host data (reference store(), :91-119) — compatibility path."""
        p = self.ptr
        for k, v in zip(KEYS, (obs, act, rew, cost, next_obs, done, logp)):
            self.n_step_buf[k][p].copy_(torch.as_tensor(np.asarray(v, np.float32)))
        c = self.cursor.cpu()
        c[0] = (p + 1) % self.max_size
        c[1] = min(int(c[1]) + 1, self.max_size)
        c[2] += 1
        c[3] = 1
        self.cursor.copy_(c)

    def add_batch(self, samples):
        if isinstance(samples, DeviceWindowBatch):
            if samples.store_owner is self:
                self._on_windows_added()
                return
            samples.sampler.bind_store(self)
            self._absorb_staged(samples)
            self._on_windows_added()
            return
        for s in samples:
            self.store(*s)
        self._on_windows_added()

    def _absorb_staged(self, batch):
        """First batch of an unbound sampler: copy its staged windows in emission order."""
        staged = batch.store_owner
        cnt = int(staged.cursor[1].item())
        if cnt == 0:
            return
        keep = min(cnt, self.max_size)  # FIFO: only the newest max_size windows survive
        src = torch.arange(cnt - keep, cnt, device=self.device)
        c = self.cursor.cpu()
        ptr = int(c[0]) + (cnt - keep)
        dst = (ptr + torch.arange(keep, device=self.device)) % self.max_size
        for k in KEYS:
            self.n_step_buf[k][dst] = staged.n_step_buf[k][src]
        c[0] = (int(c[0]) + cnt) % self.max_size
        c[1] = min(int(c[1]) + cnt, self.max_size)
        c[2] += cnt
        c[3] = cnt
        self.cursor.copy_(c)

    def _on_windows_added(self):
        pass

    # ------------------------------------------------------------------ reads
    def sample_indices(self, batch_size):
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        N.check(N.lib().mh_replay_sample_indices_dev(ctypes.byref(self.ws), self.seed, N.ptr(self._draw_state),
                                                     batch_size, N.ptr(idx), N.stream_of(self.device)),
                "mh_replay_sample_indices_dev")
        return idx

    def _fits(self, out, B):
        """`out` can receive a gather of B windows: every key, float32, contiguous, this device,
        the batch's shapes."""
        if out is None:
            return False
        n, D, A = self.n_step, self.obsv_dim, self.act_dim
        shapes = {"obs": (B, n, D), "act": (B, n, A), "rew": (B, n), "cost": (B, n), "obs2": (B, n, D),
                  "done": (B, n), "logp": (B, n)}
        for k, shp in shapes.items():
            t = out.get(k)
            if (t is None or tuple(t.shape) != shp or t.dtype != torch.float32 or t.device != self.device
                    or not t.is_contiguous()):
                return False
        return True

    def _joint_shapes(self, B):
        n, D, A = self.n_step, self.obsv_dim, self.act_dim
        return {"obs_act": (B, n, D + A), "v_in": (B + B * n, D)}

    def gather(self, idx, out=None, joint=False):
        """The windows at `idx` as [B, n, ...] tensors; into `out` (a dict of such tensors, e.g.
        the update graph's static inputs, so the replayed update needs no copy) when it fits,
        otherwise into fresh tensors. joint (or `out` holding them): also the update's joint
        layouts "obs_act" = [obs | act] and "v_in" = [obs[:, 0]; obs2 rows] (mh_replay_gather_joint)."""
        B = int(idx.numel())
        dst = self._destinations(B, out, joint)
        n, D, A = self.n_step, self.obsv_dim, self.act_dim
        idx = idx.to(self.device, torch.int64).contiguous()
        N.check(N.lib().mh_replay_gather_joint(ctypes.byref(self.ws), n, D, A, N.ptr(idx), B,
                                               *[N.ptr(dst[k]) for k in KEYS], N.ptr(dst.get("obs_act")),
                                               N.ptr(dst.get("v_in")), N.stream_of(self.device)),
                "mh_replay_gather_joint")
        return dst

    def _destinations(self, B, out, joint):
        """The gather's destination tensors: `out`'s when it fits, fresh ones otherwise."""
        n, D, A = self.n_step, self.obsv_dim, self.act_dim
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        js = self._joint_shapes(B)
        if self._fits(out, B):
            dst = {k: out[k] for k in KEYS}
            for k, shp in js.items():
                t = out.get(k)
                if (t is not None and tuple(t.shape) == shp and t.dtype == torch.float32 and t.device == self.device
                        and t.is_contiguous()):
                    dst[k] = t
        else:
            dst = {"obs": e(B, n, D), "act": e(B, n, A), "rew": e(B, n), "cost": e(B, n), "obs2": e(B, n, D),
                   "done": e(B, n), "logp": e(B, n)}
            if joint:
                dst.update({k: e(*shp) for k, shp in js.items()})
        return dst

    def sample_batch(self, batch_size: int, out=None, joint=False) -> dict:
        """nstep_replay_buffer.py:136-148. `out` (optional): destination tensors (gather); joint:
        add the update's joint layouts (gather)."""
        if out is None and not joint:
            return self.gather(self.sample_indices(batch_size))  # (the 1-step ReplayBuffer's gather takes idx only)
        # the draw and the gather in one launch (the draw counter advanced on the device)
        dst = self._destinations(batch_size, out, joint)
        n, D, A = self.n_step, self.obsv_dim, self.act_dim
        N.check(N.lib().mh_replay_draw_gather(ctypes.byref(self.ws), n, D, A, self.seed, N.ptr(self._draw_state),
                                              batch_size, None, *[N.ptr(dst[k]) for k in KEYS],
                                              N.ptr(dst.get("obs_act")), N.ptr(dst.get("v_in")),
                                              N.stream_of(self.device)), "mh_replay_draw_gather")
        return dst
