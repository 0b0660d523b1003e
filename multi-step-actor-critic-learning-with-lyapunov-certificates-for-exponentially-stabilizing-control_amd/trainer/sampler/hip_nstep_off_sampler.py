"""Device n-step off-policy sampler (drop-in for RL/trainer/sampler/nstep_off_sampler.py +
BaseSampler._n_step, RL/trainer/sampler/base.py:118-222).

Per lockstep step: the policy MLP forward on the [E, obs_dim] observation tensor — for the
reference's default StochaPolicy shape [D -> 256 -> 256 -> 2A] one fused f32-MFMA kernel
(csrc/policy_mlp.hip, parameters packed from the nn.Module once per sample()), otherwise the
PyTorch module (hipBLASLt GEMMs with the ReLU in the epilogue); the head's clamp(log_std).exp()
is folded into the rollout kernel either way — then ONE fused gfx950 kernel samples
the TanhGauss action, clips it, integrates the env, computes reward/cost, autoresets, pushes
the n-step deque and flags full windows; a scan and an emission kernel write every full window
straight into the bound replay store (env-index order, base.py:178-213).
`sample()` runs `horizon = sample_batch_size` such steps; after the first (eager) call the
whole horizon loop is captured once into a HIP graph and replayed (no per-launch host cost).
It returns a DeviceWindowBatch; the buffer's add_batch() binds the store so subsequent windows
are emitted in place (no host round trip, no per-window Python).
"""
from __future__ import annotations

import ctypes
import time
import weakref

import torch
import torch.nn as nn

from ... import _native as N
from ...utils import dist as D
from ...create_pkg.create_alg import create_approx_contrainer
from ...env.hip_vector_env import HipVectorEnv, drain_pending_handles
from ...utils.act_distribution_cls import TanhGaussDistribution
from ...utils.tensorboard_setup import tb_tags
from ..buffer.device_nstep_replay_buffer import DeviceNstepReplayBuffer, DeviceWindowBatch


class HipNstepOffSampler:
    def __init__(self, **kwargs):
        self.env_id = kwargs["env_name"]
        self.num_envs = int(kwargs["env_num"])
        dev = kwargs.get("device")
        self.device = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
        self.envs = HipVectorEnv(self.env_id, self.num_envs, seed=int(kwargs.get("env_seed") or 0) +
                                 int(kwargs.get("sampler_seed_offset", 0)), device=self.device)
        self.obs_dim = self.envs.single_observation_space.shape
        self.act_dim = self.envs.single_action_space.shape
        self.networks = create_approx_contrainer(**kwargs).to(self.device)
        self.sample_batch_size = int(kwargs["sample_batch_size"]) * self.num_envs
        self.action_type = kwargs["action_type"]
        self.reward_scale = float(kwargs["reward_scale"])
        self.cost_scale = float(kwargs["cost_scale"])
        self.noise_params = kwargs.get("noise_params")
        if self.action_type != "continu":
            raise RuntimeError("Only continuous action space is supported!")
        self.target_value = kwargs.get("target_value", 0.0)
        self.total_sample_number = 0
        self.horizon = self.sample_batch_size // self.num_envs
        self.n_step = int(kwargs.get("n_step", 1))
        self.gamma = kwargs.get("gamma", 0.99)
        self.td_lambda = kwargs.get("retrace_lambda", 0.95)
        self.sync_timing = bool(kwargs.get("sampler_sync_timing", True))
        self.use_graph = bool(kwargs.get("sampler_use_graph", True))
        # emission of each lockstep's windows deferred into the next lockstep's kernel
        # (mh_rollout_step_deferred); False: a separate emission launch after every step
        self.deferred_emission = bool(kwargs.get("sampler_deferred_emission", True))
        self.use_fused_policy = bool(kwargs.get("sampler_fused_policy", True))
        # the whole horizon as one persistent kernel (mh_sample_horizon) when the fused policy
        # applies; False: per lockstep, policy kernel + lockstep kernel (the same values)
        self.fused_horizon = bool(kwargs.get("sampler_fused_horizon", True)) and self.use_fused_policy
        self._packed = None
        self._h = self.envs.handle()
        N.check(N.lib().mh_nstep_attach(self._h, self.n_step, self.reward_scale, self.cost_scale), "mh_nstep_attach")
        if self.fused_horizon:
            # rings long enough that a horizon's windows are intact until its emission launch
            rc = N.lib().mh_nstep_reserve(self._h, self.n_step + self.horizon - 1)
            if rc != 0:
                self.fused_horizon = False
        if self.fused_horizon:
            # bound of the fused kernel's policy-wave waits; a wait that gives up is counted in the
            # handle's cumulative error word, which check_errors() reads (no hot-path cost)
            limit = int(kwargs.get("sampler_spin_limit", 0) or 0)  # test hook: forces the timeout path
            N.check(N.lib().mh_sample_horizon_set_spin_limit(self._h, limit), "mh_sample_horizon_set_spin_limit")
        # GaussNoise (explore_noise.py:3-9; base.py:83-88,136-137): ONE scalar
        # np.random.normal(mean, std) per lockstep step, added to every action before the clip.
        # Drawn on the device into a 1-float tensor (capturable), read by the rollout kernel.
        # One scalar per lockstep: the horizon's H values are drawn at its start into a device
        # tensor (capturable); lockstep t reads element t.
        self._noise = None
        if self.noise_params is not None:
            self._noise_mean = float(self.noise_params["mean"])
            self._noise_std = float(self.noise_params["std"])
            self._noise = torch.zeros(max(1, self.horizon), dtype=torch.float32, device=self.device)
            N.check(N.lib().mh_env_set_action_noise(self._h, N.ptr(self._noise)), "mh_env_set_action_noise")
        self.obs, _ = self.envs.reset(seed=None)
        self._bound = None
        self._staging = None
        self._graph = None
        self._graph_key = None
        self._eager_calls = 0
        self._last_batch = None  # weakref to the last fused horizon's batch (its count unread)

    # ------------------------------------------------------------------ reference API
    def get_total_sample_num(self) -> int:
        return self.total_sample_number

    def get_total_sample_number(self) -> int:
        return self.total_sample_number

    def load_state_dict(self, state_dict):
        self.networks.load_state_dict(state_dict)

    def bind_store(self, buffer: DeviceNstepReplayBuffer):
        """Emit windows directly into `buffer` from now on."""
        if buffer.n_step != self.n_step or buffer.obsv_dim != self.envs.obs_dim or buffer.act_dim != self.envs.act_dim:
            raise ValueError("replay buffer shape does not match the sampler (n_step / obs_dim / act_dim)")
        if buffer.device != self.device:
            raise ValueError("replay buffer lives on a different device than the sampler")
        self._bound = buffer

    def _target(self):
        if self._bound is not None:
            return self._bound
        if self._staging is None:
            self._staging = DeviceNstepReplayBuffer(obs_dim=self.envs.obs_dim, act_dim=self.envs.act_dim,
                                                    buffer_max_size=max(1, self.horizon * self.num_envs),
                                                    n_step=self.n_step, device=self.device)
        self._staging.cursor.zero_()
        return self._staging

    # ------------------------------------------------------------------ policy head
    def _fused_layers(self):
        """The three nn.Linear of a StochaPolicy [D -> 256 -> ReLU -> 256 -> ReLU -> 2A] MLP
        (mlp.py:18-30 layout), or None when the policy is another shape (PyTorch path)."""
        if not self.use_fused_policy:
            return None
        pol = self.networks.policy
        seq = getattr(pol, "policy", None)
        if getattr(pol, "action_distribution_cls", None) is not TanhGaussDistribution or not isinstance(seq, nn.Sequential):
            return None
        mods = list(seq)
        if len(mods) != 6:
            return None
        l1, a1, l2, a2, l3, a3 = mods
        if not (isinstance(l1, nn.Linear) and isinstance(l2, nn.Linear) and isinstance(l3, nn.Linear)
                and isinstance(a1, nn.ReLU) and isinstance(a2, nn.ReLU) and isinstance(a3, nn.Identity)):
            return None
        D = self.envs.obs_dim
        if (l1.in_features != D or l1.out_features != 256 or l2.in_features != 256 or l2.out_features != 256
                or l3.in_features != 256 or l3.out_features != 2 * self.envs.act_dim or D > 16):
            return None
        if any(p.device != self.device or p.dtype != torch.float32 for p in seq.parameters()):
            return None
        return l1, l2, l3

    def _pack_policy(self):
        """Pack the policy's current parameters into the fused kernel's fragment order (once per
        sample(); captured into the sampler graph). Returns False for the PyTorch path."""
        layers = self._fused_layers()
        if layers is None:
            return False
        D, N3 = self.envs.obs_dim, 2 * self.envs.act_dim
        if self._packed is None:
            n = ctypes.c_int64()
            N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "mh_policy_packed_size")
            self._packed = torch.empty(n.value, dtype=torch.float32, device=self.device)
        l1, l2, l3 = layers
        ps = [t.detach().contiguous() for t in (l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)]
        N.check(N.lib().mh_policy_pack(*[N.ptr(t) for t in ps], D, 256, 256, N3, N.ptr(self._packed),
                                       N.stream_of(self.device)), "mh_policy_pack")
        return True

    def _policy_fused(self):
        logits = torch.empty(self.num_envs, 2 * self.envs.act_dim, dtype=torch.float32, device=self.device)
        N.check(N.lib().mh_policy_forward(N.ptr(self._packed), N.ptr(self.obs), self.num_envs, self.envs.obs_dim,
                                          2 * self.envs.act_dim, N.ptr(logits), N.stream_of(self.device)),
                "mh_policy_forward")
        return logits, True

    def _policy_raw(self):
        """StochaPolicy.forward (mlp.py:132-136) up to the head: returns (logits, raw) where raw
        means the second half is log_std before clamp/exp (the kernel finishes it)."""
        pol = self.networks.policy
        seq = getattr(pol, "policy", None)
        if getattr(pol, "action_distribution_cls", None) is not TanhGaussDistribution:
            raise NotImplementedError("the HIP sampler samples TanhGaussDistribution policies")
        if not isinstance(seq, nn.Sequential):
            return pol(self.obs).contiguous(), False
        h = self.obs
        mods = list(seq)
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, nn.Linear) and isinstance(nxt, nn.ReLU):
                h = torch._addmm_activation(m.bias, h, m.weight.t())  # GEMM + bias + ReLU epilogue
                i += 2
            elif isinstance(m, nn.Linear) and (nxt is None or isinstance(nxt, nn.Identity)):
                h = torch.addmm(m.bias, h, m.weight.t())
                i += 2
            else:
                h = m(h)
                i += 1
        return h.contiguous(), True

    # ------------------------------------------------------------------ one lockstep step
    def _lockstep(self, store, logits=None, act_in=None, logp_in=None, reset_states=None, act_out=None,
                  logp_out=None, deferred=False):
        """One lockstep step; `deferred`: its windows are emitted by the next deferred step (by
        emitter waves running beside that step's env waves) or by _flush (mh_rollout_flush)."""
        fn = N.lib().mh_rollout_step_deferred if (deferred and store is not None) else N.lib().mh_rollout_step
        N.check(fn(self._h, N.ptr(logits), N.ptr(act_in), N.ptr(logp_in), N.ptr(reset_states),
                   N.ptr(self.obs), ctypes.byref(store.ws) if store is not None else None,
                   N.ptr(act_out), N.ptr(logp_out), N.stream_of(self.device)),
                "mh_rollout_step")

    def _flush(self):
        N.check(N.lib().mh_rollout_flush(self._h, N.stream_of(self.device)), "mh_rollout_flush")

    def _draw_noise(self):
        if self._noise is not None:
            self._noise.normal_(self._noise_mean, self._noise_std)

    def _noise_at(self, t):
        if self._noise is not None:
            N.check(N.lib().mh_env_set_action_noise(self._h, N.ptr(self._noise[t:t + 1])), "mh_env_set_action_noise")

    def _policy_step(self, store, fused=False, act_out=None, logp_out=None, t=0):
        self._noise_at(t)
        logits, raw = self._policy_fused() if fused else self._policy_raw()
        pol = self.networks.policy
        N.check(N.lib().mh_nstep_set_log_std_clamp(self._h, int(raw), float(getattr(pol, "min_log_std", -20.0)),
                                                   float(getattr(pol, "max_log_std", 1.0))), "log_std clamp")
        self._lockstep(store, logits=logits, deferred=self.deferred_emission, act_out=act_out, logp_out=logp_out)
        return logits

    def _fused_horizon_ok(self, fused):
        return fused and self.fused_horizon and self.envs.obs_dim <= 15

    def _horizon(self, store, act_out=None, logp_out=None, pack=True):
        # pack=False (a trainer step graph whose caller knows the packed copy is current): the
        # packed parameters of the last pack are used as they are
        fused = self._pack_policy() if (pack or self._packed is None) else self._fused_layers() is not None
        self._draw_noise()
        if self._fused_horizon_ok(fused):
            # policy -> sample -> env step -> ring push for every lockstep in ONE persistent
            # kernel, then one launch emits the horizon's windows (csrc/sample_fused.hip)
            pol = self.networks.policy
            N.check(N.lib().mh_nstep_set_log_std_clamp(self._h, 1, float(getattr(pol, "min_log_std", -20.0)),
                                                       float(getattr(pol, "max_log_std", 1.0))), "log_std clamp")
            N.check(N.lib().mh_sample_horizon(self._h, N.ptr(self._packed), self.envs.obs_dim, 2 * self.envs.act_dim,
                                              N.ptr(self.obs), self.horizon, ctypes.byref(store.ws), N.ptr(self._noise),
                                              N.ptr(act_out), N.ptr(logp_out), N.stream_of(self.device)),
                    "mh_sample_horizon")
            return
        for t in range(self.horizon):
            self._policy_step(store, fused, t=t)
        self._flush()  # the last step's windows: the store is complete when sample() returns

    def _graph_for(self, store):
        key = (id(store), id(self.networks.policy), tuple(p.data_ptr() for p in self.networks.policy.parameters()),
               self.obs.data_ptr())
        if self._graph is None or self._graph_key != key:
            g = torch.cuda.CUDAGraph()
            with D.cuda_graph(g):
                self._horizon(store)
            self._graph, self._graph_key = g, key
            drain_pending_handles()  # env handles released by a finaliser during the capture
        return self._graph

    def _window_count(self):
        """The last horizon's window count (mh_sample_horizon_windows), a fresh device int64."""
        out = torch.empty(1, dtype=torch.int64, device=self.device)
        N.check(N.lib().mh_sample_horizon_windows(self._h, N.ptr(out), N.stream_of(self.device)),
                "mh_sample_horizon_windows")
        return out[0]

    def _sample(self):
        self._handle()
        store = self._target()
        fused_h = self._fused_horizon_ok(self._fused_layers() is not None)
        if fused_h:
            # the window count stays in the fused kernel's header until the next horizon: a batch
            # that still holds it unread copies it out first (no launches on the usual path, where
            # the trainer drops the batch right after add_batch)
            prev = self._last_batch() if self._last_batch is not None else None
            if prev is not None:
                prev.resolve()
            before = None
        else:
            before = store.cursor[2].clone()
        with torch.no_grad():
            if self.use_graph and self._eager_calls >= 1 and not getattr(self, "_timing", False):
                self._graph_for(store).replay()
            else:
                if getattr(self, "_timing", False):
                    # park the stream on a GPU spin while the host enqueues the whole horizon,
                    # so the per-kernel events bracket device time, not host launch latency
                    torch.cuda._sleep(int(getattr(self, "_timing_spin_cycles", 20_000_000)))
                self._horizon(store)
                self._eager_calls += 1
        if fused_h:
            batch = DeviceWindowBatch(self, store, None, count_fn=self._window_count)
            self._last_batch = weakref.ref(batch)
            return batch
        return DeviceWindowBatch(self, store, store.cursor[2] - before)

    def policy_version(self):
        """What the packed policy copy depends on besides the algorithm's policy-update count:
        (sum of the policy parameters' version counters, the writes through .data or raw pointers
        that those counters miss, this sampler's own invalidations). torch bumps a version counter
        on every in-place write through torch (load_state_dict, optimiser steps, manual edits) but
        NOT on writes through `p.data` or a kernel given the storage's pointer: such writers call
        utils.dist.parameters_written() (broadcast_module does), or the caller invalidate_policy_pack()."""
        return (sum(p._version for p in self.networks.policy.parameters()), D.param_epoch(),
                getattr(self, "_pack_epoch", 0))

    def invalidate_policy_pack(self):
        """Force the next graphed sample() to re-pack the policy (after writing its parameters in
        a way policy_version() cannot see)."""
        self._pack_epoch = getattr(self, "_pack_epoch", 0) + 1

    def step_graph_parts(self, pack=True):
        """The pieces of one graphed sample() for a trainer-level graph that also holds the update
        after it (NstepOffSerialTrainer._graph_step): (key, pre, body, post), or None while that
        does not apply (eager horizons still due, per-kernel timing, a synchronised sampler time,
        no fused horizon, or no bound store). key: what the capture depends on (as the sampler
        graph's key); pre(): host work before the replay; body(): the horizon, exactly what the
        sampler graph captures (pack=False: without the policy pack, for a caller that knows the
        packed copy matches the parameters); post(t0) -> sample()'s return value after the replay."""
        if (self._h is None or not self.use_graph or self._eager_calls < 1 or getattr(self, "_timing", False)
                or self.sync_timing or self._bound is None):
            return None
        if not self._fused_horizon_ok(self._fused_layers() is not None):
            return None
        store = self._bound
        key = (id(store), id(self.networks.policy), tuple(p.data_ptr() for p in self.networks.policy.parameters()),
               self.obs.data_ptr())

        def pre():
            # the previous horizon's window count lives in the fused kernel's header until this one
            prev = self._last_batch() if self._last_batch is not None else None
            if prev is not None:
                prev.resolve()
            self.total_sample_number += self.sample_batch_size

        def body():
            with torch.no_grad():
                self._horizon(store, pack=pack)

        def post(t0):
            batch = DeviceWindowBatch(self, store, None, count_fn=self._window_count)
            self._last_batch = weakref.ref(batch)
            return batch, {tb_tags["sampler_time"]: (time.perf_counter() - t0) * 1000}

        return key, pre, body, post

    def sample(self):
        """-> (DeviceWindowBatch, {sampler_time ms}) (base.py:308-323)."""
        self.total_sample_number += self.sample_batch_size
        t0 = time.perf_counter()
        data = self._sample()
        if self.sync_timing:
            torch.cuda.synchronize(self.device)
        tb = {tb_tags["sampler_time"]: (time.perf_counter() - t0) * 1000}
        return data, tb

    def check_errors(self):
        """Raise if a fused horizon's bounded policy-wave wait ever timed out (mh_sample_horizon_errors:
        the logits, and so the actions and windows, of that horizon are not trustworthy). The word
        is cumulative since the handle was created, so one read covers every horizon so far; it
        waits for the device only when called (the trainer calls it every log_save_interval
        iterations and at close())."""
        if self._h is None or not self.fused_horizon:
            return
        out = torch.zeros(1, dtype=torch.int64, device=self.device)
        N.check(N.lib().mh_sample_horizon_errors(self._h, N.ptr(out), N.stream_of(self.device)), "mh_sample_horizon_errors")
        n = int(out.item())
        if n:
            raise RuntimeError(f"fused horizon sampler: {n} policy-wave wait(s) timed out (mh_sample_horizon_errors); "
                               "the sampled actions and replay windows since then are corrupt")

    def close(self):
        """Release the sampler's device resources now: its captured horizon graph, the packed
        policy, the staging store and the env handle (mh_env_destroy). Idempotent; every later
        call into the sampler raises. Raises afterwards if a fused horizon reported a timed-out
        wait (check_errors)."""
        err = None
        try:
            self.check_errors()
        except RuntimeError as ex:
            err = ex
        g, self._graph, self._graph_key = self._graph, None, None
        if g is not None:
            g.reset()
        self._packed = self._staging = self._bound = None
        self.envs.close()
        self._h = None
        self._noise = None
        if err is not None:
            raise err

    def _handle(self):
        if self._h is None:
            raise RuntimeError("HipNstepOffSampler is closed")
        return self._h

    def set_kernel_timing(self, enable: bool):
        """Per-kernel HIP-event timing (runs the horizon eagerly while enabled)."""
        self._timing = bool(enable)
        N.check(N.lib().mh_env_set_timing(self._handle(), int(enable)), "mh_env_set_timing")

    # ------------------------------------------------------------------ parity mode
    def step_traced(self, act_out, logp_out, trace=None, state_trace=None):
        """One lockstep step of the sampling path itself, eagerly: exactly what one iteration of
        the sampler's horizon runs (policy forward, then the lockstep kernel with in-kernel
        TanhGauss sampling, clip, in-kernel resets and deferred emission into the bound store),
        additionally writing the sampled actions [E, A] and log-probs [E] and, when `trace` =
        (real_next_obs [E, D], reward [E], terminated u8 [E], truncated u8 [E]) device tensors is
        given, the env step's outputs (mh_rollout_set_trace); `state_trace` = (state [S, E] float32,
        xstate [XS, E] float64 or None) device tensors receive the post-step state of the envs that
        reset, BEFORE the autoreset overwrites it (mh_rollout_set_trace_state; other columns are
        left as they were). Returns the policy logits.
        Call flush() after the last step to emit its windows."""
        self._handle()
        N.require_device(act_out, "act_out", torch.float32, self.num_envs * self.envs.act_dim, self.device)
        N.require_device(logp_out, "logp_out", torch.float32, self.num_envs, self.device)
        ptrs = [None] * 4
        if trace is not None:
            real, rew, term, trunc = trace
            N.require_device(real, "real_next_obs", torch.float32, self.num_envs * self.envs.obs_dim, self.device)
            N.require_device(rew, "reward", torch.float32, self.num_envs, self.device)
            N.require_device(term, "terminated", torch.uint8, self.num_envs, self.device)
            N.require_device(trunc, "truncated", torch.uint8, self.num_envs, self.device)
            ptrs = [N.ptr(t) for t in trace]
        if self._bound is None:
            raise RuntimeError("step_traced: bind_store(buffer) first (windows go to the bound store)")
        sptr = [None, None]
        if state_trace is not None:
            st, xs = state_trace
            env = self.envs
            N.require_device(st, "trace state", torch.float32, env.state_dim * self.num_envs, self.device)
            if env.xstate_dim:
                N.require_device(xs, "trace xstate", torch.float64, env.xstate_dim * self.num_envs, self.device)
            sptr = [N.ptr(st), N.ptr(xs) if env.xstate_dim else None]
        N.check(N.lib().mh_rollout_set_trace(self._h, *ptrs), "mh_rollout_set_trace")
        N.check(N.lib().mh_rollout_set_trace_state(self._h, *sptr), "mh_rollout_set_trace_state")
        try:
            with torch.no_grad():
                self._draw_noise()
                return self._policy_step(self._bound, self._pack_policy(), act_out=act_out, logp_out=logp_out)
        finally:
            N.check(N.lib().mh_rollout_set_trace(self._h, None, None, None, None), "mh_rollout_set_trace")
            N.check(N.lib().mh_rollout_set_trace_state(self._h, None, None), "mh_rollout_set_trace_state")

    def flush(self):
        """Emit the windows of the last deferred lockstep step (mh_rollout_flush)."""
        self._handle()
        self._flush()

    def step_injected(self, actions, logp, reset_states=None, store=None):
        """One lockstep step with injected (already clipped) actions and log-probs."""
        self._handle()
        act = torch.as_tensor(actions, dtype=torch.float32, device=self.device).contiguous()
        lp = torch.as_tensor(logp, dtype=torch.float32, device=self.device).contiguous()
        N.require_device(act, "actions", torch.float32, self.num_envs * self.envs.act_dim, self.device)
        N.require_device(lp, "logp", torch.float32, self.num_envs, self.device)
        rs = None
        if reset_states is not None:
            rs = torch.as_tensor(reset_states, dtype=torch.float32, device=self.device).contiguous()
            N.require_device(rs, "reset_states", torch.float32, self.num_envs * self.envs.reset_dim, self.device)
        self._lockstep(store if store is not None else self._bound, act_in=act, logp_in=lp, reset_states=rs)
