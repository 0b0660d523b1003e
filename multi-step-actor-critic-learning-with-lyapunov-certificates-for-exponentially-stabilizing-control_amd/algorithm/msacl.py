"""MSACL (RL/algorithm/msacl.py:23-460) on MI355X.

Networks, optimisers and autograd stay PyTorch-ROCm (the north star keeps the MLPs in
PyTorch). The element-wise/scan target math between the network evaluations runs in fused
gfx950 kernels (csrc/msacl_kernels.hip) that also return the analytic gradient w.r.t. the
network outputs, which is handed to autograd:
  * Q backup + twin MSE                          msacl.py:242-257   -> mh_msacl_q_target
  * IS cumprod, bound hinges, ESL, lambda-weighted
    Lyapunov decrease                            msacl.py:279-332   -> mh_msacl_lyapunov
  * stability advantage + batch normalisation +
    PPO clip                                     msacl.py:383-405   -> mh_msacl_stability_adv / _ppo_clip
Data-parallel (one rank per GPU): every optimiser step all-reduces its gradients as one flat
bucket over RCCL, and the advantage normalisation all-reduces its (sum, sumsq) so the batch
statistic is the global batch's (msacl.py:400).
With an explicit device="cpu" (BASELINE.json config 1) the same update runs on the CPU, the
target math through the engine's CPU build (libmsacl_host.so, mhh_msacl_*: the same element
formulas as host loops) — chosen by configuration, never as a fallback of the HIP path.
"""
__all__ = ["ApproxContainer", "MSACL"]

import math
import os
import time
from copy import deepcopy
from collections.abc import Mapping
from typing import Any, Dict, Optional

import torch
import torch.distributions.normal as tdn
import torch.nn as nn
from torch.optim import Adam

from .. import _native as N
from ..create_pkg.create_apprfunc import create_apprfunc
from ..utils import dist as D
from ..utils.common_utils import get_apprfunc_dict
from ..utils.tensorboard_setup import tb_tags


def _adam(params, lr):
    """Single-launch capturable Adam (algorithm/_update_graph.py fused_adam: mh_adam_multi on HIP
    float32 parameters), so the whole update can be replayed as a HIP graph."""
    from ._update_graph import fused_adam
    return fused_adam(params, lr)


def adam_steps(*opts):
    from ._update_graph import adam_steps as _steps
    _steps(*opts)


def _engine(name, device, *args):
    """mh_<name>(*args, stream) on a HIP device; mhh_<name>(*args) of the CPU build on the CPU."""
    if device.type == "cpu":
        N.host_check(getattr(N.host_lib(), "mhh_" + name)(*args), "mhh_" + name)
    else:
        N.check(getattr(N.lib(), "mh_" + name)(*args, N.stream_of(device)), "mh_" + name)


class ApproxContainer(nn.Module):
    """q1, q2 (+ frozen Polyak targets), Lyapunov V, policy, log_alpha and their Adams."""

    def __init__(self, **kwargs):
        super().__init__()
        q_args = get_apprfunc_dict("value", **kwargs)
        self.q1: nn.Module = create_apprfunc(**q_args)
        self.q2: nn.Module = create_apprfunc(**q_args)
        self.q1_target = deepcopy(self.q1)
        self.q2_target = deepcopy(self.q2)
        for p in list(self.q1_target.parameters()) + list(self.q2_target.parameters()):
            p.requires_grad = False
        self.lyapunov: nn.Module = create_apprfunc(**get_apprfunc_dict("lyapunov", **kwargs))
        self.policy: nn.Module = create_apprfunc(**get_apprfunc_dict("policy", **kwargs))
        self.log_alpha = nn.Parameter(torch.tensor(1.0, dtype=torch.float32))
        self._lrs = dict(q=kwargs["q_learning_rate"], lya=kwargs["lyapunov_learning_rate"],
                         pi=kwargs["policy_learning_rate"], alpha=kwargs["alpha_learning_rate"])
        self._make_optimizers()

    def _make_optimizers(self):
        self.q1_optimizer = _adam(self.q1.parameters(), self._lrs["q"])
        self.q2_optimizer = _adam(self.q2.parameters(), self._lrs["q"])
        self.lyapunov_optimizer = _adam(self.lyapunov.parameters(), self._lrs["lya"])
        self.policy_optimizer = _adam(self.policy.parameters(), self._lrs["pi"])
        self.alpha_optimizer = _adam([self.log_alpha], self._lrs["alpha"])

    def create_action_distributions(self, logits):
        return self.policy.get_act_dist_cls(logits)


_UNSET = object()
# torch's normal draw as imported: a test that monkeypatches it (recorded-noise injection) keeps
# the torch draw path; otherwise the update's rsample noise is drawn inside the head kernel
_TORCH_STANDARD_NORMAL = tdn._standard_normal


def _stacked(a, b):
    """torch.cat([a, b], 0), as a view when b directly follows a in one buffer (the replayed
    update's static inputs)."""
    if (a.is_contiguous() and b.is_contiguous() and a.shape == b.shape and a.dtype == b.dtype
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()):
        return a.as_strided((2 * a.shape[0],) + tuple(a.shape[1:]), a.stride())
    return torch.cat([a, b], 0)


_TB_SLOTS = 256  # policy updates a tb dict stays readable for (the device ring of logged scalars)


class LazyTbInfo(Mapping):
    """model_update's tb dict (msacl.py:211-222) over a device tensor of its seven scalars: the
    values are read back (one transfer, a host sync) on first access, alg_time then being the
    wall time from the update's start to that read (the reference's .item() calls sync inside
    model_update, so its alg_time includes the device work too)."""

    KEYS = ("MSACL/entropy-RL iter", "MSACL/alpha-RL iter", "MSACL/q1_mean-RL iter", "MSACL/q2_mean-RL iter",
            tb_tags["loss_critic"], tb_tags["loss_lyapunov"], tb_tags["loss_actor"])

    def __init__(self, vals: torch.Tensor, start: float, gen=None):
        self._vals, self._start, self._d, self._gen = vals, start, None, gen

    def _dict(self):
        if self._d is None:
            h = self._vals.cpu()
            if self._gen is not None:  # a ring slot (MSACL._tb_pack): it must still hold this update
                tag = int(h.view(torch.int32)[7]) & 0xFFFFFFFF
                want = self._gen & 0xFFFFFFFF
                if tag != want:
                    # a later generation in the slot: genuine reuse by later policy updates; an
                    # earlier one (or a jump of more than the ring): the host mirror (_tb_gen) and the
                    # device counter disagree, i.e. some update launch never reached _update_result
                    d = (tag - want) & 0xFFFFFFFF
                    kind = ("reused its slot" if d % _TB_SLOTS == 0 and 0 < d < 1 << 31 else
                            "host/device generation desync")
                    raise RuntimeError(f"MSACL tb dict read after {_TB_SLOTS} later policy updates {kind}: expected "
                                       f"generation {want}, slot holds {tag}")
            v = h[:7].tolist()
            self._d = dict(zip(self.KEYS, v))
            self._d[tb_tags["alg_time"]] = (time.time() - self._start) * 1000
            self._vals = None
        return self._d

    def __getitem__(self, k):
        return self._dict()[k]

    def __iter__(self):
        return iter(self._dict())

    def __len__(self):
        return len(self._dict())

    def __repr__(self):
        return repr(self._dict())


class _PolicyQLoss(torch.autograd.Function):
    """(min(q1, q2) - alpha * logp).mean() and -logp.mean() (msacl.py:383-391) in one launch,
    backward in one launch (mh_msacl_policy_loss[_backward])."""

    @staticmethod
    def forward(ctx, q1, q2, logp, log_alpha):
        out = torch.empty(2, dtype=torch.float32, device=q1.device)
        _engine("msacl_policy_loss", q1.device, N.ptr(q1), N.ptr(q2), N.ptr(logp), N.ptr(log_alpha), q1.numel(),
                N.ptr(out[0:1]), N.ptr(out[1:2]))
        ctx.save_for_backward(q1, q2, log_alpha)
        loss, entropy = out[0], out[1]
        ctx.mark_non_differentiable(entropy)
        return loss, entropy

    @staticmethod
    def backward(ctx, g_loss, g_entropy):
        q1, q2, log_alpha = ctx.saved_tensors
        dq1, dq2, dlogp = torch.empty_like(q1), torch.empty_like(q2), torch.empty_like(q1)
        _engine("msacl_policy_loss_backward", q1.device, N.ptr(q1), N.ptr(q2), N.ptr(log_alpha),
                N.ptr(g_loss.contiguous()), q1.numel(), N.ptr(dq1), N.ptr(dq2), N.ptr(dlogp))
        return dq1, dq2, dlogp, None


class _PolicyHead(torch.autograd.Function):
    """The policy step's head (msacl.py:340-394): StochaPolicy's [mean | exp(clamp(log_std))] of the
    MLP's raw rows, the TanhGauss reparameterised sample written into the critic input
    xq = [obs | act] (ActionValue's concat), its log-prob, and log_prob(old_act), as one launch
    forward (mh_policy_head) and one backward (mh_policy_head_backward) instead of StochaHead +
    rsample + two concats + log_prob forward and their four backward kernels + gradient adds."""

    @staticmethod
    def forward(ctx, raw, eps, obs, old_act, high, low, lo, hi, rng=None):
        R, A, D = raw.shape[0], raw.shape[1] // 2, obs.shape[1]
        xq = torch.empty(R, D + A, dtype=raw.dtype, device=raw.device)
        new_logp = torch.empty(R, dtype=raw.dtype, device=raw.device)
        old_logp = torch.empty(R, dtype=raw.dtype, device=raw.device)
        if eps is None:  # rng = (seed, counter): the noise drawn in-kernel, kept for the backward
            eps = torch.empty(R, A, dtype=raw.dtype, device=raw.device)
            N.check(N.lib().mh_policy_head_sample(N.ptr(raw), N.ptr(obs), N.ptr(old_act), N.ptr(high), N.ptr(low), R,
                                                  A, D, lo, hi, rng[0], N.ptr(rng[1]), N.ptr(eps), N.ptr(xq),
                                                  N.ptr(new_logp), N.ptr(old_logp), N.stream_of(raw.device)),
                    "mh_policy_head_sample")
        else:
            _engine("policy_head", raw.device, N.ptr(raw), N.ptr(eps), N.ptr(obs), N.ptr(old_act), N.ptr(high),
                    N.ptr(low), R, A, D, lo, hi, N.ptr(xq), N.ptr(new_logp), N.ptr(old_logp))
        ctx.save_for_backward(raw, eps, old_act, high, low)
        ctx.dims = (R, A, D, lo, hi)
        return xq, new_logp, old_logp

    @staticmethod
    def backward(ctx, d_xq, d_new_logp, d_old_logp):
        raw, eps, old_act, high, low = ctx.saved_tensors
        R, A, D, lo, hi = ctx.dims
        d_raw = torch.empty_like(raw)
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        _engine("policy_head_backward", raw.device, N.ptr(raw), N.ptr(eps), N.ptr(old_act), N.ptr(high), N.ptr(low),
                N.ptr(c(d_xq)), N.ptr(c(d_new_logp)), N.ptr(c(d_old_logp)), R, A, D, lo, hi, N.ptr(d_raw))
        return d_raw, None, None, None, None, None, None, None, None


class _PolicyObjective(torch.autograd.Function):
    """loss_policy = -(min(q1, q2) - alpha logp).mean() - PPO-clip(exp(lp_new - old_logp)[:, 0],
    normalised stability advantage) (msacl.py:379-405) and the entropy, as one single-workgroup
    launch (mh_msacl_policy_objective: the policy-loss, ratio, clip and total kernels' own
    expressions, writing ratio / adv / loss_ppo / d_ratio into the scratch) and one backward
    launch; bit-identical to those kernels and their autograd seeds (-1, -d_ratio)."""

    @staticmethod
    def forward(ctx, q1, q2, logp, lp_new, old_logp, log_alpha, s, n_total, clip):
        B, n = lp_new.shape
        out = torch.empty(3, dtype=torch.float32, device=q1.device)  # loss_q, entropy, loss_policy
        _engine("msacl_policy_objective", q1.device, N.ptr(q1), N.ptr(q2), N.ptr(logp), N.ptr(log_alpha),
                N.ptr(lp_new), N.ptr(old_logp), N.ptr(s.adv_raw), N.ptr(s.stats), n_total, clip, B, n,
                N.ptr(out[0:1]), N.ptr(out[1:2]), N.ptr(s.ratio), N.ptr(s.adv), N.ptr(s.loss_ppo), N.ptr(s.d_ratio),
                N.ptr(out[2:3]))
        ctx.save_for_backward(q1, q2, log_alpha)
        ctx.s, ctx.shape = s, (B, n)
        entropy = out[1]
        ctx.mark_non_differentiable(entropy)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the entropy (a fill launch)
        return out[2], entropy

    @staticmethod
    def backward(ctx, g_loss, g_entropy):
        q1, q2, log_alpha = ctx.saved_tensors
        s = ctx.s
        B, n = ctx.shape
        dq = torch.empty((2,) + tuple(q1.shape), dtype=q1.dtype, device=q1.device)  # one buffer: TwinQ reads both
        dq1, dq2, dlogp = dq[0], dq[1], torch.empty_like(q1)
        dlp = torch.empty(B, n, dtype=torch.float32, device=q1.device)
        _engine("msacl_policy_objective_backward", q1.device, N.ptr(q1), N.ptr(q2), N.ptr(log_alpha), N.ptr(s.ratio),
                N.ptr(s.d_ratio), N.ptr(g_loss.contiguous()), B, n, N.ptr(dq1), N.ptr(dq2), N.ptr(dlogp), N.ptr(dlp))
        return dq1, dq2, dlogp, dlp, None, None, None, None, None


def _policy_objective_step(q1, q2, logp, lp_new, old_logp, log_alpha, s, n_total, clip, target_entropy=0.0,
                           alpha_grad=None):
    """_PolicyObjective forward AND its backward for the unit seed of the policy step
    (torch.autograd.backward([loss_policy], [1])), plus alpha_grad = (entropy - target_entropy)
    exp(log_alpha) (mh_msacl_alpha_grad's expression, msacl.py:429-441) when alpha_grad is given,
    in ONE launch (mh_msacl_policy_objective_step; the same expressions as the objective, its
    backward with g = 1 and the alpha kernel, so the same bits). Returns the logged loss and
    entropy and the seeds (dq1, dq2, dlogp, dlp_new) for the upstream graph."""
    B, n = lp_new.shape
    out = torch.empty(3, dtype=torch.float32, device=q1.device)  # loss_q, entropy, loss_policy
    dq = s.dq_obj  # dq1 | dq2 as one buffer: TwinQ's grouped backward reads both
    _engine("msacl_policy_objective_step", q1.device, N.ptr(q1), N.ptr(q2), N.ptr(logp), N.ptr(log_alpha),
            N.ptr(lp_new), N.ptr(old_logp), N.ptr(s.adv_raw), N.ptr(s.stats), n_total, clip, B, n,
            N.ptr(out[0:1]), N.ptr(out[1:2]), N.ptr(s.ratio), N.ptr(s.adv), N.ptr(s.loss_ppo), N.ptr(s.d_ratio),
            N.ptr(out[2:3]), N.ptr(dq[0]), N.ptr(dq[1]), N.ptr(s.dlogp_obj), N.ptr(s.dlp_obj), float(target_entropy),
            N.ptr(alpha_grad))
    return out[2], out[1], (dq[0], dq[1], s.dlogp_obj, s.dlp_obj)


class _Ratio0(torch.autograd.Function):
    """exp(logp_new - old_logp)[:, 0] (msacl.py:392-394) and its backward, one launch each."""

    @staticmethod
    def forward(ctx, lp, old):
        B, n = lp.shape
        ratio = torch.empty(B, dtype=torch.float32, device=lp.device)
        _engine("msacl_ratio0", lp.device, N.ptr(lp), N.ptr(old), B, n, N.ptr(ratio))
        ctx.save_for_backward(ratio)
        ctx.n = n
        return ratio

    @staticmethod
    def backward(ctx, g):
        (ratio,) = ctx.saved_tensors
        B, n = ratio.shape[0], ctx.n
        dlp = torch.empty(B, n, dtype=torch.float32, device=ratio.device)
        _engine("msacl_ratio0_backward", ratio.device, N.ptr(ratio), N.ptr(g.contiguous()), B, n, N.ptr(dlp))
        return dlp, None


class _Scratch:
    """Per-shape device work buffers for the fused kernels (allocated once per batch shape)."""

    def __init__(self, B, n, device):
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=device)  # noqa: E731
        self.backup = f(B, n)
        # dq1 | dq2 as the two halves of one buffer: the twin critics' grouped backward reads both
        self.dq_both = f(2, B, n)
        self.dq1, self.dq2 = self.dq_both[0], self.dq_both[1]
        self.abs_td, self.loss_q, self.q_means = f(B), f(1), f(2)
        self.is_clip, self.esl, self.lya_diff, self.loss_lya = f(B, n), f(B, n), f(B), f(1)
        # dV | dV2 as the two halves of one buffer: the two Lyapunov evaluations run as one batch
        self.dV_both = f(2 * B, n)
        self.dV, self.dV2 = self.dV_both[:B], self.dV_both[B:]
        self.adv_raw, self.adv, self.loss_ppo, self.d_ratio = f(B), f(B), f(1), f(B)
        self.loss_policy, self.neg_d_ratio, self.ratio = f(1), f(B), f(B)
        self.stats = torch.empty(2, dtype=torch.float64, device=device)
        # the policy objective's gradients (dq1 | dq2, dlogp, dlp_new), written by its fused step
        self.dq_obj, self.dlogp_obj, self.dlp_obj = f(2, B, n), f(B, n), f(B, n)


class MSACL:
    def __init__(self, gamma: float = 0.99, retrace_lambda: float = 0.95, lya_eta: float = 0.15,
                 tau: float = 0.005, alpha: float = math.e, auto_alpha: bool = True,
                 target_entropy: Optional[float] = None, policy_frequency: int = 2,
                 target_network_frequency: int = 1, lya_diff_scale: float = 1.0, lya_zero_scale: float = 1.0,
                 lya_positive_scale: float = 1.0, **kwargs: Any):
        dev = kwargs.get("device")
        if dev is None:
            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        if dev is None:
            raise RuntimeError("MSACL's fused target kernels need a HIP device (device=\"cpu\" selects the CPU build)")
        self.device = torch.device(dev)
        self.networks = ApproxContainer(**kwargs).to(self.device)
        self.gamma, self.retrace_lambda, self.lya_eta, self.tau = gamma, retrace_lambda, lya_eta, tau
        self.q_learning_rate = kwargs["q_learning_rate"]
        self.lyapunov_learning_rate = kwargs["lyapunov_learning_rate"]
        self.policy_learning_rate = kwargs["policy_learning_rate"]
        self.alpha_learning_rate = kwargs["alpha_learning_rate"]
        self.policy_frequency = policy_frequency
        self.target_network_frequency = target_network_frequency
        self.n_step = int(kwargs["n_step"])
        self.batch_size = kwargs["replay_batch_size"]
        self.anneal_lr = kwargs.get("anneal_lr", False)
        self.max_iteration = kwargs["max_iteration"]
        self.disable_auto_alpha = kwargs.get("disable_auto_alpha", False)
        self.auto_alpha = not self.disable_auto_alpha
        self.set_alpha_bound = kwargs.get("set_alpha_bound", False)
        self.alpha_bound = kwargs.get("alpha_bound", 2.0)
        self.per_flag = kwargs.get("buffer_name") == "prioritized_replay_buffer"
        with torch.no_grad():
            self.networks.log_alpha.fill_(math.log(alpha))
        if target_entropy is None:
            target_entropy = -kwargs["act_dim"] - (1 if kwargs["env_name"] == "QuadTracking" else 0)
        self.target_entropy = target_entropy
        self.lya_diff_scale, self.lya_zero_scale, self.lya_positive_scale = lya_diff_scale, lya_zero_scale, lya_positive_scale
        self.alpha1 = kwargs.get("alpha1", 1.0)
        self.alpha2 = kwargs.get("alpha2", 2.0)
        self.clip_coef = kwargs.get("clip_coef", 0.1)
        n = self.n_step
        # coefficient vectors (msacl.py:153-164), same torch expressions, on this device
        self.start_obs_norm_coef = ((torch.tensor(1 - self.lya_eta) ** torch.arange(1, n + 1)
                                     * torch.tensor(self.alpha2 / self.alpha1)) ** 0.5).to(self.device).contiguous()
        w = torch.pow(self.retrace_lambda, torch.arange(n))
        self.lya_diff_coef = (w / torch.sum(w)).to(self.device).contiguous()
        self.start_lya_coef = torch.pow((1 - self.lya_eta), torch.arange(n) + 1).to(self.device).contiguous()
        self._scratch = {}
        self.last_priority = None
        self._neg_one = torch.tensor(-1.0, device=self.device)
        self._head_cache = _UNSET
        self._one = torch.tensor(1.0, device=self.device)
        self._alpha_grad = None
        self._alpha_grad_ready = False  # _alpha_grad already holds this policy step's gradient
        self.use_graph = bool(kwargs.get("alg_use_graph", True))
        # the trainer asks a device replay buffer for the batch's [obs | act] and [obs_0; obs2]
        # layouts too (gathered, not concatenated per update); MSACL_JOINT_BATCH=0: torch.cat (A/B)
        self.wants_joint_batch = (self.device.type == "cuda" and os.environ.get("MSACL_JOINT_BATCH", "1") == "1")
        # the policy step's first policy forward reuses the Lyapunov step's (MSACL_REUSE_POLICY_FWD=0: off)
        self._reuse_policy_fwd = os.environ.get("MSACL_REUSE_POLICY_FWD", "1") == "1"
        # later policy steps of an update (nothing beside them on the GPU) launch the critics'
        # forward on the one-workgroup-per-CU grid (MSACL_POLICY_ALONE_RT=0: the default grid)
        self._policy_alone_rt = os.environ.get("MSACL_POLICY_ALONE_RT", "1") == "1"
        self._pol_kept = None
        # the policy step's stability advantage on the side stream beside the policy / critic
        # forward chain (MSACL_POLICY_ADV_SIDE=0: on the main stream, before it)
        self._policy_adv_side = os.environ.get("MSACL_POLICY_ADV_SIDE", "1") == "1"
        # the update's rsample noise drawn inside the policy-head kernel (Philox, a device counter);
        # MSACL_KERNEL_NOISE=0: torch's normal draw (A/B)
        self._kernel_noise = os.environ.get("MSACL_KERNEL_NOISE", "1") == "1"
        self._noise_seed = ((int(kwargs.get("seed", 0) or 0) * 0x9E3779B97F4A7C15 + 0x6A09E667F3BCC909
                             + (D.rank() << 40)) & ((1 << 64) - 1))
        self._noise_ctr = None
        # the Lyapunov update shares no parameter with the critic update (both only read the
        # policy and the batch): on one GPU it runs on a second stream, concurrently
        self.concurrent = bool(kwargs.get("alg_concurrent_streams", True))
        self.twin_streams = bool(kwargs.get("alg_twin_streams", True))  # q1 / q2 branches in parallel
        self._twin = None
        self._side = None
        # the twin critics (and their targets) as one grouped network (apprfunc/_twin.py);
        # alg_twin_grouped=False: two networks, one launch per layer each (A/B)
        self.twin_grouped = bool(kwargs.get("alg_twin_grouped", True))
        self._tc = None
        self.force_graph_segments = bool(kwargs.get("alg_force_graph_segments", False))
        self._static = None
        self._static_shapes = None
        self._static_gen = 0  # bumped whenever _static is rebuilt (keys the trainer's step graphs)
        self._graphs = {}
        self._warm = set()
        # the logged scalars of each policy update land in a device ring (mh_msacl_tb_pack_ring)
        # keyed by a device generation counter that the host mirrors (_tb_gen)
        self._tb_ring = None
        self._tb_ctr = None
        self._tb_gen = 0
        self.policy_updates = 0  # policy optimiser steps taken (host count, read by the trainer's step graph)

    def close(self):
        """Release the captured update graphs, their static inputs, the scratch buffers and the
        side streams now, deterministically (idempotent). A dropped MSACL is freed by refcount
        anyway (it sits in no reference cycle); close() also frees it while it is still referenced."""
        from ._update_graph import release_graph
        graphs, self._graphs = self._graphs, {}
        for g, _outs, _prio in graphs.values():
            release_graph(g)
        self._static = self._static_shapes = None
        self._static_gen += 1
        self._warm = set()
        self._scratch = {}
        self.last_priority = None
        self._twin = self._side = None
        self._tc = None

    def _twin_critics(self, rows):
        """(TwinCritic of q1/q2, TwinCritic of their targets) when the grouped path applies to a
        batch of `rows` rows, else None. Built on first use (the parameters move into joint
        buffers then); a rebuilt joint storage invalidates the captured update graphs."""
        if not self.twin_grouped or self.device.type != "cuda" or self._head() is None:
            return None
        from ..apprfunc._fused import gemm_backend
        if gemm_backend() == "blas":
            return None
        nets = self.networks
        if self._tc is None:
            from ..apprfunc._twin import TwinCritic
            a = TwinCritic.build(nets.q1, nets.q2)
            b = TwinCritic.build(nets.q1_target, nets.q2_target) if a is not None else None
            self._tc = (a, b) if (a is not None and b is not None) else False
        if not self._tc:
            return None
        a, b = self._tc
        if (a.joined() | b.joined()) and self._graphs:  # parameters were re-pointed: stale graphs
            from ._update_graph import release_graph
            for g, _o, _p in self._graphs.values():
                release_graph(g)
            self._graphs, self._warm = {}, set()
        return self._tc if a.applies(rows) else None

    @property
    def adjustable_parameters(self):
        return ("gamma", "tau", "auto_alpha", "alpha", "target_entropy", "policy_frequency", "target_network_frequency")

    def _head(self):
        """(high, low, log_std lo, hi) when the fused policy head applies (HIP float32 StochaPolicy
        MLP + TanhGaussDistribution with A <= 8, ActionValue critics), else None."""
        if self._head_cache is not _UNSET:
            return self._head_cache
        from ..apprfunc.mlp import ActionValue, StochaPolicy
        from ..utils.act_distribution_cls import TanhGaussDistribution
        nets, h = self.networks, None
        pol = nets.policy
        if (self.device.type == "cuda" and isinstance(pol, StochaPolicy)
                and pol.action_distribution_cls is TanhGaussDistribution
                and all(isinstance(q, ActionValue) for q in (nets.q1, nets.q2, nets.q1_target, nets.q2_target))):
            hi, lo = pol.act_high_lim, pol.act_low_lim
            A = hi.numel()
            if (0 < A <= 8 and hi.shape == (A,) and lo.shape == (A,) and hi.dtype == torch.float32
                    and lo.dtype == torch.float32 and hi.device == self.device and lo.device == self.device):
                h = (hi.contiguous(), lo.contiguous(), float(pol.min_log_std), float(pol.max_log_std))
        self._head_cache = h
        return h

    def _noise(self, raw):
        """The rsample noise, drawn where TanhGaussDistribution.rsample draws it (same generator
        call, same shape: the tests' recorded-noise injection sees the same sequence). None on a
        HIP device when nothing patched the draw: the head kernel then draws it (mh_policy_head_sample,
        _noise_rng), saving the normal_ launch per head."""
        if (self._kernel_noise and raw.is_cuda and tdn._standard_normal is _TORCH_STANDARD_NORMAL):
            return None
        shape = raw.shape[:-1] + (raw.shape[-1] // 2,)
        return tdn._standard_normal(shape, dtype=raw.dtype, device=raw.device)

    def _noise_rng(self):
        """(seed, device counter) of the in-kernel rsample noise: the counter advances on the
        device once per head launch, so graph replays draw new noise; the seed differs per rank."""
        if self._noise_ctr is None:
            self._noise_ctr = torch.zeros(2, dtype=torch.int64, device=self.device)
        return self._noise_seed, self._noise_ctr

    def rng_state(self) -> dict:
        """The algorithm's random state beyond its networks: the in-kernel rsample noise's seed and
        device counter. The reference checkpoints only `networks.state_dict()` (its torch generator
        restarts from the seed on resume); saving this as well lets a resumed run continue the
        noise sequence instead of replaying it from the start."""
        ctr = None if self._noise_ctr is None else self._noise_ctr.detach().cpu().clone()
        return {"noise_seed": int(self._noise_seed), "noise_ctr": ctr}

    def load_rng_state(self, state: dict) -> None:
        """Restore rng_state(): the counter is written in place (captured update graphs hold its
        address); a changed seed drops the captured graphs (the seed is a kernel argument)."""
        seed = int(state["noise_seed"])
        if seed != self._noise_seed and self._graphs:
            from ._update_graph import release_graph
            graphs, self._graphs = self._graphs, {}
            for g, _o, _p in graphs.values():
                release_graph(g)
            self._warm = set()
        self._noise_seed = seed
        ctr = state.get("noise_ctr")
        if ctr is not None:
            _seed, dev_ctr = self._noise_rng()
            dev_ctr.copy_(torch.as_tensor(ctr, dtype=torch.int64).to(dev_ctr.device))

    def _buf(self, B, n):
        key = (B, n)
        if key not in self._scratch:
            self._scratch[key] = _Scratch(B, n, self.device)
        return self._scratch[key]

    def _get_alpha(self, requires_grad: bool = False):
        alpha = self.networks.log_alpha.exp()
        return alpha if requires_grad else alpha.item()

    # ------------------------------------------------------------------ update
    def model_update(self, data: Dict[str, torch.Tensor], global_iteration: int):
        start = time.time()
        if self.anneal_lr:
            frac = max(0.0, 1.0 - global_iteration / self.max_iteration)
            for opt, lr in ((self.networks.q1_optimizer, self.q_learning_rate), (self.networks.q2_optimizer, self.q_learning_rate),
                            (self.networks.lyapunov_optimizer, self.lyapunov_learning_rate),
                            (self.networks.policy_optimizer, self.policy_learning_rate),
                            (self.networks.alpha_optimizer, self.alpha_learning_rate)):
                opt.param_groups[0]["lr"] = lr * frac
        data = {k: (v.to(self.device).contiguous() if torch.is_tensor(v) else v) for k, v in data.items()}
        flags = (global_iteration % self.target_network_frequency == 0, global_iteration % self.policy_frequency == 0)
        if self._graphable():
            outs = self._graph_update(data, flags)
        else:
            outs = self._update_body(data, *flags)
        return self._update_result(outs, flags, data, start)

    def model_update_drawn(self, draw, global_iteration: int):
        """model_update with the replay draw inside the replayed update: `draw(out)` gathers the
        next batch into the static inputs `out` (DeviceNstepReplayBuffer.sample_batch(B, out=out):
        one launch keyed by the buffer's device draw counter), and runs as the first node of the
        captured graph instead of as separate launches before it. Only valid once replay_inputs()
        returns the static inputs (the trainer checks); same batches, same results as
        model_update(buffer.sample_batch(B, out=replay_inputs(B))) in the same order."""
        start = time.time()
        if self.anneal_lr or self._static is None:
            raise RuntimeError("model_update_drawn needs the replayed update's static inputs (replay_inputs)")
        flags = (global_iteration % self.target_network_frequency == 0, global_iteration % self.policy_frequency == 0)
        outs = self._graph_update(None, flags, draw=draw)
        return self._update_result(outs, flags, self._static, start)

    def drawn_step_parts(self, draw, global_iteration: int):
        """model_update_drawn as parts for a trainer-level graph that also holds the sampling
        before it (NstepOffSerialTrainer._graph_step): (key, body, post), or None until this
        branch's eager first run happened (through model_update_drawn) or when the update is not
        one graph (annealed learning rates, data-parallel segments). body() -> outs: the draw and
        the update, exactly what the drawn graph captures; post(outs, start) -> model_update's
        return value."""
        if self.anneal_lr or self._static is None or self._segmented():
            return None
        flags = (global_iteration % self.target_network_frequency == 0, global_iteration % self.policy_frequency == 0)
        if flags + ("drawn",) not in self._warm:
            return None
        # the static inputs' generation, not one tensor's address: a rebuilt static dict may reuse
        # one old address while its other tensors moved
        key = flags + (self._static_gen,)

        def body():
            draw(self._static)
            return self._update_body(self._static, *flags)

        return key, body, lambda outs, start: self._update_result(outs, flags, self._static, start)

    def _update_result(self, outs, flags, data, start):
        if flags[1]:
            self.policy_updates += 1  # (every update path: eager, replayed, or inside a step graph)
        tb_info = None
        if flags[1]:
            # the logged scalars (msacl.py:211-222), stacked on the device inside the update and
            # snapshotted here (the next replay overwrites the graph's output); read back only when
            # the caller reads the dict (the trainer: on logging iterations), so an update leaves
            # no host sync behind and the next sampling is enqueued while it still runs
            tb = outs[-1]
            if tb is self._tb_ring:  # this update's slot of the ring (no copy out of the graph)
                gen = self._tb_gen
                self._tb_gen += 1
                tb_info = LazyTbInfo(tb[gen % _TB_SLOTS], start, gen)
            else:
                tb_info = LazyTbInfo(tb.clone(), start)
        if self.per_flag:
            return tb_info, data.get("idx"), self.last_priority
        return tb_info

    def _twin_stream(self):
        """Stream for the second critic's branch (q2 / q2 target forward; autograd runs each
        backward op on its forward's stream, so the two critics' backward passes overlap too).
        None when streams are off or on CPU."""
        if not (self.concurrent and self.device.type == "cuda" and self.twin_streams):
            return None
        if self._twin is None:
            self._twin = D.side_stream(self.device)
        return self._twin

    def _twin_pair(self, f1, f2):
        """(f1(), f2()) with f2 on the twin stream (fork/join around it); outputs produced there
        are recorded for the current stream that consumes them.

        Invariant: no twin-stream work may outlive the join (`cur.wait_stream(tw)` below). The
        inputs f2 reads (obs, act, next_act, new_act, ...) are allocated on the current stream
        and are NOT record_stream'ed for the twin stream; they stay safe only because every
        kernel f2 enqueues is ordered before the join, and autograd runs the backward of f2's ops
        on this same twin stream before the current stream's later consumers (autograd's own
        stream sync). Launching further work on the twin stream after the join would let the
        caching allocator hand those inputs' blocks out while it still reads them."""
        tw = self._twin_stream()
        if tw is None:
            return f1(), f2()
        cur = torch.cuda.current_stream(self.device)
        with D.fork(tw):
            r2 = f2()
        r1 = f1()
        cur.wait_stream(tw)
        for t in (r2 if isinstance(r2, tuple) else (r2,)):
            t.record_stream(cur)
        return r1, r2

    def _seg_side_stream(self):
        if self._side is None:
            self._side = D.side_stream(self.device)
        return self._side

    def _side_stream(self):
        if not (self.concurrent and not D.collectives_active() and self.device.type == "cuda"
                and not self.force_graph_segments and not D.segment_capture_active()):
            return None
        if self._side is None:
            self._side = D.side_stream(self.device)
        return self._side

    def _update_body(self, data, do_target, do_policy):
        """One model_update's device work (msacl.py:193-210); returns device tensors only. The
        critic (+ target) and Lyapunov updates are independent (disjoint parameters, read-only
        policy and batch) and run on two streams (fork/join; captured as parallel graph branches);
        the policy and alpha updates, which read both, follow the join."""
        side = self._side_stream()
        if side is not None:
            main = torch.cuda.current_stream(self.device)
            with D.fork(side):
                loss_lya = self._lyapunov_update(data, keep_policy=do_policy)
            loss_q, q1_mean, q2_mean = self._q_update(data, stats=do_policy)
            main.wait_stream(side)
            # the target update after the join: a graph whose last node sits on a side queue makes
            # the next graph launch wait ~20 us for its completion instead of ~5 us (kernel trace,
            # profiles/r05_update_tail_ab.txt); the Polyak step reads only the stepped critics
            if do_target:
                self._target_update()
        elif (self._segmented() or D.collectives_active()) and self.concurrent and self.device.type == "cuda":
            # data parallel: the two backward passes still run as parallel branches, and their
            # gradients are averaged by ONE all-reduce at the join (one graph cut instead of two,
            # the branches stay concurrent inside the segment); the optimizer steps follow it.
            # Same result as the serial order: the critic and Lyapunov losses read disjoint
            # parameters, and each optimizer step only reads its own network's gradients.
            main = torch.cuda.current_stream(self.device)
            side = self._seg_side_stream()
            with D.fork(side):
                loss_lya = self._lyapunov_update(data, defer_step=True, keep_policy=do_policy)
            loss_q, q1_mean, q2_mean = self._q_update(data, defer_step=True, stats=do_policy)
            main.wait_stream(side)
            nets = self.networks
            D.allreduce_grads(list(nets.q1.parameters()) + list(nets.q2.parameters()) +
                              list(nets.lyapunov.parameters()))
            adam_steps(nets.q1_optimizer, nets.q2_optimizer)
            nets.lyapunov_optimizer.step()
            if do_target:
                self._target_update()
        else:
            loss_q, q1_mean, q2_mean = self._q_update(data, stats=do_policy)
            if do_target:
                self._target_update()
            loss_lya = self._lyapunov_update(data, keep_policy=do_policy)
        loss_policy = entropy = None
        if not do_policy:
            return loss_q, q1_mean, q2_mean, loss_lya, loss_policy, entropy
        # the policy and alpha gradients share one all-reduce under data parallelism (the alpha
        # loss reads the policy forward's entropy, not the stepped policy), and both optimiser
        # steps are one Adam launch (disjoint parameters, each with its own learning rate)
        merge = self.auto_alpha
        for k in range(self.policy_frequency):
            loss_policy, entropy = self._policy_update(data=data, defer_step=merge, reuse_adv=k > 0)
            if self.auto_alpha:
                self._alpha_update(entropy=entropy, defer_step=merge)
            if merge:
                nets = self.networks
                D.allreduce_grads(list(nets.policy.parameters()) + [nets.log_alpha])
                adam_steps(nets.policy_optimizer, nets.alpha_optimizer)
                self._alpha_clamp()
        # the logged scalars (msacl.py:211-222), stacked inside the update (model_update snapshots them)
        tb = self._tb_pack(entropy, q1_mean, q2_mean, loss_q, loss_lya, loss_policy)
        return loss_q, q1_mean, q2_mean, loss_lya, loss_policy, entropy, tb

    def _tb_pack(self, entropy, q1_mean, q2_mean, loss_q, loss_lya, loss_policy):
        """The logged scalars (msacl.py:211-222) as one [7] tensor: one launch on a HIP device
        when the critic means are the q-target kernel's (adjacent in its scratch), torch.stack
        otherwise."""
        la = self.networks.log_alpha.detach()
        parts = (entropy, loss_q, loss_lya, loss_policy)
        if (self.device.type == "cuda" and q2_mean.data_ptr() == q1_mean.data_ptr() + 4
                and all(t.numel() == 1 and t.dtype == torch.float32 for t in parts)):
            if self._tb_ring is None:  # (first policy update: eager, before any capture)
                self._tb_ring = torch.zeros(_TB_SLOTS, 8, dtype=torch.float32, device=self.device)
                self._tb_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
                self._tb_gen = 0
            _engine("msacl_tb_pack_ring", self.device, N.ptr(entropy), N.ptr(la), N.ptr(q1_mean), N.ptr(loss_q),
                    N.ptr(loss_lya), N.ptr(loss_policy), N.ptr(self._tb_ring), N.ptr(self._tb_ctr), _TB_SLOTS)
            return self._tb_ring
        return torch.stack([entropy, la.exp(), q1_mean, q2_mean, loss_q, loss_lya, loss_policy])

    # ------------------------------------------------------------------ HIP-graph replay
    def _graphable(self):
        return (self.use_graph and not self.anneal_lr and self.device.type == "cuda" and torch.cuda.is_available()
                and not torch.cuda.is_current_stream_capturing())

    def _segmented(self):
        """World size > 1 (or the test switch): the graph is cut at every collective
        (utils/dist.py GraphSegments) instead of capturing the update as one graph."""
        return D.graph_segments_wanted() or self.force_graph_segments

    def replay_inputs(self, batch_size: int):
        """The replayed update's static input tensors, for the replay buffer to gather the next
        batch straight into (DeviceNstepReplayBuffer.sample_batch(out=...)): the replay then
        needs no copy of the batch. None until the first graph-mode update has created them (or
        when the update does not replay graphs, or the batch size differs)."""
        st = self._static
        if st is None or not self._graphable() or st["rew"].shape[0] != batch_size:
            return None
        return st

    def _graph_update(self, data, flags, draw=None):
        """Replay the whole update (~250 launches) as one HIP graph (with data parallelism: a
        chain of graphs cut at the gradient all-reduces, utils/dist.py GraphSegments). The first
        call per branch (even/odd iteration) runs eagerly on the static inputs (lazy BLAS / Adam
        state init), the second captures, later calls only copy the new batch in and replay.
        draw (model_update_drawn): the batch is gathered into the static inputs by draw(static),
        eagerly or as part of the capture, instead of being passed in."""
        if draw is not None:  # (its own graphs: a replay must draw exactly when its capture did)
            return self._graph_run(flags + ("drawn",),
                                   lambda: (draw(self._static), self._update_body(self._static, *flags))[1])
        shapes = tuple((k, tuple(v.shape)) for k, v in sorted(data.items()) if torch.is_tensor(v))
        if self._static is None or self._static_shapes != shapes:
            self._static = {k: v.clone() for k, v in data.items() if torch.is_tensor(v)}
            o, o2 = self._static.get("obs"), self._static.get("obs2")
            if o is not None and o2 is not None and o.shape == o2.shape and o.dtype == o2.dtype:
                # obs and obs2 as the two halves of one buffer: the Lyapunov step's batch of both
                # (msacl.py:275-276) is then a view, not a concatenation per update
                joint = torch.empty((2,) + tuple(o.shape), dtype=o.dtype, device=o.device)
                joint[0].copy_(o)
                joint[1].copy_(o2)
                self._static["obs"], self._static["obs2"] = joint[0], joint[1]
            self._static_shapes = shapes
            self._static_gen += 1
            self._graphs = {}
            self._warm = set()
        for k, v in self._static.items():
            if data[k].data_ptr() != v.data_ptr():
                v.copy_(data[k])
        return self._graph_run(flags, lambda: self._update_body(self._static, *flags))

    def _graph_run(self, key, body):
        """body() eagerly on the branch's first call, captured on its second, replayed after."""
        if key not in self._warm:
            self._warm.add(key)
            return body()
        if key not in self._graphs:
            if self._segmented():
                g = D.GraphSegments()
                with D.capturing(g):
                    outs = body()
                    prio = self.last_priority
            else:
                g = torch.cuda.CUDAGraph()
                with D.cuda_graph(g):
                    outs = body()
                    prio = self.last_priority
            self._graphs[key] = (g, outs, prio)
        g, outs, prio = self._graphs[key]
        g.replay()
        self.last_priority = prio
        return outs

    def _q_update(self, data, defer_step=False, stats=True):
        obs, act, rew, obs2, done = data["obs"], data["act"], data["rew"], data["obs2"], data["done"]
        B, n = rew.shape
        s = self._buf(B, n)
        nets = self.networks
        head = self._head()
        if head is not None:
            # policy(obs2) -> head + rsample written straight into the target critics' input
            # [obs2 | next_act] (one launch); the batch's [obs | act] concatenated once for both
            hi, lo, lsl, lsh = head
            A, Dd = hi.numel(), obs.shape[-1]
            with torch.no_grad():
                raw = nets.policy.policy(obs2)
                eps = self._noise(raw)
                xq2 = torch.empty(B, n, Dd + A, dtype=torch.float32, device=self.device)
                next_logp = torch.empty(B, n, dtype=torch.float32, device=self.device)
                if eps is None:
                    seed, ctr = self._noise_rng()
                    eps_out = torch.empty(B * n, A, dtype=torch.float32, device=self.device)
                    N.check(N.lib().mh_policy_head_sample(N.ptr(raw.contiguous()), N.ptr(obs2), None, N.ptr(hi),
                                                          N.ptr(lo), B * n, A, Dd, lsl, lsh, seed, N.ptr(ctr),
                                                          N.ptr(eps_out), N.ptr(xq2), N.ptr(next_logp), None,
                                                          N.stream_of(self.device)), "mh_policy_head_sample")
                else:
                    _engine("policy_head", self.device, N.ptr(raw.contiguous()), N.ptr(eps.contiguous()), N.ptr(obs2),
                            None, N.ptr(hi), N.ptr(lo), B * n, A, Dd, lsl, lsh, N.ptr(xq2), N.ptr(next_logp), None)
            xa = data.get("obs_act")  # [obs | act], written by the replay gather (mh_replay_gather_joint)
            if xa is None:
                xa = torch.cat([obs, act], dim=-1)
            tc = self._twin_critics(B * n)
            if tc is not None:
                return self._q_update_twin(tc, data, xa, xq2, next_logp, s, defer_step, stats)
            q_in = lambda q: q.q(xa).squeeze(-1)  # noqa: E731  (ActionValue.forward on the shared concat)
            qt_in = lambda q: q.q(xq2).squeeze(-1)  # noqa: E731
        else:
            with torch.no_grad():
                dist = nets.create_action_distributions(nets.policy(obs2))
                next_act, next_logp = dist.rsample()
            q_in = lambda q: q(obs, act)  # noqa: E731
            qt_in = lambda q: q(obs2, next_act)  # noqa: E731

        def critic1():
            q = q_in(nets.q1)
            with torch.no_grad():
                return q, qt_in(nets.q1_target).contiguous()

        def critic2():
            q = q_in(nets.q2)
            with torch.no_grad():
                return q, qt_in(nets.q2_target).contiguous()

        (q1, q1t), (q2, q2t) = self._twin_pair(critic1, critic2)
        weight = data.get("weight") if self.per_flag else None
        means = self._q_target(q1.detach().contiguous(), q2.detach().contiguous(), q1t, q2t, next_logp, rew, done,
                               weight, B, n, s, stats)
        self.networks.q1_optimizer.zero_grad()
        self.networks.q2_optimizer.zero_grad()
        torch.autograd.backward([q1, q2], [s.dq1, s.dq2])
        if not defer_step:  # deferred: the caller all-reduces and steps (data-parallel join)
            D.allreduce_grads(list(self.networks.q1.parameters()) + list(self.networks.q2.parameters()))
            adam_steps(self.networks.q1_optimizer, self.networks.q2_optimizer)  # one launch for both
        if self.per_flag:
            self.last_priority = s.abs_td.clone()
        if not stats:  # iterations without a policy step log nothing (model_update returns None)
            return s.loss_q[0], None, None
        if means is not None:  # the kernel's means (scratch views, read by model_update right after)
            return s.loss_q[0], means[0], means[1]
        return s.loss_q[0], q1.detach().mean(), q2.detach().mean()

    def _q_target(self, q1, q2, q1t, q2t, next_logp, rew, done, weight, B, n, s, stats):
        """The backup / twin-MSE kernel (msacl.py:242-257). On a HIP device with stats wanted it
        also writes the logged critic means into s.q_means (one pass, no extra reductions) and
        returns that buffer; otherwise None (the caller takes the means itself)."""
        args = (N.ptr(q1), N.ptr(q2), N.ptr(q1t), N.ptr(q2t), N.ptr(next_logp.contiguous()), N.ptr(rew), N.ptr(done),
                N.ptr(self.networks.log_alpha.detach()), N.ptr(weight.contiguous() if weight is not None else None),
                float(self.gamma), B, n, N.ptr(s.backup), N.ptr(s.dq1), N.ptr(s.dq2), N.ptr(s.loss_q),
                N.ptr(s.abs_td))
        if stats and self.device.type == "cuda":
            _engine("msacl_q_target_stats", self.device, *args, N.ptr(s.q_means))
            return s.q_means
        _engine("msacl_q_target", self.device, *args)
        return None

    def _q_update_twin(self, tc, data, xa, xq2, next_logp, s, defer_step, stats):
        """_q_update with both critics (and both targets) as one grouped network each
        (apprfunc/_twin.py): same math, one launch per layer instead of one per layer per critic."""
        twin, twin_t = tc
        rew, done = data["rew"], data["done"]
        B, n = rew.shape
        M = B * n
        xa2 = xa.reshape(M, xa.shape[-1])
        xq2f = xq2.reshape(M, xq2.shape[-1])
        both = twin.forward_pair(xa2, twin_t, xq2f)  # critics + target critics in one launch
        if both is not None:
            q, h1, h2, qt = both
        else:
            q, h1, h2 = twin.forward(xa2)
            qt, _, _ = twin_t.forward(xq2f, keep=False)
        weight = data.get("weight") if self.per_flag else None
        means = self._q_target(q[0], q[1], qt[0], qt[1], next_logp, rew, done, weight, B, n, s, stats)
        twin.backward_weights(xa2, s.dq_both.view(2, M), h1, h2)  # binds q1 / q2 .grad
        if not defer_step:
            D.allreduce_grads(list(self.networks.q1.parameters()) + list(self.networks.q2.parameters()))
            adam_steps(self.networks.q1_optimizer, self.networks.q2_optimizer)
        if self.per_flag:
            self.last_priority = s.abs_td.clone()
        if not stats:
            return s.loss_q[0], None, None
        if means is not None:
            return s.loss_q[0], means[0], means[1]
        return s.loss_q[0], q[0].mean(), q[1].mean()

    def _lyapunov_update(self, data, defer_step=False, keep_policy=False):
        """keep_policy: a policy step follows in this update: keep the policy forward's activations
        (the policy step's first forward is this same evaluation: same rows, weights unchanged
        until its optimiser step) for it (_pol_kept, MLP3Kept)."""
        obs, obs2, act, old_logp = data["obs"], data["obs2"], data["act"], data["logp"]
        B, n = old_logp.shape
        s = self._buf(B, n)
        head = self._head()
        self._pol_kept = None
        with torch.no_grad():
            if head is not None:  # policy(obs) -> head + log_prob(act) in one launch
                hi, lo, lsl, lsh = head
                kept = None
                if keep_policy and self._reuse_policy_fwd:
                    from ..apprfunc._fused import mlp3_forward_kept
                    kept = mlp3_forward_kept(self.networks.policy.policy, obs.reshape(B * n, obs.shape[-1]))
                if kept is not None:
                    raw = kept[0]
                    self._pol_kept = (obs.data_ptr(),) + tuple(kept[1:])
                else:
                    raw = self.networks.policy.policy(obs).contiguous()
                logp = torch.empty(B, n, dtype=torch.float32, device=self.device)
                _engine("policy_head", self.device, N.ptr(raw), None, None, N.ptr(act), N.ptr(hi), N.ptr(lo), B * n,
                        hi.numel(), 0, lsl, lsh, None, None, N.ptr(logp))
            else:
                dist = self.networks.create_action_distributions(self.networks.policy(obs))
                logp = dist.log_prob(act).contiguous()
        # V(obs) and V(obs2) (msacl.py:275-276) as ONE batch through the network: one forward and
        # one backward instead of two each (the weight gradients sum the same 2 B n rows)
        V_both = self.networks.lyapunov(_stacked(obs, obs2))
        V, V2 = V_both[:B], V_both[B:]
        _engine(
            "msacl_lyapunov", self.device,
            N.ptr(logp), N.ptr(old_logp), N.ptr(V.detach().contiguous()), N.ptr(V2.detach().contiguous()), N.ptr(obs),
            N.ptr(obs2), N.ptr(self.start_obs_norm_coef), N.ptr(self.lya_diff_coef), N.ptr(self.start_lya_coef),
            float(self.alpha1), float(self.alpha2), float(self.lya_positive_scale), float(self.lya_diff_scale), B, n,
            obs.shape[-1], N.ptr(s.is_clip), N.ptr(s.esl), N.ptr(s.lya_diff), N.ptr(s.loss_lya), N.ptr(s.dV),
            N.ptr(s.dV2))
        self.networks.lyapunov_optimizer.zero_grad()
        torch.autograd.backward([V_both], [s.dV_both])
        if not defer_step:
            D.allreduce_grads(list(self.networks.lyapunov.parameters()))
            self.networks.lyapunov_optimizer.step()
        return s.loss_lya[0]  # a view of the scratch (no allocation on the side stream)

    def _stability_advantage(self, data, s):
        """V(obs_0), V(obs2) and the raw stability advantage with its (sum, sum of squares)
        statistics into the scratch (msacl.py:392-400); the (Σ, Σ²) all-reduce makes them the
        global batch's under data parallelism."""
        obs, obs2, old_logp = data["obs"], data["obs2"], data["logp"]
        B, n = old_logp.shape
        with torch.no_grad():
            # V(obs_0) and V(obs2) as one batch (msacl.py:395-396)
            D_ = obs.shape[-1]
            v_in = data.get("v_in")  # [obs[:, 0]; obs2 rows], written by the replay gather
            if v_in is None:
                v_in = torch.cat([obs[:, 0], obs2.reshape(-1, D_)], 0)
            V_all = self.networks.lyapunov(v_in)
            V0 = V_all[:B].contiguous()
            V2 = V_all[B:].reshape(B, n).contiguous()
        _engine("msacl_stability_adv", self.device, N.ptr(V0), N.ptr(V2), N.ptr(self.lya_diff_coef),
                N.ptr(self.start_lya_coef), B, n, N.ptr(s.adv_raw), N.ptr(s.stats))
        D.allreduce_(s.stats)

    def _policy_update(self, data, defer_step=False, reuse_adv=False):
        """One policy step (msacl.py:340-405). reuse_adv: a later step of the same update (the
        policy_frequency loop): the Lyapunov network and the batch are unchanged since the first
        step, so its stability advantage and statistics, still in the scratch, are the values a
        recomputation would produce (deterministic kernels), and are not recomputed. The first
        step computes them on the side stream, beside the policy / critic forward chain (joined
        before the clip)."""
        obs, old_act, obs2, old_logp = data["obs"], data["act"], data["obs2"], data["logp"]
        B, n = old_logp.shape
        s = self._buf(B, n)
        side = None
        if not reuse_adv:
            side = self._side_stream() if self._policy_adv_side else None
            if side is not None:
                main = torch.cuda.current_stream(self.device)
                with D.fork(side):
                    self._stability_advantage(data, s)
            else:
                self._stability_advantage(data, s)
        for p in list(self.networks.q1.parameters()) + list(self.networks.q2.parameters()):
            p.requires_grad = False
        nets = self.networks
        head = self._head()
        if head is not None:
            hi, lo, lsl, lsh = head
            A, Dd = hi.numel(), obs.shape[-1]
            pk, self._pol_kept = self._pol_kept, None
            if not reuse_adv and pk is not None and pk[0] == obs.data_ptr():
                # the Lyapunov step's evaluation of this same forward (MLP3Kept: backward only)
                from ..apprfunc._fused import MLP3Kept
                (l1, l2, l3), acts = pk[2], pk[3]
                cur = torch.cuda.current_stream(self.device)
                for t in pk[1]:  # made on the Lyapunov branch's stream, read here after the join
                    t.record_stream(cur)
                raw = MLP3Kept.apply(obs.reshape(B * n, Dd), l1[0], l1[1], l2[0], l2[1], l3[0], l3[1], acts,
                                     pk[1]).view(B, n, 2 * A)  # (the [B, n, 2A] of policy.policy(obs))
            else:
                raw = nets.policy.policy(obs)
            eps = self._noise(raw)
            xq, new_act_logp, old_lp = _PolicyHead.apply(raw.reshape(B * n, 2 * A).contiguous(),
                                                         None if eps is None else eps.reshape(B * n, A).contiguous(),
                                                         obs.reshape(B * n, Dd), old_act.reshape(B * n, A), hi, lo,
                                                         lsl, lsh, self._noise_rng() if eps is None else None)
            xq = xq.reshape(B, n, Dd + A)
            new_act_logp, old_lp = new_act_logp.reshape(B, n), old_lp.reshape(B, n)
            tc = self._twin_critics(B * n)
            if tc is not None:
                from ..apprfunc._twin import TwinQ
                # the policy step's chain runs alone on the GPU (after the branches' join): the
                # critics' forward takes the one-workgroup-per-CU grid (mh_mlp3_set_row_tiles)
                alone = self._policy_alone_rt and reuse_adv
                if alone:
                    N.check(N.lib().mh_mlp3_set_row_tiles(-1), "mh_mlp3_set_row_tiles")
                try:
                    q1, q2 = TwinQ.apply(xq.reshape(B * n, Dd + A), tc[0])
                finally:
                    if alone:
                        N.lib().mh_mlp3_set_row_tiles(0)
                q1, q2 = q1.view(B, n), q2.view(B, n)
            else:
                q1, q2 = self._twin_pair(lambda: nets.q1.q(xq).squeeze(-1), lambda: nets.q2.q(xq).squeeze(-1))
        else:
            dist = nets.create_action_distributions(nets.policy(obs))
            new_act, new_act_logp = dist.rsample()
            q1, q2 = self._twin_pair(lambda: nets.q1(obs, new_act), lambda: nets.q2(obs, new_act))
            old_lp = None
        # (min(q1, q2) - alpha logp).mean() with alpha = exp(log_alpha) read on the device (the
        # reference's alpha.item() float has the same f32 value), and the entropy, in one kernel
        if head is not None:
            # the whole objective (policy loss, step-0 ratio, PPO clip on the stability advantage,
            # the total) in one launch forward and one backward (mh_msacl_policy_objective)
            if side is not None:
                main.wait_stream(side)  # the side branch wrote only the scratch's adv_raw / stats
            # ... and its backward for the unit seed, with the alpha gradient (the alpha loss
            # reads this step's entropy and the unchanged log_alpha), in the same launch
            la = self.networks.log_alpha
            ag = None
            if self.auto_alpha:
                if self._alpha_grad is None:
                    self._alpha_grad = torch.zeros_like(la)
                ag = self._alpha_grad
            loss_policy, entropy, seeds = _policy_objective_step(
                q1.contiguous(), q2.contiguous(), new_act_logp.contiguous(), old_lp.contiguous(),
                old_logp.contiguous(), la.detach(), s, float(B * D.world_size()), float(self.clip_coef),
                float(self.target_entropy) if ag is not None else 0.0, ag)
            self._alpha_grad_ready = ag is not None
            self.networks.policy_optimizer.zero_grad()
            torch.autograd.backward([q1, q2, new_act_logp, old_lp], list(seeds))
            if not defer_step:
                D.allreduce_grads(list(self.networks.policy.parameters()))
                self.networks.policy_optimizer.step()
            for p in list(self.networks.q1.parameters()) + list(self.networks.q2.parameters()):
                p.requires_grad = True
            return loss_policy, entropy
        loss_policy_q, entropy = _PolicyQLoss.apply(q1.contiguous(), q2.contiguous(), new_act_logp.contiguous(),
                                                    self.networks.log_alpha.detach())
        if old_lp is None:
            old_lp = dist.log_prob(old_act)
        is_ratio = _Ratio0.apply(old_lp.contiguous(), old_logp.contiguous())
        if side is not None:
            main.wait_stream(side)  # the side branch wrote only the scratch's adv_raw / stats
        n_total = float(B * D.world_size())
        r_det = is_ratio.detach().contiguous()
        _engine("msacl_ppo_clip", self.device, N.ptr(r_det), N.ptr(s.adv_raw), N.ptr(s.stats), n_total,
                float(self.clip_coef), B, N.ptr(s.adv), N.ptr(s.loss_ppo), N.ptr(s.d_ratio))
        if self.device.type == "cuda":
            # the logged total and the ratio seed -d_ratio in one launch (a view of the scratch,
            # read by model_update right after the update)
            _engine("msacl_policy_combine", self.device, N.ptr(loss_policy_q.detach()), N.ptr(s.loss_ppo),
                    N.ptr(s.d_ratio), B, N.ptr(s.loss_policy), N.ptr(s.neg_d_ratio))
            loss_policy, seed = s.loss_policy[0], s.neg_d_ratio
        else:
            loss_policy, seed = -loss_policy_q.detach() - s.loss_ppo[0], -s.d_ratio
        self.networks.policy_optimizer.zero_grad()
        torch.autograd.backward([loss_policy_q, is_ratio], [self._neg_one, seed])
        if not defer_step:
            D.allreduce_grads(list(self.networks.policy.parameters()))
            self.networks.policy_optimizer.step()
        entropy = entropy.detach()
        for p in list(self.networks.q1.parameters()) + list(self.networks.q2.parameters()):
            p.requires_grad = True
        return loss_policy.detach(), entropy

    def _alpha_update(self, entropy, defer_step=False):
        """msacl.py:429-441. On the device the gradient of alpha * (entropy - target_entropy)
        w.r.t. log_alpha is formed by one kernel (mh_msacl_alpha_grad, autograd's own product)
        into a persistent .grad (the zero_grad + backward it replaces write the same value)."""
        la = self.networks.log_alpha
        if self.device.type == "cuda":
            if self._alpha_grad is None:
                self._alpha_grad = torch.zeros_like(la)
            la.grad = self._alpha_grad
            if not self._alpha_grad_ready:  # else written by the policy objective's launch
                _engine("msacl_alpha_grad", self.device, N.ptr(la.detach()), N.ptr(entropy.contiguous()),
                        float(self.target_entropy), N.ptr(self._alpha_grad))
            self._alpha_grad_ready = False
        else:
            alpha = self._get_alpha(requires_grad=True)
            loss_alpha = alpha * (entropy - self.target_entropy)
            self.networks.alpha_optimizer.zero_grad()
            loss_alpha.backward()
        if not defer_step:
            D.allreduce_grads([self.networks.log_alpha])
            self._alpha_step()

    def _alpha_step(self):
        self.networks.alpha_optimizer.step()
        self._alpha_clamp()

    def _alpha_clamp(self):
        if self.set_alpha_bound:
            with torch.no_grad():
                self.networks.log_alpha.clamp_(max=math.log(self.alpha_bound))

    def _target_update(self):
        """Polyak averaging (msacl.py:445-460): one mh_polyak_multi launch for both target nets."""
        from ._update_graph import polyak_pairs
        polyak_pairs(((self.networks.q1, self.networks.q1_target), (self.networks.q2, self.networks.q2_target)),
                     self.tau)
