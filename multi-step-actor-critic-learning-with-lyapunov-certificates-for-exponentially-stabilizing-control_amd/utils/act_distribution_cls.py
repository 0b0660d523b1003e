"""Action distributions behind StochaPolicy/DetermPolicy (RL/utils/act_distribution_cls.py:15-159).

Same math and the same torch.distributions objects as the reference, so log-probabilities and
the reparameterised noise path (Normal.rsample -> _standard_normal) are identical. The device
rollout samples in-kernel instead (csrc/rollout.hip, TanhGauss + clip fused into the env step).

On HIP float32 logits, TanhGaussDistribution.rsample / log_prob run as one kernel forward and
one backward each (csrc/dist_kernels.hip via the mh_tanh_gauss_* C ABI) instead of ~25 + ~30
elementwise/reduction launches; the noise is still drawn by torch's `_standard_normal`, so the
sample path, seeding and the tests' noise injection are unchanged.
"""
import ctypes

import torch
import torch.distributions.normal as tdn

EPS = 1e-6


class Action_Distribution_Cls:
    """Mixin giving a policy network `get_act_dist_cls(logits)`."""

    def get_act_dist_cls(self, logits):
        dist = getattr(self, "action_distribution_cls")(logits)
        if hasattr(self, "act_high_lim") and hasattr(self, "act_low_lim"):
            dist.act_high_lim = getattr(self, "act_high_lim")
            dist.act_low_lim = getattr(self, "act_low_lim")
        return dist


def _independent_normal(mean, std):
    # validate_args=False: argument validation only raises on invalid parameters but costs a
    # device->host sync per construction (and forbids HIP-graph capture); numerics unchanged.
    return torch.distributions.Independent(torch.distributions.Normal(mean, std, validate_args=False),
                                           reinterpreted_batch_ndims=1, validate_args=False)


def _native():
    from .. import _native as N
    return N


class _TanhGaussRsample(torch.autograd.Function):
    """(logits, eps) -> (act, logp); act_distribution_cls.py:39-55 math, csrc/dist_kernels.hip."""

    @staticmethod
    def forward(ctx, logits, eps, high, low):
        N = _native()
        M, A = eps.shape
        act = torch.empty_like(eps)
        logp = torch.empty(M, dtype=eps.dtype, device=eps.device)
        N.check(N.lib().mh_tanh_gauss_rsample(N.ptr(logits), N.ptr(eps), N.ptr(high), N.ptr(low), M, A,
                                              N.ptr(act), N.ptr(logp), N.stream_of(eps.device)),
                "mh_tanh_gauss_rsample")
        ctx.save_for_backward(logits, eps, high, low)
        return act, logp

    @staticmethod
    def backward(ctx, d_act, d_logp):
        logits, eps, high, low = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        N = _native()
        M, A = eps.shape
        d_logits = torch.empty_like(logits)
        d_act = None if d_act is None else d_act.contiguous()
        d_logp = None if d_logp is None else d_logp.contiguous()
        N.check(N.lib().mh_tanh_gauss_rsample_backward(
            N.ptr(logits), N.ptr(eps), N.ptr(high), N.ptr(low), N.ptr(d_act), N.ptr(d_logp), M, A,
            N.ptr(d_logits), N.stream_of(logits.device)), "mh_tanh_gauss_rsample_backward")
        return d_logits, None, None, None


class _TanhGaussLogProb(torch.autograd.Function):
    """(logits, act) -> logp; act_distribution_cls.py:57-62 math, csrc/dist_kernels.hip."""

    @staticmethod
    def forward(ctx, logits, act, high, low):
        N = _native()
        M, A = act.shape
        logp = torch.empty(M, dtype=act.dtype, device=act.device)
        N.check(N.lib().mh_tanh_gauss_log_prob(N.ptr(logits), N.ptr(act), N.ptr(high), N.ptr(low), M, A,
                                               N.ptr(logp), N.stream_of(act.device)), "mh_tanh_gauss_log_prob")
        ctx.save_for_backward(logits, act, high, low)
        return logp

    @staticmethod
    def backward(ctx, d_logp):
        logits, act, high, low = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        N = _native()
        M, A = act.shape
        d_logits = torch.empty_like(logits)
        N.check(N.lib().mh_tanh_gauss_log_prob_backward(
            N.ptr(logits), N.ptr(act), N.ptr(high), N.ptr(low), N.ptr(d_logp.contiguous()), M, A,
            N.ptr(d_logits), N.stream_of(logits.device)), "mh_tanh_gauss_log_prob_backward")
        return d_logits, None, None, None


class TanhGaussDistribution:
    """a = (h-l)/2 * tanh(z) + (h+l)/2, z ~ N(mean, std); log-prob with the tanh Jacobian."""

    def __init__(self, logits):
        self.logits = logits
        self.mean, self.std = torch.chunk(logits, chunks=2, dim=-1)
        self.gauss_distribution = _independent_normal(self.mean, self.std)
        self.act_high_lim = torch.tensor([1.0])
        self.act_low_lim = torch.tensor([-1.0])

    def _squash(self, z):
        half = (self.act_high_lim - self.act_low_lim) / 2
        mid = (self.act_high_lim + self.act_low_lim) / 2
        return half * torch.tanh(z) + mid

    def _logp_of_pre_tanh(self, z):
        return (self.gauss_distribution.log_prob(z)
                - torch.log(1 + EPS - torch.pow(torch.tanh(z), 2)).sum(-1)
                - torch.log((self.act_high_lim - self.act_low_lim) / 2).sum(-1))

    def sample(self):
        z = self.gauss_distribution.sample()
        return self._squash(z), self._logp_of_pre_tanh(z)

    def _fused_bounds(self):
        """(logits2d, high, low) when the device kernels apply, else None."""
        lg = self.logits
        if not (lg.is_cuda and lg.dtype == torch.float32 and lg.dim() >= 1):
            return None
        A = lg.shape[-1] // 2
        hi, lo = self.act_high_lim, self.act_low_lim
        if not (0 < A <= 8 and lg.shape[-1] == 2 * A and hi.shape == (A,) and lo.shape == (A,)
                and hi.dtype == torch.float32 and lo.dtype == torch.float32
                and hi.device == lg.device and lo.device == lg.device):
            return None
        return lg.reshape(-1, 2 * A).contiguous(), hi.contiguous(), lo.contiguous()

    def rsample(self):
        fb = self._fused_bounds()
        if fb is not None:
            lg, hi, lo = fb
            eps = tdn._standard_normal(self.mean.shape, dtype=self.mean.dtype, device=self.mean.device)
            lead = self.mean.shape[:-1]
            act, logp = _TanhGaussRsample.apply(lg, eps.reshape(lg.shape[0], lg.shape[1] // 2).contiguous(), hi, lo)
            return act.reshape(self.mean.shape), logp.reshape(lead)
        z = self.gauss_distribution.rsample()
        return self._squash(z), self._logp_of_pre_tanh(z)

    def log_prob(self, action_limited):
        fb = self._fused_bounds()
        if fb is not None and action_limited.shape == self.mean.shape \
                and action_limited.dtype == torch.float32 and action_limited.device == self.logits.device \
                and not action_limited.requires_grad:
            lg, hi, lo = fb
            a = action_limited.reshape(lg.shape[0], lg.shape[1] // 2).contiguous()
            return _TanhGaussLogProb.apply(lg, a, hi, lo).reshape(self.mean.shape[:-1])
        z = torch.atanh((1 - EPS) * (2 * action_limited - (self.act_high_lim + self.act_low_lim))
                        / (self.act_high_lim - self.act_low_lim))
        return self.gauss_distribution.log_prob(z) - torch.log(
            (self.act_high_lim - self.act_low_lim) / 2 * (1 + EPS - torch.pow(torch.tanh(z), 2))).sum(-1)

    def entropy(self):
        return self.gauss_distribution.entropy()

    def mode(self):
        return self._squash(self.mean)

    def kl_divergence(self, other):
        return torch.distributions.kl.kl_divergence(self.gauss_distribution, other.gauss_distribution)


class GaussDistribution:
    """Unsquashed Gaussian; mode() clamps the mean to the action box."""

    def __init__(self, logits):
        self.logits = logits
        self.mean, self.std = torch.chunk(logits, chunks=2, dim=-1)
        self.gauss_distribution = _independent_normal(self.mean, self.std)
        self.act_high_lim = torch.tensor([1.0])
        self.act_low_lim = torch.tensor([-1.0])

    def sample(self):
        a = self.gauss_distribution.sample()
        return a, self.gauss_distribution.log_prob(a)

    def rsample(self):
        a = self.gauss_distribution.rsample()
        return a, self.gauss_distribution.log_prob(a)

    def log_prob(self, action):
        return self.gauss_distribution.log_prob(action)

    def entropy(self):
        return self.gauss_distribution.entropy()

    def mode(self):
        return torch.clamp(self.mean, self.act_low_lim, self.act_high_lim)

    def kl_divergence(self, other):
        return torch.distributions.kl.kl_divergence(self.gauss_distribution, other.gauss_distribution)


class DiracDistribution:
    """Deterministic policy output: the logits are the action, log-prob 0."""

    def __init__(self, logits):
        self.logits = logits

    def sample(self):
        return self.logits, torch.zeros_like(self.logits).sum(-1)

    def mode(self):
        return self.logits
