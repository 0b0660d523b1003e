"""Action distributions behind StochaPolicy/DetermPolicy (RL/utils/act_distribution_cls.py:15-159).

Same math and the same torch.distributions objects as the reference, so log-probabilities and
the reparameterised noise path (Normal.rsample -> _standard_normal) are identical. The device
rollout samples in-kernel instead (csrc/rollout.hip, TanhGauss + clip fused into the env step).
"""
import torch

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

    def rsample(self):
        z = self.gauss_distribution.rsample()
        return self._squash(z), self._logp_of_pre_tanh(z)

    def log_prob(self, action_limited):
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
