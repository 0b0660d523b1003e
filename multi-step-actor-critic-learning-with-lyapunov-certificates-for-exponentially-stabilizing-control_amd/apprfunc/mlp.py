"""MLP function approximators (RL/apprfunc/mlp.py:2-160). These stay PyTorch-ROCm modules
(hipBLASLt GEMMs); only their I/O layout matters to the HIP rollout ([E][obs_dim] rows in,
[E][2*act_dim] (mean | std) rows out)."""
__all__ = ["ActionValue", "StateValue", "LyapunovValue", "ActionValueDistri", "StochaPolicy", "DetermPolicy"]

import torch
import torch.nn as nn

from ..utils.act_distribution_cls import Action_Distribution_Cls
from ..utils.common_utils import get_activation_func
from ._fused import MLP, SquareSum, StochaHead


def mlp(sizes, activation, output_activation=nn.Identity):
    """Linear layers with `activation` between them and `output_activation` after the last
    (an nn.Sequential; on HIP tensors each layer runs fused, apprfunc/_fused.py)."""
    layers = []
    last = len(sizes) - 2
    for j, (a, b) in enumerate(zip(sizes[:-1], sizes[1:])):
        layers.append(nn.Linear(a, b))
        layers.append((output_activation if j == last else activation)())
    return MLP(*layers)


def _acts(kw):
    return get_activation_func(kw["hidden_activation"]), get_activation_func(kw["output_activation"])


class ActionValue(nn.Module):
    """Q(s, a) -> scalar."""

    def __init__(self, **kw):
        super().__init__()
        self.q = mlp([kw["obs_dim"] + kw["act_dim"]] + list(kw["hidden_sizes"]) + [1], *_acts(kw))

    def forward(self, obs, act):
        return self.q(torch.cat([obs, act], dim=-1)).squeeze(-1)


class StateValue(nn.Module):
    """V(s) -> scalar."""

    def __init__(self, **kw):
        super().__init__()
        self.v = mlp([kw["obs_dim"]] + list(kw["hidden_sizes"]) + [1], *_acts(kw))

    def forward(self, obs):
        return self.v(obs).squeeze(-1)


class LyapunovValue(nn.Module):
    """V(x) = ||MLP(x)||^2 (non-negative by construction)."""

    def __init__(self, **kw):
        super().__init__()
        self.lya = mlp([kw["input_dim"]] + list(kw["hidden_sizes"]) + [kw["output_dim"]], *_acts(kw))

    def forward(self, input_obs):
        if input_obs.is_cuda and input_obs.dtype == torch.float32:
            from ._fused import square_sum_mlp
            v = square_sum_mlp(self.lya, input_obs)  # the square sums inside the MLP's launches
            if v is not None:
                return v
        y = self.lya(input_obs)
        if y.is_cuda and y.dtype == torch.float32:
            return SquareSum.apply(y)  # one launch each way (apprfunc/_fused.py)
        return torch.pow(y, 2).sum(dim=-1, keepdim=True).squeeze(-1)


class ActionValueDistri(nn.Module):
    """Distributional Q: (mean, softplus std)."""

    def __init__(self, **kw):
        super().__init__()
        self.q = mlp([kw["obs_dim"] + kw["act_dim"]] + list(kw["hidden_sizes"]) + [2], *_acts(kw))

    def forward(self, obs, act):
        mean, std = torch.chunk(self.q(torch.cat([obs, act], dim=-1)), chunks=2, dim=-1)
        return torch.cat((mean, torch.nn.functional.softplus(std)), dim=-1)


class StochaPolicy(nn.Module, Action_Distribution_Cls):
    """obs -> (mean, exp(clamp(log_std))), consumed by TanhGaussDistribution (or the fused
    in-kernel sampler of the HIP rollout)."""

    def __init__(self, **kw):
        super().__init__()
        self.policy = mlp([kw["obs_dim"]] + list(kw["hidden_sizes"]) + [kw["act_dim"] * 2], *_acts(kw))
        self.min_log_std = kw["min_log_std"]
        self.max_log_std = kw["max_log_std"]
        self.register_buffer("act_high_lim", torch.from_numpy(kw["act_high_lim"]))
        self.register_buffer("act_low_lim", torch.from_numpy(kw["act_low_lim"]))
        self.action_distribution_cls = kw["action_distribution_cls"]

    def forward(self, obs):
        raw = self.policy(obs)
        if raw.is_cuda and raw.dtype == torch.float32:
            return StochaHead.apply(raw.contiguous(), float(self.min_log_std), float(self.max_log_std))
        mean, log_std = torch.chunk(raw, chunks=2, dim=-1)
        return torch.cat((mean, torch.clamp(log_std, self.min_log_std, self.max_log_std).exp()), dim=-1)


class DetermPolicy(nn.Module, Action_Distribution_Cls):
    """obs -> action squashed into the action box."""

    def __init__(self, **kw):
        super().__init__()
        self.pi = mlp([kw["obs_dim"]] + list(kw["hidden_sizes"]) + [kw["act_dim"]], *_acts(kw))
        self.register_buffer("act_high_lim", torch.from_numpy(kw["act_high_lim"]))
        self.register_buffer("act_low_lim", torch.from_numpy(kw["act_low_lim"]))
        self.action_distribution_cls = kw["action_distribution_cls"]

    def forward(self, obs):
        half = (self.act_high_lim - self.act_low_lim) / 2
        return half * torch.tanh(self.pi(obs)) + (self.act_high_lim + self.act_low_lim) / 2
