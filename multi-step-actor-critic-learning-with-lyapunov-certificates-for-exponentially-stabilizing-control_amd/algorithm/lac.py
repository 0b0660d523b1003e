"""LAC (RL/algorithm/lac.py:23-313) on the MI355X engine.

Two cost critics L1/L2 with Polyak targets, a TanhGauss policy, a Lyapunov-decrease
coefficient log_alpha and an entropy coefficient log_beta, updated in the reference's order:
L update on the 1-step cost backup (:169-205), target averaging, then `policy_frequency`
policy updates every `policy_frequency` iterations (:107-125), each followed (auto_alpha) by
the alpha and beta updates (:258-295). Device-side differences only: alpha/beta enter the
policy loss as detached 0-d device tensors instead of `.item()` floats (same float32 values),
fused capturable Adam, HIP-graph replay of the whole update, cross-rank gradient averaging.
"""
__all__ = ["ApproxContainer", "LAC"]

import math
import time
from copy import deepcopy
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from ..create_pkg.create_apprfunc import create_apprfunc
from ..utils.common_utils import get_apprfunc_dict
from ..utils.tensorboard_setup import tb_tags
from ._update_graph import UpdateGraph, fused_adam, polyak_, set_requires_grad, step


class ApproxContainer(nn.Module):
    """l1, l2 (+ frozen targets), policy, log_alpha, log_beta and optimisers (lac.py:23-63)."""

    def __init__(self, **kwargs):
        super().__init__()
        l_args = get_apprfunc_dict("value", **kwargs)
        self.l1: nn.Module = create_apprfunc(**l_args)
        self.l2: nn.Module = create_apprfunc(**l_args)
        self.l1_target = deepcopy(self.l1)
        self.l2_target = deepcopy(self.l2)
        set_requires_grad((self.l1_target, self.l2_target), False)
        self.policy: nn.Module = create_apprfunc(**get_apprfunc_dict("policy", **kwargs))
        self.log_alpha = nn.Parameter(torch.tensor(1, dtype=torch.float32))
        self.log_beta = nn.Parameter(torch.tensor(1, dtype=torch.float32))
        self._lrs = (kwargs["l_learning_rate"], kwargs["policy_learning_rate"], kwargs["alpha_learning_rate"],
                     kwargs["beta_learning_rate"])
        self.make_optimizers()

    def make_optimizers(self):
        l_lr, pi_lr, a_lr, b_lr = self._lrs
        self.l1_optimizer = fused_adam(self.l1.parameters(), l_lr)
        self.l2_optimizer = fused_adam(self.l2.parameters(), l_lr)
        self.policy_optimizer = fused_adam(self.policy.parameters(), pi_lr)
        self.alpha_optimizer = fused_adam([self.log_alpha], a_lr)
        self.beta_optimizer = fused_adam([self.log_beta], b_lr)

    def create_action_distributions(self, logits):
        return self.policy.get_act_dist_cls(logits)


class LAC:
    def __init__(self, gamma: float = 0.99, tau: float = 0.005, alpha3: float = 0.05, alpha: float = math.e,
                 beta: float = math.e, auto_alpha: bool = True, target_entropy: Optional[float] = None,
                 policy_frequency: int = 2, target_network_frequency: int = 1, **kwargs: Any):
        dev = kwargs.get("device")
        if dev is None and torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(dev) if dev is not None else torch.device("cpu")
        self.networks = ApproxContainer(**kwargs).to(self.device)
        if self.device.type == "cuda":
            self.networks.make_optimizers()
        self.gamma = gamma
        self.tau = tau
        self.alpha3 = alpha3
        with torch.no_grad():
            self.networks.log_alpha.fill_(math.log(alpha))
            self.networks.log_beta.fill_(math.log(beta))
        self.auto_alpha = auto_alpha
        self.target_entropy = -kwargs["act_dim"] if target_entropy is None else target_entropy
        self.policy_frequency = policy_frequency
        self.target_network_frequency = target_network_frequency
        self._graph = UpdateGraph(self._update_body, enabled=bool(kwargs.get("alg_use_graph", True)))

    def close(self):
        """Release the captured update graphs deterministically (idempotent)."""
        self._graph.close()

    @property
    def adjustable_parameters(self):
        return ("gamma", "tau", "alpha", "auto_alpha", "target_entropy")

    def _get_alpha(self, requires_grad: bool = False):
        alpha = self.networks.log_alpha.exp()
        return alpha if requires_grad else alpha.item()

    def _get_beta(self, requires_grad: bool = False):
        beta = self.networks.log_beta.exp()
        return beta if requires_grad else beta.item()

    def model_update(self, data: Dict[str, torch.Tensor], global_iteration: int):
        start = time.time()
        data = {k: v.to(self.device).contiguous() for k, v in data.items() if torch.is_tensor(v)}
        key = (global_iteration % self.target_network_frequency == 0, global_iteration % self.policy_frequency == 0)
        loss_l, l1, l2, loss_policy, entropy = self._graph(data, key)
        if not key[1]:
            return None
        vals = torch.stack([l1, l2, entropy, self.networks.log_alpha.detach().exp(),
                            self.networks.log_beta.detach().exp(), loss_l, loss_policy]).tolist()
        return {
            "LAC/critic_l1-RL iter": vals[0],
            "LAC/critic_l2-RL iter": vals[1],
            "LAC/entropy-RL iter": vals[2],
            "LAC/alpha-RL iter": vals[3],
            "LAC/beta-RL iter": vals[4],
            tb_tags["loss_critic"]: vals[5],
            tb_tags["loss_actor"]: vals[6],
            tb_tags["alg_time"]: (time.time() - start) * 1000,
        }

    def _update_body(self, data, do_target, do_policy):
        loss_l, l1, l2 = self._l_update(data)
        if do_target:
            self._target_update()
        loss_policy = entropy = None
        if do_policy:
            for _ in range(self.policy_frequency):
                dist = self.networks.create_action_distributions(self.networks.policy(data["obs2"]))
                next_act, next_logp = dist.rsample()
                loss_policy, entropy, l_val, next_l_val = self._policy_update(data, next_act, next_logp)
                if self.auto_alpha:
                    self._alpha_update(l_val, next_l_val, data["cost"])
                    self._beta_update(entropy)
        return loss_l, l1, l2, loss_policy, entropy

    def _l_update(self, data):
        obs, act, cost, obs2, done = data["obs"], data["act"], data["cost"], data["obs2"], data["done"]
        l1 = self.networks.l1(obs, act)
        l2 = self.networks.l2(obs, act)
        with torch.no_grad():
            next_dist = self.networks.create_action_distributions(self.networks.policy(obs2))
            next_act, _ = next_dist.rsample()
            next_l = torch.min(self.networks.l1_target(obs2, next_act), self.networks.l2_target(obs2, next_act))
            backup = cost + (1 - done) * self.gamma * next_l
        loss_l = ((l1 - backup) ** 2).mean() + ((l2 - backup) ** 2).mean()
        self.networks.l1_optimizer.zero_grad()
        self.networks.l2_optimizer.zero_grad()
        loss_l.backward()
        step(self.networks.l1_optimizer, self.networks.l1.parameters())
        step(self.networks.l2_optimizer, self.networks.l2.parameters())
        return loss_l.detach(), l1.detach().mean(), l2.detach().mean()

    def _policy_update(self, data, next_act, next_logp):
        set_requires_grad((self.networks.l1, self.networks.l2), False)
        obs, act, cost, obs2 = data["obs"], data["act"], data["cost"], data["obs2"]
        l_min = torch.min(self.networks.l1(obs, act), self.networks.l2(obs, act))
        next_l_min = torch.min(self.networks.l1(obs2, next_act), self.networks.l2(obs2, next_act))
        alpha = self.networks.log_alpha.detach().exp()
        beta = self.networks.log_beta.detach().exp()
        loss_stability = alpha * (next_l_min - l_min + self.alpha3 * cost).mean()
        loss_entropy = beta * (next_logp.mean() + self.target_entropy)
        loss_policy = loss_stability + loss_entropy
        entropy = -next_logp.detach().mean()
        self.networks.policy_optimizer.zero_grad()
        loss_policy.backward()
        step(self.networks.policy_optimizer, self.networks.policy.parameters())
        set_requires_grad((self.networks.l1, self.networks.l2), True)
        return loss_policy.detach(), entropy, l_min.detach(), next_l_min.detach()

    def _alpha_update(self, l_val, next_l_val, cost):
        alpha = self._get_alpha(True)
        loss_alpha = -alpha * (next_l_val - l_val + self.alpha3 * cost).mean()
        self.networks.alpha_optimizer.zero_grad()
        loss_alpha.backward()
        step(self.networks.alpha_optimizer, [self.networks.log_alpha])

    def _beta_update(self, entropy):
        beta = self._get_beta(True)
        loss_beta = beta * (entropy - self.target_entropy)
        self.networks.beta_optimizer.zero_grad()
        loss_beta.backward()
        step(self.networks.beta_optimizer, [self.networks.log_beta])

    def _target_update(self):
        polyak_(self.networks.l1, self.networks.l1_target, self.tau)
        polyak_(self.networks.l2, self.networks.l2_target, self.tau)
