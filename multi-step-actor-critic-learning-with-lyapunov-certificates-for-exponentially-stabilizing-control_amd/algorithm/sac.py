"""SAC (RL/algorithm/sac.py:26-217) on the MI355X engine.

Same networks, losses, update order and hyper-parameters as the reference: twin Q with Polyak
targets, a TanhGauss StochaPolicy, and an auto-tuned log_alpha; the policy (and alpha) update
runs `policy_frequency` times every `policy_frequency` iterations (:86-112). Device-side
differences only: alpha enters the losses as a 0-d device tensor instead of `alpha.item()`
(the same float32 value, no host sync), Adam is the fused capturable kernel, and the whole
update is replayed as one HIP graph per (update-target, update-policy) branch. Gradients are
averaged across ranks (RCCL) before every optimiser step when torch.distributed is up.
"""
__all__ = ["ApproxContainer", "SAC"]

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
    """q1, q2 (+ frozen targets), policy, log_alpha and their optimisers (sac.py:26-54)."""

    def __init__(self, **kwargs):
        super().__init__()
        q_args = get_apprfunc_dict("value", **kwargs)
        self.q1: nn.Module = create_apprfunc(**q_args)
        self.q2: nn.Module = create_apprfunc(**q_args)
        self.q1_target = deepcopy(self.q1)
        self.q2_target = deepcopy(self.q2)
        set_requires_grad((self.q1_target, self.q2_target), False)
        self.policy: nn.Module = create_apprfunc(**get_apprfunc_dict("policy", **kwargs))
        self.log_alpha = nn.Parameter(torch.tensor(1, dtype=torch.float32))
        self._lrs = (kwargs["q_learning_rate"], kwargs["policy_learning_rate"], kwargs["alpha_learning_rate"])
        self.make_optimizers()

    def make_optimizers(self):
        q_lr, pi_lr, a_lr = self._lrs
        self.q1_optimizer = fused_adam(self.q1.parameters(), q_lr)
        self.q2_optimizer = fused_adam(self.q2.parameters(), q_lr)
        self.policy_optimizer = fused_adam(self.policy.parameters(), pi_lr)
        self.alpha_optimizer = fused_adam([self.log_alpha], a_lr)

    def create_action_distributions(self, logits):
        return self.policy.get_act_dist_cls(logits)


class SAC:
    def __init__(self, gamma: float = 0.99, tau: float = 0.005, alpha: float = math.e, auto_alpha: bool = True,
                 target_entropy: Optional[float] = None, policy_frequency: int = 2,
                 target_network_frequency: int = 1, **kwargs: Any):
        dev = kwargs.get("device")
        if dev is None and torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(dev) if dev is not None else torch.device("cpu")
        self.networks = ApproxContainer(**kwargs).to(self.device)
        if self.device.type == "cuda":
            self.networks.make_optimizers()  # capturable Adam state must live with the params
        self.gamma = gamma
        self.tau = tau
        with torch.no_grad():
            self.networks.log_alpha.fill_(math.log(alpha))
        self.auto_alpha = auto_alpha
        self.target_entropy = target_entropy if target_entropy else -kwargs["act_dim"]
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

    def model_update(self, data: Dict[str, torch.Tensor], global_iteration: int):
        start = time.time()
        data = {k: v.to(self.device).contiguous() for k, v in data.items() if torch.is_tensor(v)}
        key = (global_iteration % self.target_network_frequency == 0, global_iteration % self.policy_frequency == 0)
        loss_q, q1, q2, loss_policy, entropy = self._graph(data, key)
        if not key[1]:
            return None
        vals = torch.stack([q1, q2, entropy, self.networks.log_alpha.detach().exp(), loss_q, loss_policy]).tolist()
        return {
            "SAC/critic_q1-RL iter": vals[0],
            "SAC/critic_q2-RL iter": vals[1],
            "SAC/entropy-RL iter": vals[2],
            "SAC/alpha-RL iter": vals[3],
            tb_tags["loss_critic"]: vals[4],
            tb_tags["loss_actor"]: vals[5],
            tb_tags["alg_time"]: (time.time() - start) * 1000,
        }

    def _update_body(self, data, do_target, do_policy):
        loss_q, q1, q2 = self._q_update(data)
        if do_target:
            self._target_update()
        loss_policy = entropy = None
        if do_policy:
            for _ in range(self.policy_frequency):
                dist = self.networks.create_action_distributions(self.networks.policy(data["obs"]))
                new_act, new_logp = dist.rsample()
                loss_policy, entropy = self._policy_update(data["obs"], new_act, new_logp)
                if self.auto_alpha:
                    self._alpha_update(new_logp)
        return loss_q, q1, q2, loss_policy, entropy

    def _q_update(self, data):
        obs, act, rew, obs2, done = data["obs"], data["act"], data["rew"], data["obs2"], data["done"]
        q1 = self.networks.q1(obs, act)
        q2 = self.networks.q2(obs, act)
        with torch.no_grad():
            next_dist = self.networks.create_action_distributions(self.networks.policy(obs2))
            next_act, next_logp = next_dist.rsample()
            next_q = torch.min(self.networks.q1_target(obs2, next_act), self.networks.q2_target(obs2, next_act))
            alpha = self.networks.log_alpha.detach().exp()
            backup = rew + (1 - done) * self.gamma * (next_q - alpha * next_logp)
        loss_q = ((q1 - backup) ** 2).mean() + ((q2 - backup) ** 2).mean()
        self.networks.q1_optimizer.zero_grad()
        self.networks.q2_optimizer.zero_grad()
        loss_q.backward()
        step(self.networks.q1_optimizer, self.networks.q1.parameters())
        step(self.networks.q2_optimizer, self.networks.q2.parameters())
        return loss_q.detach(), q1.detach().mean(), q2.detach().mean()

    def _policy_update(self, obs, new_act, new_logp):
        set_requires_grad((self.networks.q1, self.networks.q2), False)
        q1 = self.networks.q1(obs, new_act)
        q2 = self.networks.q2(obs, new_act)
        loss_policy = (self._get_alpha(True) * new_logp - torch.min(q1, q2)).mean()
        self.networks.policy_optimizer.zero_grad()
        loss_policy.backward()
        step(self.networks.policy_optimizer, self.networks.policy.parameters())
        entropy = -new_logp.detach().mean()
        set_requires_grad((self.networks.q1, self.networks.q2), True)
        return loss_policy.detach(), entropy

    def _alpha_update(self, new_logp):
        alpha = self._get_alpha(True)
        loss_alpha = -alpha * (new_logp.detach() + self.target_entropy).mean()
        self.networks.alpha_optimizer.zero_grad()
        loss_alpha.backward()
        step(self.networks.alpha_optimizer, [self.networks.log_alpha])

    def _target_update(self):
        polyak_(self.networks.q1, self.networks.q1_target, self.tau)
        polyak_(self.networks.q2, self.networks.q2_target, self.tau)
