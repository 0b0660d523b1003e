"""POLYC (RL/algorithm/polyc.py:26-299) on the MI355X engine: PPO plus a self-learned almost
Lyapunov critic. Per sample batch, before the PPO mini-batch passes: one Lyapunov-risk step on
the whole batch (zero term + decrease hinge, :239-259), then the hybrid advantage
adv <- (1 - beta) adv + beta min(-norm(V(obs2) - V(obs)), 0) (:168-182).

One deliberate divergence: the reference builds the Lyapunov net with
`create_apprfunc(**kwargs)` (polyc.py:36), i.e. from the top-level config, which raises
KeyError('apprfunc') for every config its own example writes; here it is built from the
`lyapunov_*` config (get_apprfunc_dict("lyapunov")), as PPO's container does. With top-level
apprfunc/name/hidden keys equal to the lyapunov_* ones the two constructions coincide.
"""
__all__ = ["ApproxContainer", "POLYC"]

import torch

from ..utils.tensorboard_setup import tb_tags  # noqa: F401  (tb keys shared with PPO)
from ._update_graph import step
from .ppo import PPO, batch_normalize
from .ppo import ApproxContainer as _PPOContainer


class ApproxContainer(_PPOContainer):
    """value, lyapunov, policy and their Adams (polyc.py:26-50)."""


class POLYC(PPO):
    container_cls = ApproxContainer

    def _before_minibatches(self, data):
        loss_lya = self._compute_loss_lya(data)
        self.networks.lyapunov_optimizer.zero_grad()
        loss_lya.backward()
        step(self.networks.lyapunov_optimizer, self.networks.lyapunov.parameters())
        with torch.no_grad():
            data["lya"] = self.networks.lyapunov(data["obs"])
            data["lya2"] = self.networks.lyapunov(data["obs2"])
        d = batch_normalize(data["lya2"] - data["lya"], self.EPS)
        d = torch.min(-d, torch.zeros_like(d))
        data["diff_lya"] = d
        data["adv"] = (1 - self.beta) * data["adv"] + self.beta * d
        return data
