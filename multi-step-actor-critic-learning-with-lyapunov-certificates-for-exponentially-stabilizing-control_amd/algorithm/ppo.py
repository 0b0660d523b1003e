"""PPO (RL/algorithm/ppo.py:25-283) on the MI355X engine.

The on-policy mini-batch update of the reference, on device tensors: the advantage is
normalised once per sample batch, then `num_repeat` passes each shuffle the sample indices
with NumPy's global RNG (`np.random.shuffle`, :167 — the same host draw, so the same
permutation for the same seed) and take `num_mini_batch` mini-batches, each a policy step
(clipped surrogate + entropy + KL to the pre-update policy, :221-250) and a value step
(optionally clipped, :253-283). The permutation is uploaded once per pass and mini-batches are
gathered on the device. The Lyapunov network exists (and its lr is annealed) as in the
reference but PPO never trains it. Data-parallel (one rank per GPU, each with its own envs):
gradients are averaged across ranks (one RCCL all-reduce per optimiser step) and the advantage
normalisation uses the global batch's statistics; each rank shuffles its local indices.
"""
__all__ = ["ApproxContainer", "PPO"]

import time
from typing import Dict

import numpy as np
import torch
import torch.nn as nn

from ..create_pkg.create_apprfunc import create_apprfunc
from ..utils import dist as D
from ..utils.common_utils import get_apprfunc_dict
from ..utils.tensorboard_setup import tb_tags
from ._update_graph import fused_adam, step


def batch_normalize(x, eps):
    """(x - mean) / (std + eps) with torch's unbiased std (ppo.py:162). Under torch.distributed the
    statistics are the GLOBAL batch's: (sum, sum of squares, count) are all-reduced (float64), so
    data-parallel ranks normalise exactly like one process holding the whole sample batch."""
    if D.world_size() == 1:
        return (x - x.mean()) / (x.std() + eps)
    xd = x.double()
    st = torch.stack([xd.sum(), (xd * xd).sum(), torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device)])
    D.allreduce_(st)
    n = st[2]
    mean = st[0] / n
    std = ((st[1] - n * mean * mean) / (n - 1)).clamp_min(0).sqrt()
    return (x - mean.to(x.dtype)) / (std.to(x.dtype) + eps)


class ApproxContainer(nn.Module):
    """value, lyapunov, policy and their Adams (ppo.py:25-50)."""

    def __init__(self, **kwargs):
        super().__init__()
        self.value: nn.Module = create_apprfunc(**get_apprfunc_dict("value", **kwargs))
        self.lyapunov: nn.Module = create_apprfunc(**get_apprfunc_dict("lyapunov", **kwargs))
        self.policy: nn.Module = create_apprfunc(**get_apprfunc_dict("policy", **kwargs))
        self._lrs = (kwargs["learning_rate"], kwargs["policy_learning_rate"])
        self.make_optimizers()

    def make_optimizers(self):
        lr, pi_lr = self._lrs
        self.value_optimizer = fused_adam(self.value.parameters(), lr)
        self.lyapunov_optimizer = fused_adam(self.lyapunov.parameters(), lr)
        self.policy_optimizer = fused_adam(self.policy.parameters(), pi_lr)

    def create_action_distributions(self, logits):
        return self.policy.get_act_dist_cls(logits)


class PPO:
    container_cls = ApproxContainer

    def __init__(self, *, max_iteration: int, num_repeat: int, num_mini_batch: int, mini_batch_size: int,
                 sample_batch_size: int, env_num: int, index: int = 0, gamma: float = 0.99, clip: float = 0.1,
                 beta: float = 0.2, lya_diff_scale: float = 1.0, lya_zero_scale: float = 20.0,
                 lya_positive_scale: float = 1.0, advantage_norm: bool = True, loss_value_clip: bool = True,
                 value_clip: float = 0.2, loss_value_norm: bool = False, loss_coefficient_kl: float = 0.2,
                 loss_coefficient_value: float = 1.0, loss_coefficient_entropy: float = 0.01,
                 schedule_adam: str = "None", schedule_clip: str = "None", **kwargs):
        dev = kwargs.get("device")
        if dev is None and torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(dev) if dev is not None else torch.device("cpu")
        self.max_iteration = max_iteration
        self.num_repeat = num_repeat
        self.num_mini_batch = num_mini_batch
        self.env_num = env_num
        self.sample_batch_size = sample_batch_size * self.env_num
        self.indices = np.arange(self.sample_batch_size)
        self.mini_batch_size = mini_batch_size * self.env_num
        self.gamma = gamma
        self.clip = clip
        self.clip_now = self.clip
        self.advantage_norm = advantage_norm
        self.loss_value_clip = loss_value_clip
        self.value_clip = value_clip
        self.loss_value_norm = loss_value_norm
        self.loss_coefficient_kl = loss_coefficient_kl
        self.loss_coefficient_value = loss_coefficient_value
        self.loss_coefficient_entropy = loss_coefficient_entropy
        self.schedule_adam = schedule_adam
        self.schedule_clip = schedule_clip
        self.lya_diff_scale = lya_diff_scale
        self.lya_zero_scale = lya_zero_scale
        self.lya_positive_scale = lya_positive_scale
        self.env_name = kwargs["env_name"]
        self.env_id = self.env_name
        self.target_value = kwargs["target_value"]
        self.networks = self.container_cls(**kwargs).to(self.device)
        if self.device.type == "cuda":
            self.networks.make_optimizers()
        self.learning_rate = kwargs["learning_rate"]
        self.policy_learning_rate = kwargs["policy_learning_rate"]
        self.EPS = 1e-8
        self.beta = beta
        self.global_iteration = 0

    @property
    def adjustable_parameters(self):
        return ("gamma", "clip", "advantage_norm", "loss_value_clip", "value_clip", "loss_value_norm",
                "loss_coefficient_kl", "loss_coefficient_value", "loss_coefficient_entropy", "schedule_adam",
                "schedule_clip")

    # ------------------------------------------------------------------ update
    def _prepare(self, data):
        data = {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in data.items()}
        if self.env_id == "HalfCheetah-v4":
            data["obs"][:, 8] -= self.target_value
            data["obs2"][:, 8] -= self.target_value
        with torch.no_grad():
            data["logits"] = self.networks.policy(data["obs"])
        data["adv"] = batch_normalize(data["adv"], self.EPS)
        return data

    def _before_minibatches(self, data):
        """Hook for POLYC (Lyapunov update + hybrid advantage)."""
        return data

    def model_update(self, data: Dict[str, torch.Tensor]):
        start = time.perf_counter()
        data = self._before_minibatches(self._prepare(data))
        keys = ("obs", "act", "logp", "adv", "logits", "ret", "val")
        loss_policy = loss_value = None
        for _ in range(self.num_repeat):
            np.random.shuffle(self.indices)
            perm = torch.from_numpy(self.indices).to(self.device, non_blocking=True)
            for n in range(self.num_mini_batch):
                self.global_iteration += 1
                mb_idx = perm[self.mini_batch_size * n:self.mini_batch_size * (n + 1)]
                mb = {k: data[k].index_select(0, mb_idx) for k in keys}
                loss_policy = self._compute_loss_policy(mb, self.global_iteration)
                self.networks.policy_optimizer.zero_grad()
                loss_policy.backward()
                step(self.networks.policy_optimizer, self.networks.policy.parameters())
                loss_value = self._compute_loss_value(mb)
                self.networks.value_optimizer.zero_grad()
                loss_value.backward()
                step(self.networks.value_optimizer, self.networks.value.parameters())
                if self.schedule_adam == "linear":
                    decay = max(0.0, 1 - (self.global_iteration / self.max_iteration))
                    lr_now = self.learning_rate * decay
                    self.networks.lyapunov_optimizer.param_groups[0]["lr"] = lr_now
                    self.networks.value_optimizer.param_groups[0]["lr"] = lr_now
                    self.networks.policy_optimizer.param_groups[0]["lr"] = self.policy_learning_rate * decay
        end = time.perf_counter()
        vals = torch.stack([loss_policy.detach(), loss_value.detach()]).tolist()
        tb_info = {tb_tags["loss_actor"]: vals[0], tb_tags["loss_critic"]: vals[1],
                   tb_tags["alg_time"]: (end - start) * 1000}
        return tb_info, self.global_iteration

    def _compute_loss_lya(self, data):
        obs, obs2 = data["obs"], data["obs2"]
        if self.env_id == "HalfCheetah-v4":
            obs_zero = data["obs"].clone()
            obs_zero[:, 8] = 0
        else:
            obs_zero = torch.zeros_like(obs)
        loss_lya1 = torch.pow(self.networks.lyapunov(obs_zero), 2).mean() * self.lya_zero_scale
        diff = self.networks.lyapunov(obs2) - self.networks.lyapunov(obs)
        loss_lya3 = torch.max(diff, torch.zeros_like(diff)).mean() * self.lya_diff_scale
        return loss_lya1 + loss_lya3

    def _compute_loss_policy(self, data, global_iteration):
        obs, act, logp, advantages, logits = data["obs"], data["act"], data["logp"], data["adv"], data["logits"]
        new_dist = self.networks.create_action_distributions(self.networks.policy(obs))
        new_logp = new_dist.log_prob(act)
        old_dist = self.networks.create_action_distributions(logits)
        adv = advantages.detach()
        ratio = torch.exp(new_logp - logp)
        sur1 = ratio * adv
        sur2 = ratio.clamp(1 - self.clip_now, 1 + self.clip_now) * adv
        loss_surrogate = -torch.mean(torch.min(sur1, sur2))
        loss_entropy = -torch.mean(new_dist.entropy()) * self.loss_coefficient_entropy
        loss_kl = torch.mean(old_dist.kl_divergence(new_dist)) * self.loss_coefficient_kl
        loss_policy = loss_surrogate + loss_entropy + loss_kl
        if self.schedule_clip == "linear":
            self.clip_now = self.clip * (1 - (global_iteration / self.max_iteration))
        return loss_policy

    def _compute_loss_value(self, data):
        obs, returns, values = data["obs"], data["ret"], data["val"]
        new_value = self.networks.value(obs)
        ret = returns.detach()
        if self.loss_value_clip:
            l1 = torch.pow(new_value - ret, 2)
            clipped = values + (new_value - values).clamp(-self.value_clip, self.value_clip)
            l2 = torch.pow(clipped - ret, 2)
            losses = torch.max(l1, l2)
        else:
            losses = torch.pow(new_value - ret, 2)
        if self.loss_value_norm:
            return torch.mean(losses) / (6 * ret.std())
        return torch.mean(losses)
