"""Deterministic-policy evaluation on the device env kernels (RL/trainer/evaluator.py:9-212).

Same metric as the reference: every eval env runs one episode with the distribution's mode()
action; per-episode per-step-mean reward and cost (rew_plus_cost scales), then mean/std over
episodes. The rollout is the HIP env step; the loop checks completion on the host each step.
"""
import numpy as np
import torch

from ..create_pkg.create_alg import create_approx_contrainer
from ..env.hip_vector_env import HipVectorEnv


class Evaluator:
    def __init__(self, index=0, **kwargs):
        self.seed = kwargs.get("eval_env_seed", 2)
        self.env_id = kwargs["env_name"]
        self.reward_scale = kwargs["reward_scale"]
        self.cost_scale = kwargs["cost_scale"]
        self.target_value = kwargs.get("target_value", 0.0)
        self.num_eval_episode = int(kwargs["num_eval_episode"])
        self.is_parallel_eval = kwargs.get("is_parallel_eval", True)
        dev = kwargs.get("device")
        self.device = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
        env_num = self.num_eval_episode if self.is_parallel_eval else 1
        self.envs = HipVectorEnv(self.env_id, env_num, seed=int(self.seed) + 7919 * (index + 1), device=self.device)
        self.networks = create_approx_contrainer(**kwargs)
        self.render = kwargs.get("is_render", False)
        self.action_type = kwargs["action_type"]
        self.policy_func_name = kwargs["policy_func_name"]
        self.save_folder = kwargs.get("save_folder")
        self.max_eval_steps = int(kwargs.get("max_eval_steps", 1000))

    def load_state_dict(self, state_dict):
        self.networks.load_state_dict(state_dict)

    @torch.no_grad()
    def _episodes(self):
        obs, _ = self.envs.reset()
        E = self.envs.num_envs
        dev = self.device
        sum_r = torch.zeros(E, dtype=torch.float64, device=dev)
        sum_c = torch.zeros(E, dtype=torch.float64, device=dev)
        cnt = torch.zeros(E, dtype=torch.float64, device=dev)
        finished = torch.zeros(E, dtype=torch.bool, device=dev)
        for _ in range(self.max_eval_steps + 1):
            act = self.networks.create_action_distributions(self.networks.policy(obs)).mode().float().contiguous()
            nxt, rew, term, trunc, info = self.envs.step(act)
            real = info["final_observation"]
            r = rew * self.reward_scale
            c = (real ** 2).sum(dim=1) * self.cost_scale
            live = (~finished).double()
            sum_r += r.double() * live
            sum_c += c.double() * live
            cnt += live
            finished |= term | trunc
            obs = nxt
            if bool(finished.all()):
                break
        ret = (sum_r / cnt.clamp_min(1)).cpu().numpy()
        cost = (sum_c / cnt.clamp_min(1)).cpu().numpy()
        return ret, cost

    def run_parallel_episodes(self):
        ret, cost = self._episodes()
        return np.mean(ret), np.std(ret), np.mean(cost), np.std(cost)

    def run_n_episodes(self, n, iteration):
        rets, costs = [], []
        for _ in range(n):
            r, c = self._episodes()
            rets.append(float(r[0]))
            costs.append(float(c[0]))
        return np.mean(rets), np.std(rets), np.mean(costs), np.std(costs)

    def run_evaluation(self, iteration):
        if self.is_parallel_eval:
            return self.run_parallel_episodes()
        return self.run_n_episodes(self.num_eval_episode, iteration)
