"""Deterministic-policy evaluation on the device env kernels (RL/trainer/evaluator.py:9-212).

Same metrics as the reference: parallel evaluation runs num_eval_episode envs in lockstep, one
episode each with the distribution's mode() action, and reports the mean/std over episodes of
the per-step MEAN scaled reward and cost (rew_plus_cost scales); sequential evaluation runs
episodes on one env and reports mean/std of the episode SUMS. The rollout is the HIP env step
kernel; per-episode means accumulate on the device in float64 (the reference's np.mean of a
float32 list sums pairwise in float32), episode sums in float32 in step order exactly like the
reference's sum(); completion is checked on the host once every 8 lockstep steps. With an
explicit device="cpu" the same loop runs on the engine's CPU build (env/host_vector_env.py).
"""
import numpy as np
import torch

from ..create_pkg.create_alg import create_approx_contrainer
from ..env.host_vector_env import make_vector_env


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
        self.envs = make_vector_env(self.env_id, env_num, seed=int(self.seed) + 7919 * (index + 1), device=self.device)
        self.networks = create_approx_contrainer(**kwargs)
        self.render = kwargs.get("is_render", False)
        self.action_type = kwargs["action_type"]
        self.policy_func_name = kwargs["policy_func_name"]
        self.save_folder = kwargs.get("save_folder")
        self.max_eval_steps = int(kwargs.get("max_eval_steps", 1000))

    def close(self):
        """Release the evaluation envs' device handle (idempotent)."""
        close = getattr(self.envs, "close", None)
        if close is not None:
            close()

    def load_state_dict(self, state_dict):
        self.networks.load_state_dict(state_dict)

    @torch.no_grad()
    def _episodes(self, initial_states=None):
        """Run every env until its first episode ends (mode() actions). Returns per-env sums of
        the scaled reward and cost over the episode and the episode lengths (float64).
        `initial_states` [E][reset_dim] injects the initial states (parity mode); resets after
        an env's episode ended do not enter the metric, so they are never injected."""
        obs, _ = self.envs.reset(reset_states=initial_states)
        E = self.envs.num_envs
        dev = self.device
        sum_r = torch.zeros(E, dtype=torch.float64, device=dev)
        sum_c = torch.zeros(E, dtype=torch.float64, device=dev)
        cnt = torch.zeros(E, dtype=torch.float64, device=dev)
        # float32 running sums in step order: the reference's run_an_episode uses Python's
        # sum() over float32 scalars (evaluator.py:114-115), i.e. sequential float32 adds
        sum_r32 = torch.zeros(E, dtype=torch.float32, device=dev)
        sum_c32 = torch.zeros(E, dtype=torch.float32, device=dev)
        finished = torch.zeros(E, dtype=torch.bool, device=dev)
        for k in range(self.max_eval_steps + 1):
            act = self.networks.create_action_distributions(self.networks.policy(obs)).mode().float().contiguous()
            nxt, rew, term, trunc, info = self.envs.step(act)
            real = info["final_observation"]
            r = rew * self.reward_scale                                  # rew_plus_cost.py:18-21
            c = (real ** 2).sum(dim=1) * self.cost_scale
            live = (~finished).double()
            sum_r += r.double() * live
            sum_c += c.double() * live
            sum_r32 = torch.where(finished, sum_r32, sum_r32 + r)
            sum_c32 = torch.where(finished, sum_c32, sum_c32 + c)
            cnt += live
            finished |= term | trunc
            obs = nxt
            if k % 8 == 7 and bool(finished.all()):  # one host sync per 8 lockstep steps
                break
        self._last_sums32 = (sum_r32, sum_c32)
        return sum_r, sum_c, cnt

    def run_parallel_episodes(self, initial_states=None):
        """evaluator.py:145-197: per-episode per-step-MEAN reward/cost, then mean/std over the
        num_eval_episode parallel episodes."""
        sum_r, sum_c, cnt = self._episodes(initial_states)
        ret = (sum_r / cnt.clamp_min(1)).cpu().numpy()
        cost = (sum_c / cnt.clamp_min(1)).cpu().numpy()
        return np.mean(ret), np.std(ret), np.mean(cost), np.std(cost)

    def run_an_episode(self, iteration, render=False, initial_state=None):
        """evaluator.py:59-117: episode SUM of reward and cost of env 0 (float32 running sum)."""
        self._episodes(initial_state)
        sum_r32, sum_c32 = self._last_sums32
        return float(sum_r32[0]), float(sum_c32[0])

    def run_n_episodes(self, n, iteration, initial_states=None):
        """evaluator.py:119-134: n sequential episodes, mean/std of their sums."""
        rets, costs = [], []
        for i in range(n):
            r, c = self.run_an_episode(iteration, self.render,
                                       None if initial_states is None else initial_states[i:i + 1])
            rets.append(r)
            costs.append(c)
        return np.mean(rets), np.std(rets), np.mean(costs), np.std(costs)

    def run_evaluation(self, iteration):
        if self.is_parallel_eval:
            return self.run_parallel_episodes()
        return self.run_n_episodes(self.num_eval_episode, iteration)
