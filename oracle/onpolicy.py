"""CPU ORACLE — test infrastructure only (imported by tests/, never by the product package).

Restatement of the 1-step and on-policy sampler paths:
  * RL/trainer/sampler/base.py:225-298 (`_step`): one Experience per env per step, env-index
    order, done = terminated | truncated, real_next_obs substituted for finished envs.
  * RL/trainer/sampler/on_sampler.py:44-79 (`_sample`) and :108-154 (`_process_experiences`,
    `_finish_trajs`): [E][H] mini-batch arrays; per env, a trajectory segment ends at done or at
    t == H-1, its bootstrap is V(real_next_obs) * (1 - done); GAE is accumulated in float64
    (the value slice is np.append(float32 values, python float) -> float64) and the discounted
    return in float32 (NumPy-2 promotion: np.float32 + weak Python float stays float32).
"""
from __future__ import annotations

import numpy as np

from oracle import sampler as OS

F32 = np.float32


class OneStepRollout:
    """BaseSampler._step with injected (already clipped) actions and their log-probs."""

    def __init__(self, venv: OS.VectorEnv, reward_scale=100.0, cost_scale=100.0):
        self.venv = venv
        self.reward_scale = reward_scale
        self.cost_scale = cost_scale
        self.obs = venv.reset()

    def step(self, actions_clip, logp):
        next_obs, rewards, term, trunc, final_obs = self.venv.step(actions_clip)
        next_obs = np.float32(next_obs)
        original_rewards = np.float32(rewards)
        obs = np.float32(self.obs)
        dones = np.logical_or(term, trunc)
        real_next_obs = next_obs.copy()
        real_next_obs[dones] = final_obs[dones]
        rew, cost = OS.rew_plus_cost(real_next_obs, original_rewards, self.reward_scale, self.cost_scale)
        self.obs = next_obs
        return dict(obs=obs, act=np.asarray(actions_clip, F32), rew=rew, cost=cost, obs2=real_next_obs,
                    done=dones, logp=np.asarray(logp, F32))


def finish_trajs(val, val2, rew, done, gamma, gae_lambda):
    """_process_experiences' segment bookkeeping + _finish_trajs (on_sampler.py:120-154) for
    every env of a [E][H] block. val2[i, t] is V(real_next_obs) (only read at segment ends)."""
    E, H = rew.shape
    adv = np.zeros((E, H), F32)
    ret = np.zeros((E, H), F32)
    for i in range(E):
        last_ptr = -1
        for t in range(H):
            d = np.bool_(done[i, t])
            if d or t == H - 1:
                est_last_val = float(val2[i, t]) * (1 - d)
                path = slice(last_ptr + 1, t + 1)
                value_preds = np.append(val[i, path], est_last_val)
                rews = rew[i, path]
                length = len(rews)
                r_ = np.zeros(length)
                a_ = np.zeros(length)
                gae = 0.0
                G_t = 0
                for k in reversed(range(length)):
                    delta = rews[k] + gamma * value_preds[k + 1] - value_preds[k]
                    gae = delta + gamma * gae_lambda * gae
                    a_[k] = gae
                    G_t = rews[k] + gamma * G_t
                    r_[k] = G_t
                adv[i, path] = a_
                ret[i, path] = r_
                last_ptr = t
    return adv, ret


def onpolicy_trace(name, init_reset, init_steps, actions, logp, resets, reward_scale=100.0, cost_scale=100.0):
    """OnSampler mini-batch arrays ([E][H] / [E][H][dim]) for injected actions and resets."""
    E, H = init_reset.shape[0], actions.shape[0]
    t = {"t": -1}
    venv = OS.VectorEnv(name, E, lambda idx: init_reset[idx] if t["t"] < 0 else resets[t["t"]][idx])
    ro = OneStepRollout(venv, reward_scale, cost_scale)
    venv.steps[:] = init_steps
    cols = {k: [] for k in ("obs", "act", "rew", "cost", "obs2", "done", "logp")}
    for k in range(H):
        t["t"] = k
        x = ro.step(actions[k], logp[k])
        for key in cols:
            cols[key].append(x[key])
    return {k: np.stack(v, axis=1) for k, v in cols.items()}
