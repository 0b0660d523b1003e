"""Device 1-step off-policy sampler (drop-in for RL/trainer/sampler/off_sampler.py:8-26 +
BaseSampler._step, RL/trainer/sampler/base.py:225-298), the sampler of SAC / LAC.

`_step` produces one Experience per env per lockstep step, in env-index order; on the device
that is the n-step window path with n = 1 (every env emits every step, done = term | trunc,
real_next_obs substituted), so the same fused gfx950 rollout kernel (TanhGauss sample, clip,
env step, autoreset, rew_plus_cost) and emission kernel write each transition straight into
the bound HBM ReplayBuffer, and the whole horizon replays as one HIP graph.
"""
from .hip_nstep_off_sampler import HipNstepOffSampler

__all__ = ["OffSampler"]


class OffSampler(HipNstepOffSampler):
    def __init__(self, **kwargs):
        kw = dict(kwargs)
        kw["n_step"] = 1
        super().__init__(**kw)
