"""`sampler_name="nstep_off_sampler"` (the reference default, RL/trainer/sampler/
nstep_off_sampler.py) resolves to the device sampler, so unchanged configs get the HIP path."""
from .hip_nstep_off_sampler import HipNstepOffSampler


class NstepOffSampler(HipNstepOffSampler):
    pass
