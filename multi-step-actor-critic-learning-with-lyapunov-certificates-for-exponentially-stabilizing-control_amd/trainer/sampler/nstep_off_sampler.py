"""`sampler_name="nstep_off_sampler"` (the reference default, RL/trainer/sampler/
nstep_off_sampler.py) resolves to the device sampler, so unchanged configs get the HIP path. An
explicit device="cpu" (BASELINE.json config 1) selects the engine's CPU build instead."""
import torch

from .hip_nstep_off_sampler import HipNstepOffSampler


class NstepOffSampler(HipNstepOffSampler):
    def __new__(cls, **kwargs):
        dev = kwargs.get("device")
        if dev is not None and torch.device(dev).type == "cpu":
            from .cpu_nstep_off_sampler import CpuNstepOffSampler
            return CpuNstepOffSampler(**kwargs)
        return super().__new__(cls)
