"""`buffer_name="nstep_replay_buffer"` (the reference default) resolves to the HBM buffer; an
explicit device="cpu" (BASELINE.json config 1) to the host buffer."""
import torch

from .device_nstep_replay_buffer import DeviceNstepReplayBuffer


class NstepReplayBuffer(DeviceNstepReplayBuffer):
    def __new__(cls, **kwargs):
        dev = kwargs.get("device")
        if dev is not None and torch.device(dev).type == "cpu":
            from .host_nstep_replay_buffer import HostNstepReplayBuffer
            return HostNstepReplayBuffer(**kwargs)
        return super().__new__(cls)
