"""`buffer_name="nstep_replay_buffer"` (the reference default) resolves to the HBM buffer."""
from .device_nstep_replay_buffer import DeviceNstepReplayBuffer


class NstepReplayBuffer(DeviceNstepReplayBuffer):
    pass
