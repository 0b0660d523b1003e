"""1-step off-policy serial trainer (RL/trainer/off_serial_trainer.py:18-158) for SAC / LAC.

The reference's OffSerialTrainer and NstepOffSerialTrainer run the same loop (warm-up fill,
then sample -> add_batch -> sample_batch -> model_update (PER: update_batch) -> log / save /
evaluate); only the sampler and buffer plugged in differ (off_sampler + replay_buffer). The
device-boundary differences are those of NstepOffSerialTrainer: networks stay on the sampler's
device, replay batches are already HBM tensors, the sampler emits into the bound buffer.
"""
from .nstep_off_serial_trainer import NstepOffSerialTrainer

__all__ = ["OffSerialTrainer"]


class OffSerialTrainer(NstepOffSerialTrainer):
    pass
