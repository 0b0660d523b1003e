"""TensorBoard tag table (identical tag strings to RL/utils/tensorboard_setup.py:13-40) and a
writer factory: torch's SummaryWriter when tensorboard is installed, otherwise an in-memory
writer with the same add_scalar/flush/close surface (tensorboard is absent from this image)."""
tb_tags = {
    "TRM of RL iteration": "Evaluation/1-1. TRM-RL iter",
    "TRS of RL iteration": "Evaluation/1-1. TRS-RL iter",
    "TRM of total time": "Evaluation/2-1. TRM-Total time [s]",
    "TRM of collected samples": "Evaluation/3-1. TRM-Collected samples",
    "TRM of replay samples": "Evaluation/4-1. TRM-Replay samples",
    "TCM of RL iteration": "Evaluation/1-2. TCM-RL iter",
    "TCS of RL iteration": "Evaluation/1-2. TCS-RL iter",
    "TCM of total time": "Evaluation/2-2. TCM-Total time [s]",
    "TCM of collected samples": "Evaluation/3-2. TCM-Collected samples",
    "TCM of replay samples": "Evaluation/4-2. TCM-Replay samples",
    "Buffer RAM of RL iteration": "RAM/RAM [MB]-RL iter",
    "loss_actor": "Loss/Actor loss-RL iter",
    "loss_critic": "Loss/Critic loss-RL iter",
    "loss_entropy": "Loss/Entropy loss-RL iter",
    "loss_lyapunov": "Loss/Lyapunov loss-RL iter",
    "alg_time": "Time/Algorithm time [ms]-RL iter",
    "sampler_time": "Time/Sampler time [ms]-RL iter",
    "env_steps_per_sec": "Time/Env steps per second-RL iter",
}


class MemoryWriter:
    """Minimal SummaryWriter stand-in for runs without tensorboard: keeps scalars in memory."""

    def __init__(self, log_dir=None, flush_secs=20):
        self.log_dir = log_dir
        self.scalars = {}

    def add_scalar(self, tag, value, step):
        self.scalars.setdefault(tag, []).append((int(step), float(value)))

    def flush(self):
        pass

    def close(self):
        pass


def make_writer(log_dir, flush_secs=20):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=flush_secs)
    except Exception:
        return MemoryWriter(log_dir, flush_secs)


def add_scalars(tb_info, writer, step):
    for key, value in tb_info.items():
        writer.add_scalar(key, value, step)
