#!/usr/bin/env python3
"""Kernel mix of the MSACL replay + update phase alone (for rocprofv3 --kernel-trace --stats):
the bench's pipeline (QuadTracking, 65,536 envs, B = 256, n = 20), 3 warm trainer steps, then
`--updates` (replay sample_batch + model_update) iterations, graph-replayed like the bench."""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--updates", type=int, default=20)
    p.add_argument("--envs", type=int, default=65536)
    a = p.parse_args()
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=a.envs, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(3):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    for i in range(a.updates):
        batch = buffer.sample_batch(256)
        alg.model_update(batch, trainer.iteration + i)
    end.record()
    torch.cuda.synchronize()
    print(f"update phase: {start.elapsed_time(end) / a.updates:.3f} ms per iteration")


if __name__ == "__main__":
    main()
