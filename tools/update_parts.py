#!/usr/bin/env python3
"""Device time of the MSACL update and of its parts at the bench config (QuadTracking, 65,536
envs, B = 256, n = 20, 256-wide nets): the whole update as the trainer replays it (even and odd
iterations), and each part captured alone into a HIP graph and replayed (critic, Lyapunov,
one policy step, alpha, Polyak, replay sample + gather). Diagnostic only."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(4):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()

    def timeit(fn, reps=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3  # us

    batch = buffer.sample_batch(256)
    res = {}
    it = {"i": 0}

    def upd_even():
        alg.model_update(batch, 0)

    def upd_odd():
        alg.model_update(batch, 1)
    res["update_even"] = timeit(upd_even)
    res["update_odd"] = timeit(upd_odd)
    res["sample_batch"] = timeit(lambda: buffer.sample_batch(256))
    data = alg._static

    def part(fn):
        g = torch.cuda.CUDAGraph()
        fn()  # warm (lazy state)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        return timeit(g.replay)
    res["critic(q_update)"] = part(lambda: alg._q_update(data))
    res["lyapunov"] = part(lambda: alg._lyapunov_update(data))
    res["policy_step"] = part(lambda: alg._policy_update(data))
    res["polyak"] = part(lambda: alg._target_update())
    for k, v in res.items():
        print(f"{k:20s} {v:9.1f} us")


if __name__ == "__main__":
    main()
