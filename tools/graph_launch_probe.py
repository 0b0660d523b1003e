#!/usr/bin/env python3
"""Is the replayed MSACL update bound by the host's graph launch? At the bench config, times the
even and the odd update graph (a) replayed back to back as the trainer does (HIP events around
R replays), (b) with the stream first parked on a GPU spin so the host has submitted every
replay before the device starts (tools/gputime.py: device time only), and (c) the host time of
one replay() call. (a) >> (b) with (c) ~ (a) means the GPU waits on the host's node
submission. Environment knobs of the HIP runtime are read from the environment the caller sets.
Diagnostic only (parameters are updated by every replay)."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    from tools.gputime import time_launches
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(6):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()
    res = {}
    for name, policy in (("even", True), ("odd", False)):
        flags = [k for k in alg._graphs if bool(k[1]) == policy]  # (do_target, do_policy)
        if not flags:
            continue
        flags = flags[0]
        fn = alg._graphs[flags][0].replay
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 30
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_back_to_back_us"] = e0.elapsed_time(e1) / reps * 1e3
        res[f"{name}_device_only_us"] = time_launches(fn, reps, host_us_per_call=1500.0, warm=2) * 1e3
        torch.cuda.synchronize()
        hs = []
        for _ in range(10):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            hs.append((time.perf_counter() - t) * 1e6)
        torch.cuda.synchronize()
        res[f"{name}_host_replay_call_us"] = sorted(hs)[len(hs) // 2]
        res[f"{name}_flags"] = str(flags)
    env = {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_HIP", "DEBUG_CLR", "GPU_MAX"))}
    print({"env": env, **{k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}}, flush=True)


if __name__ == "__main__":
    main()
