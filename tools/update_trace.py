#!/usr/bin/env python3
"""Timeline of single MSACL updates at the bench config, for a rocprofv3 kernel trace.

run:     rocprofv3 --kernel-trace -d gpurun_out/ut -o ut --output-format csv -- python3 tools/update_trace.py
analyse: python3 tools/update_trace.py --analyse <kernel_trace.csv>

The program replays the even and the odd update graph R times each, separated by host sleeps,
so each replay is an isolated burst in the trace; the analysis prints, for the median burst of
each kind, its span, the summed kernel time, and every kernel with its start offset, duration
and queue (the parallel graph branches land on different queues). Diagnostic only."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(reps=6):
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
    for _ in range(6):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()
    if os.environ.get("TRACE_WHAT") == "sample":  # sampler.sample() bursts instead of updates
        for _ in range(12):
            time.sleep(0.02)
            sampler.sample()
            torch.cuda.synchronize()
        print("done", flush=True)
        return
    batch = buffer.sample_batch(256)
    for it in (0, 1):
        for _ in range(reps):
            time.sleep(0.02)
            alg.model_update(batch, it)
            torch.cuda.synchronize()
        time.sleep(0.05)
    print("done", flush=True)


def analyse(path, gap_us=2000.0):
    import csv
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?")))
    ks.sort()
    bursts, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(c[1] for c in cur[-8:]) > gap_us * 1e3:
            bursts.append(cur)
            cur = [k]
        else:
            cur.append(k)
    bursts.append(cur)
    # the last 2 x reps bursts are the even / odd replays (earlier ones: pipeline warm-up)
    big = [b for b in bursts if len(b) > 40][-12:]
    for name, group in (("even", big[:6]), ("odd", big[6:])):
        if not group:
            continue
        spans = sorted((max(k[1] for k in b) - b[0][0], i) for i, b in enumerate(group))
        b = group[spans[len(spans) // 2][1]]
        t0 = b[0][0]
        span = max(k[1] for k in b) - t0
        busy = sum(k[1] - k[0] for k in b)
        print(f"== {name}: {len(b)} kernels, span {span / 1e3:.1f} us, summed kernel time {busy / 1e3:.1f} us")
        for s, e, n, q in b:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3}  {n[:100]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()
