"""Probe: where the synchronised replay + update phase (bench.py phases.replay_and_update_ms) spends
its time. Per step: host time of the replay draw, host time of model_update up to and inside the
graph replay, the device's first-kernel delay (HIP event recorded before any launch vs the replay
draw's completion) and the device time to the end of the update."""
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

dev = torch.device("cuda", 0)
cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, env_seed=1, seed=0, sample_batch_size=20, n_step=20,
                         replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                         max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                         apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), num_eval_episode=1,
                         sampler_sync_timing=False, device=dev)
_a, alg, sampler, buffer, _e, trainer = build_pipeline(cfg)
for _ in range(8):
    trainer.step()
    trainer.iteration += 1

# wrap each captured graph's replay with a host timer
rep_t = []
for key, (g, outs, prio) in alg._graphs.items():
    orig = g.replay

    def timed(o=orig):
        t = time.perf_counter()
        o()
        rep_t.append(time.perf_counter() - t)
    g.replay = timed

rows = []
for it in range(12):
    samples, _ = sampler.sample()
    buffer.add_batch(samples)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    t0 = time.perf_counter()
    e0.record()
    drawn = trainer._drawn_update()
    rs = None if drawn else trainer._replay_batch()
    e1.record()
    t1 = time.perf_counter()
    n_rep = len(rep_t)
    trainer._update(rs)
    t2 = time.perf_counter()
    e2.record()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    trainer.iteration += 1
    rows.append({"policy_step": (trainer.iteration - 1) % alg.policy_frequency == 0,
                 "host_replay_draw_us": round((t1 - t0) * 1e6, 1), "host_model_update_us": round((t2 - t1) * 1e6, 1),
                 "host_graph_replay_us": round(rep_t[-1] * 1e6, 1) if len(rep_t) > n_rep else None,
                 "dev_draw_us": round(e0.elapsed_time(e1) * 1e3, 1), "dev_total_us": round(e0.elapsed_time(e2) * 1e3, 1),
                 "wall_us": round((t3 - t0) * 1e6, 1)})
    print(json.dumps(rows[-1]), flush=True)
for flag in (False, True):
    sel = [r for r in rows if r["policy_step"] == flag][2:]
    if sel:
        print(json.dumps({"policy_step": flag, **{k: round(sum(r[k] for r in sel) / len(sel), 1)
                                                   for k in sel[0] if k not in ("policy_step",) and sel[0][k] is not None}}))
