"""Probe: the horizon emission (k_emit_cells via mh_sample_horizon_emit, idempotent re-emission of
the last horizon) against the horizon's window count, trainer step by trainer step at the bench
config; plus the first, in-step emission's duration from HIP events bracketing the sampler call
is not separable here, so the re-emission is timed right after each step (warm L2) and once more
after an L2-flushing copy (cold)."""
import ctypes
import json
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import msacl_amd  # noqa: F401,E402
import msacl_amd._native as N  # noqa: E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

policy = sys.argv[1] if len(sys.argv) > 1 else "init"
dev = torch.device("cuda", 0)
cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, env_seed=1, seed=0, sample_batch_size=20, n_step=20,
                         replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000 if policy == "init" else 0,
                         max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                         apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), num_eval_episode=1,
                         sampler_sync_timing=False, device=dev)
_a, alg, sampler, buffer, _e, trainer = build_pipeline(cfg)
if policy == "hover":
    sys.path.insert(0, ROOT)
    from bench import set_hover_policy  # noqa: E402
    set_hover_policy(alg.networks.policy, float(sampler.envs.single_action_space.high[0]) / 2)
h, st, H = sampler.envs.handle(), N.stream_of(dev), sampler.horizon
win = torch.zeros(1, dtype=torch.int64, device=dev)
flush = torch.empty(512 * 1024 * 1024 // 4, dtype=torch.float32, device=dev)


def emit():
    N.check(N.lib().mh_sample_horizon_emit(h, H, ctypes.byref(buffer.ws), N.ptr(win), st), "emit")


def timed(reps, cold):
    ts = []
    for _ in range(reps):
        if cold:
            flush.add_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        emit()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return round(sorted(ts)[len(ts) // 2], 2)


for it in range(40):
    c0 = int(buffer.cursor[2].item())
    trainer.step()
    trainer.iteration += 1
    torch.cuda.synchronize()
    c1 = int(buffer.cursor[2].item())
    if it < 6:
        continue
    warm = timed(5, False)
    cold = timed(3, True)
    w = int(win.item())
    print(json.dumps({"step": it, "windows_cursor": c1 - c0, "windows_hdr": w, "emit_us_warm": warm,
                      "emit_us_cold": cold, "GBps_cold": round(w * 2560 / (cold * 1e-6) / 1e9, 1) if cold else None}),
          flush=True)
