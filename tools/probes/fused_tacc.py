"""Probe (diagnostic build -DMH_FUSED_EXP_TACC via MSACL_HIP_LIB): s_memtime deltas of the fused
kernel's policy waves summed per segment kind in registers (no memory traffic in the horizon),
workgroups 0-3 x policy waves 0-3; prints the mean cycles per pass of each kind."""
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

env = sys.argv[1] if len(sys.argv) > 1 else "QuadTracking"
dev = torch.device("cuda", 0)
cfg = default_msacl_args(env_name=env, env_num=65536, env_seed=1, seed=0, sample_batch_size=20, n_step=20,
                         replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=0, max_iteration=10 ** 9,
                         eval_interval=10 ** 9, log_save_interval=10 ** 9, apprfunc_save_interval=10 ** 9,
                         save_folder=tempfile.mkdtemp(), num_eval_episode=1, sampler_sync_timing=False, device=dev)
_a, _alg, sampler, buffer, _e, _t = build_pipeline(cfg)
for _ in range(3):
    buffer.add_batch(sampler.sample()[0])
h, st, H = sampler.envs.handle(), N.stream_of(dev), sampler.horizon
E, A, D = 65536, sampler.envs.act_dim, sampler.envs.obs_dim
dbg = torch.zeros(H * E * 2 * A, dtype=torch.float32, device=dev)
dob = torch.zeros(H * E * D, dtype=torch.float32, device=dev)
N.check(N.lib().mh_sample_horizon_debug_logits(h, N.ptr(dbg), N.ptr(dob)), "dbg")
rows = []
for rep in range(4):
    dbg.zero_()
    N.check(N.lib().mh_sample_horizon(h, N.ptr(sampler._packed), D, 2 * A, N.ptr(sampler.obs), H, None, None, None,
                                      None, st), "horizon")
    torch.cuda.synchronize()
    rows.append(dbg[:4 * 4 * 8 * 2].view(torch.int64).view(16, 8).cpu().double())
N.check(N.lib().mh_sample_horizon_debug_logits(h, None, None), "dbg off")
t = torch.stack(rows[1:]).mean(0)  # skip the first (cold) horizon
passes = float(t[0, 7])
names = ["prologue", "hand-offs (8)", "phases 0-6", "phase 7 layer 2 + splits", "layer 3", "logits store",
         "pass barrier + loop"]
out = {nm: round(float(t[:, k].mean() / passes), 1) for k, nm in enumerate(names)}
out["pass total"] = round(float(t[:, :7].sum(1).mean() / passes), 1)
out["per wave pass total"] = [round(float(x / passes), 1) for x in t[:, :7].sum(1)]
print(json.dumps({"env": env, "cycles_per_pass": out}, indent=1))
