"""Probe (diagnostic build -DMH_FUSED_EXP_STAMPS via MSACL_HIP_LIB): s_memtime stamps of the fused
kernel's policy waves (workgroups 0-3, waves 0-3, every pass): per-phase cycle breakdown."""
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

dev = torch.device("cuda", 0)
cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, env_seed=1, seed=0, sample_batch_size=20, n_step=20,
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
for rep in range(3):
    dbg.zero_()
    N.check(N.lib().mh_sample_horizon(h, N.ptr(sampler._packed), D, 2 * A, N.ptr(sampler.obs), H, None, None, None,
                                      None, st), "horizon")
    torch.cuda.synchronize()
N.check(N.lib().mh_sample_horizon_debug_logits(h, None, None), "dbg off")
t = dbg[:4 * 4 * 64 * 32 * 2].view(torch.int64).view(4, 4, 64, 32).cpu().double()
passes = 2 * H
# per pass: entry(0), pre-sync ib (1+2ib), post-sync ib (2+2ib), pre-epilogue 17, after barrier 18
seg = {"prologue (entry -> pre-sync 0)": (0, 1), "epilogue (pre-epi -> barrier)": (17, 18)}
for ib in range(8):
    seg[f"sync {ib}"] = (1 + 2 * ib, 2 + 2 * ib)
    seg[f"phase {ib} body"] = (2 + 2 * ib, 3 + 2 * ib if ib < 7 else 17)
out = {}
for k, (a_, b_) in seg.items():
    d = (t[:, :, 1:passes - 1, b_] - t[:, :, 1:passes - 1, a_])
    out[k] = round(float(d.mean()), 1)
tot = (t[:, :, 2:passes - 1, 0] - t[:, :, 1:passes - 2, 0]).mean()
out["pass total (entry -> next entry)"] = round(float(tot), 1)
print(json.dumps(out, indent=1))
