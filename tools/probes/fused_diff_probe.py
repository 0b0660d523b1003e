"""Probe: first lockstep where the fused horizon and the lockstep kernels disagree (QuadTracking)."""
import ctypes
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import msacl_amd  # noqa: F401,E402
import msacl_amd._native as N  # noqa: E402
from test_gpu_fused_horizon import _pair  # noqa: E402
import pathlib  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
a, ba, b, bb = _pair("QuadTracking", E, 20, pathlib.Path(tempfile.mkdtemp()))
H, A, D = a.horizon, a.envs.act_dim, a.envs.obs_dim
actA, lpA = torch.empty(H, E, A, device="cuda"), torch.empty(H, E, device="cuda")
with torch.no_grad():
    a._pack_policy()
    pol = a.networks.policy
    N.check(N.lib().mh_nstep_set_log_std_clamp(a._h, 1, -20.0, 1.0), "clamp")
    obs_before = a.obs.clone()
    N.check(N.lib().mh_sample_horizon(a._h, N.ptr(a._packed), D, 2 * A, N.ptr(a.obs), H, ctypes.byref(ba.ws), None,
                                      N.ptr(actA), N.ptr(lpA), N.stream_of()), "horizon")
assert torch.equal(obs_before, b.obs)
actB, lpB, lgB = [], [], []
for t in range(H):
    act, lp = torch.empty(E, A, device="cuda"), torch.empty(E, device="cuda")
    lg = b.step_traced(act, lp)
    actB.append(act.clone()); lpB.append(lp.clone()); lgB.append(lg.clone())
b.flush()
torch.cuda.synchronize()
actB, lpB = torch.stack(actB), torch.stack(lpB)
diff = (actA != actB).any(2) | (lpA != lpB)
bad = diff.any(0).nonzero().flatten().tolist()
print("envs differing:", len(bad), bad[:10])
for e in bad[:6]:
    t0 = int(diff[:, e].nonzero()[0])
    print(f"env {e}: first t {t0}: actA {actA[t0, e].tolist()} actB {actB[t0, e].tolist()} lpA {lpA[t0, e].item()} lpB {lpB[t0, e].item()}")
    print("   logitsB", lgB[t0][e].tolist())
