"""Probe: per lockstep, the fused kernel's logits / actions vs the lockstep path's (QuadTracking)."""
import ctypes
import os
import pathlib
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import msacl_amd  # noqa: F401,E402
import msacl_amd._native as N  # noqa: E402
from test_gpu_fused_horizon import _pair  # noqa: E402

E, T = 4000, 6
a, ba, b, bb = _pair("QuadTracking", E, 20, pathlib.Path(tempfile.mkdtemp()))
A, D = a.envs.act_dim, a.envs.obs_dim
lgA = torch.zeros(T, E, 2 * A, device="cuda")
actA, lpA = torch.empty(T, E, A, device="cuda"), torch.empty(T, E, device="cuda")
obA = torch.zeros(T, E, D, device="cuda")
N.check(N.lib().mh_sample_horizon_debug_logits(a._h, N.ptr(lgA), N.ptr(obA)), "dbg")
with torch.no_grad():
    a._pack_policy()
    N.check(N.lib().mh_nstep_set_log_std_clamp(a._h, 1, -20.0, 1.0), "clamp")
    N.check(N.lib().mh_sample_horizon(a._h, N.ptr(a._packed), D, 2 * A, N.ptr(a.obs), T, ctypes.byref(ba.ws), None,
                                      N.ptr(actA), N.ptr(lpA), N.stream_of()), "horizon")
    obsB, lgB, actB = [], [], []
    for t in range(T):
        obsB.append(b.obs.clone())
        act, lp = torch.empty(E, A, device="cuda"), torch.empty(E, device="cuda")
        lgB.append(b.step_traced(act, lp).clone())
        actB.append(act.clone())
    b.flush()
torch.cuda.synchronize()
for t in range(T):
    dl = (lgA[t] != lgB[t]).any(1)
    da = (actA[t] != actB[t]).any(1)
    print(f"t={t}: logits rows differ {int(dl.sum())} {dl.nonzero().flatten()[:10].tolist()}; actions rows differ {int(da.sum())}")
    if dl.any():
        e = int(dl.nonzero()[0])
        print("   env", e, "A", lgA[t, e].tolist())
        print("   env", e, "B", lgB[t][e].tolist())
        # the standalone policy on B's observation at that step (same packed weights)
        lg, _ = a._policy_fused.__func__(type("S", (), {"num_envs": E, "envs": a.envs, "device": a.device,
                                                         "_packed": a._packed, "obs": obsB[t]})())
        print("   env", e, "standalone on B obs", lg[e].tolist())
        break
