"""Probe: two fused-horizon runs from the same state — where do they first disagree?"""
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

E, T = int(sys.argv[1]) if len(sys.argv) > 1 else 4000, 8


def run(dbg):
    a, ba, b, bb = _pair("QuadTracking", E, 20, pathlib.Path(tempfile.mkdtemp()))
    A, D = a.envs.act_dim, a.envs.obs_dim
    lg = torch.zeros(T, E, 2 * A, device="cuda")
    ob = torch.zeros(T, E, D, device="cuda")
    act, lp = torch.empty(T, E, A, device="cuda"), torch.empty(T, E, device="cuda")
    if dbg:
        N.check(N.lib().mh_sample_horizon_debug_logits(a._h, N.ptr(lg), N.ptr(ob)), "dbg")
    with torch.no_grad():
        a._pack_policy()
        N.check(N.lib().mh_nstep_set_log_std_clamp(a._h, 1, -20.0, 1.0), "clamp")
        N.check(N.lib().mh_sample_horizon(a._h, N.ptr(a._packed), D, 2 * A, N.ptr(a.obs), T, ctypes.byref(ba.ws), None,
                                          N.ptr(act), N.ptr(lp), N.stream_of()), "horizon")
    torch.cuda.synchronize()
    st = a.envs.get_state()
    return lg, act, a.obs.clone(), st[0].clone(), st[1].clone(), ob


for dbg in (True, True):
    r1, r2 = run(dbg), run(dbg)
    first = None
    for t in range(T):
        dl = (r1[0][t] != r2[0][t]).any(1)
        da = (r1[1][t] != r2[1][t]).any(1)
        do_ = (r1[5][t] != r2[5][t]).any(1)
        if do_.any() and first is None:
            e = int(do_.nonzero()[0])
            print("  t", t, "env", e, "obs run1", [round(x, 7) for x in r1[5][t][e].tolist()])
            print("  t", t, "env", e, "obs run2", [round(x, 7) for x in r2[5][t][e].tolist()])
            if t > 0:
                print("  t-1 act run1", r1[1][t - 1][e].tolist(), "run2", r2[1][t - 1][e].tolist())
                print("  t-1 obs run1", [round(x, 7) for x in r1[5][t - 1][e].tolist()])
        if (dl.any() or da.any() or do_.any()) and first is None:
            first = (t, "obs", int(do_.sum()), do_.nonzero().flatten()[:6].tolist(), "logits", int(dl.sum()),
                     dl.nonzero().flatten()[:6].tolist(), "act", int(da.sum()))
    do = (r1[2] != r2[2]).any(1)
    ds = (r1[3] != r2[3]).any(1)
    print(f"dbg={dbg}: first differing step (t, logits rows, action rows, envs) {first}; final obs rows {int(do.sum())} "
          f"{do.nonzero().flatten()[:8].tolist()} state rows {int(ds.sum())}")
