"""Probe: is each path deterministic (two identical runs of the same path agree)?"""
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
name = sys.argv[1] if len(sys.argv) > 1 else "QuadTracking"


def run_fused(s, bs):
    with torch.no_grad():
        s._pack_policy()
        N.check(N.lib().mh_nstep_set_log_std_clamp(s._h, 1, -20.0, 1.0), "clamp")
        N.check(N.lib().mh_sample_horizon(s._h, N.ptr(s._packed), s.envs.obs_dim, 2 * s.envs.act_dim, N.ptr(s.obs), T,
                                          ctypes.byref(bs.ws), None, None, None, N.stream_of()), "horizon")
    torch.cuda.synchronize()
    return s.obs.clone()


def run_lock(s):
    with torch.no_grad():
        for _ in range(T):
            act, lp = torch.empty(E, s.envs.act_dim, device="cuda"), torch.empty(E, device="cuda")
            s.step_traced(act, lp)
        s.flush()
    torch.cuda.synchronize()
    return s.obs.clone()


a1, ba1, b1, bb1 = _pair(name, E, 20, pathlib.Path(tempfile.mkdtemp()))
a2, ba2, b2, bb2 = _pair(name, E, 20, pathlib.Path(tempfile.mkdtemp()))
oa1, oa2 = run_fused(a1, ba1), run_fused(a2, ba2)
ob1, ob2 = run_lock(b1), run_lock(b2)
d = lambda x, y: (x != y).any(1).nonzero().flatten().tolist()  # noqa: E731
print(name, "fused vs fused:", d(oa1, oa2)[:12], " lock vs lock:", d(ob1, ob2)[:12], " fused vs lock:", d(oa1, ob1)[:12])
