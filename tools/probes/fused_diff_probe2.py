"""Probe: after T locksteps, do the fused horizon and the lockstep kernels agree on obs / state?"""
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

E = 4000
for T in (1, 2, 5, 8, 9):
    a, ba, b, bb = _pair("QuadTracking", E, 20, pathlib.Path(tempfile.mkdtemp()))
    A, D = a.envs.act_dim, a.envs.obs_dim
    with torch.no_grad():
        a._pack_policy()
        N.check(N.lib().mh_nstep_set_log_std_clamp(a._h, 1, -20.0, 1.0), "clamp")
        N.check(N.lib().mh_sample_horizon(a._h, N.ptr(a._packed), D, 2 * A, N.ptr(a.obs), T, ctypes.byref(ba.ws), None,
                                          None, None, N.stream_of()), "horizon")
        lg_last = None
        for t in range(T):
            act, lp = torch.empty(E, A, device="cuda"), torch.empty(E, device="cuda")
            lg_last = b.step_traced(act, lp)
        b.flush()
        # the policy on the same (current) obs through the standalone kernel, for both samplers' obs
        la, _ = a._policy_fused()
        lb, _ = b._policy_fused()
    torch.cuda.synchronize()
    so = (a.obs != b.obs).any(1)
    sa = [x for x in a.envs.get_state()]
    sb = [x for x in b.envs.get_state()]
    ss = (sa[0] != sb[0]).any(1)
    print(f"T={T}: obs rows differ {int(so.sum())} {so.nonzero().flatten()[:8].tolist()}  state rows differ {int(ss.sum())}"
          f"  xstate {int((sa[1] != sb[1]).any(1).sum())}  steps {int((sa[2] != sb[2]).sum())}"
          f"  logits-on-own-obs rows differ {int((la != lb).any(1).sum())}")
    del a, ba, b, bb
