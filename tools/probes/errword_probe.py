"""Probe: run the fused horizon a few times and print the device error word."""
import ctypes, os, pathlib, sys, tempfile
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msacl_amd  # noqa
import msacl_amd._native as N  # noqa
from test_gpu_fused_horizon import _pair, _fused_errors  # noqa
a, ba, b, bb = _pair("QuadTracking", 4000, 20, pathlib.Path(tempfile.mkdtemp()))
for i in range(4):
    a.sample()
    torch.cuda.synchronize()
    print("after sample", i, "error word", _fused_errors(a), "(1<<20 units: LDS obs mismatch; 1: wait timeout)")
