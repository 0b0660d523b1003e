#!/usr/bin/env python3
"""Microbenchmark of the sampler's fused policy forward (mh_policy_forward, csrc/policy_mlp.hip)
at the benchmark shape (QuadTracking: 12 -> 256 -> 256 -> 8) on E envs: HIP-event device time
per launch and f32-equivalent TFLOP/s. MH_POLICY_KERNEL=f32 selects the all-f32 kernel.
Usage: python tools/policy_bench.py [E] [reps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    import msacl_amd._native as N
    from tools.gputime import time_launches
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    D, N3 = 12, 8
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(D, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                              torch.nn.Linear(256, N3)).cuda()
    n = ctypes.c_int64()
    N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "size")
    P = torch.empty(n.value, device="cuda")
    ps = [p.detach().contiguous() for p in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                            net[4].bias)]
    N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, N3, N.ptr(P), N.stream_of()), "pack")
    obs = torch.randn(E, D, device="cuda")
    out = torch.empty(E, N3, device="cuda")
    fn = lambda: N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, N3, N.ptr(out), N.stream_of())  # noqa: E731
    ms = time_launches(fn, reps)
    flops = 2.0 * E * (D * 256 + 256 * 256 + 256 * N3)
    with torch.no_grad():
        ref = net.double()(obs.double())
    err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
    print(f"policy_forward kernel={os.environ.get('MH_POLICY_KERNEL', 'x3')} E={E}: {ms * 1e3:.2f} us, "
          f"{flops / ms / 1e9:.1f} TFLOP/s (f32-equivalent), max |err| / max |ref| = {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
