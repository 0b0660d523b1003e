#!/usr/bin/env python3
"""Launch a few mh_gemm_f32 shapes back to back (for rocprofv3 --kernel-trace / --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.apprfunc._fused import gemm
    dev = torch.device("cuda", 0)
    shapes = [(5120, 256, 1, 0, 0), (5120, 256, 16, 0, 1), (5120, 256, 256, 0, 1), (256, 256, 5120, 1, 0),
              (256, 256, 256, 0, 1)]
    for (M, N, K, ta, tb) in shapes:
        a = torch.randn(*((K, M) if ta else (M, K)), device=dev)
        b = torch.randn(*((N, K) if tb else (K, N)), device=dev)
        for _ in range(10):
            gemm(a, b, None, M, N, K, a.shape[1], b.shape[1], ta, tb, 0)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
