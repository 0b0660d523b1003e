#!/usr/bin/env python3
"""Device time of mh_gemm_f32 on the update's tall shapes (B x n = 5,120 rows) and weight
gradients (K = 5,120) for the library
MSACL_HIP_LIB points at (tools/ab_libs.sh variants), next to PyTorch's BLAS."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.apprfunc._fused import gemm
    from tools.gputime import time_launches
    dev = torch.device("cuda", 0)
    for (M, N, K, tb, act) in [(5120, 256, 256, 1, 1), (5120, 256, 256, 0, 0), (5120, 256, 16, 1, 1),
                               (10240, 256, 256, 0, 0)]:
        A = torch.randn(M, K, device=dev)
        B = torch.randn(*((N, K) if tb else (K, N)), device=dev)
        bias = torch.randn(N, device=dev) if tb else None
        us = time_launches(lambda: gemm(A, B, bias, M, N, K, K, B.shape[1], 0, tb, act), 50,
                           host_us_per_call=120.0, warm=3) * 1e3
        opB = B.t() if tb else B
        bl = time_launches(lambda: A.mm(opB), 50, host_us_per_call=120.0, warm=3) * 1e3
        print(f"M={M} N={N} K={K} tb={tb} act={act}: hip {us:.2f} us  blas {bl:.2f} us", flush=True)
    for (M, N, K) in [(256, 256, 5120), (256, 256, 10240)]:  # weight gradients g^T x
        gr = torch.randn(K, M, device=dev)
        x = torch.randn(K, N, device=dev)
        us = time_launches(lambda: gemm(gr, x, None, M, N, K, M, N, 1, 0), 50, host_us_per_call=120.0, warm=3) * 1e3
        bl = time_launches(lambda: gr.t().mm(x), 50, host_us_per_call=120.0, warm=3) * 1e3
        print(f"M={M} N={N} K={K} ta=1 (g^T x): hip {us:.2f} us  blas {bl:.2f} us", flush=True)


if __name__ == "__main__":
    main()
