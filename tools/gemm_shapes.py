#!/usr/bin/env python3
"""Per-shape timing of the update's MLP GEMMs: mh_gemm_f32 (csrc/gemm.hip) vs PyTorch's BLAS.

Records the (M, N, K, trans_a, trans_b, act) of every LinearAct GEMM during a few MSACL updates
of the bench pipeline (QuadTracking, 65,536 envs, B = 256, n = 20), then times each distinct
shape both ways (HIP events around 50 back-to-back calls, device time: tools/gputime.py) and prints one JSON line per shape.
"""
import argparse
import collections
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.apprfunc import _fused
    from msacl_amd.utils.config import build_pipeline, default_msacl_args

    seen = collections.Counter()
    orig = _fused.gemm

    def rec(x, w, bias, M, N, K, lda, ldb, ta, tb, act=0):
        seen[(M, N, K, ta, tb, act, bias is not None)] += 1
        return orig(x, w, bias, M, N, K, lda, ldb, ta, tb, act)

    _fused.gemm = rec
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False, update_gemm="hip", alg_use_graph=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(2):
        trainer.step()
    seen.clear()
    trainer.step()
    _fused.gemm = orig

    from tools.gputime import time_launches

    def timed(fn):  # device microseconds per call (stream parked on a spin while the host enqueues)
        return time_launches(fn, a.reps, host_us_per_call=120.0, warm=3) * 1e3

    rows = []
    for (M, N, K, ta, tb, act, has_b), calls in sorted(seen.items(), key=lambda kv: -kv[1]):
        A = torch.randn(*((K, M) if ta else (M, K)), device=dev)
        B = torch.randn(*((N, K) if tb else (K, N)), device=dev)
        bias = torch.randn(N, device=dev) if has_b else None
        hip = timed(lambda: orig(A, B, bias, M, N, K, A.shape[1], B.shape[1], ta, tb, act))
        opA = A.t() if ta else A
        opB = B.t() if tb else B
        if bias is not None and act == 1:
            blas_fn = lambda: torch._addmm_activation(bias, opA, opB)  # noqa: E731
        elif bias is not None:
            blas_fn = lambda: torch.addmm(bias, opA, opB)  # noqa: E731
        else:
            blas_fn = lambda: opA.mm(opB)  # noqa: E731
        blas = timed(blas_fn)
        prev_lib = torch.backends.cuda.preferred_blas_library()
        torch.backends.cuda.preferred_blas_library("cublaslt")
        blaslt = timed(blas_fn)
        torch.backends.cuda.preferred_blas_library(prev_lib)
        r = {"M": M, "N": N, "K": K, "ta": ta, "tb": tb, "act": act, "bias": has_b, "calls_per_update": calls,
             "hip_us": round(hip, 2), "blas_us": round(blas, 2), "hipblaslt_us": round(blaslt, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot_h = sum(r["hip_us"] * r["calls_per_update"] for r in rows)
    tot_b = sum(r["blas_us"] * r["calls_per_update"] for r in rows)
    tot_min = sum(min(r["hip_us"], r["blas_us"], r["hipblaslt_us"]) * r["calls_per_update"] for r in rows)
    print(json.dumps({"per_update_us": {"hip": round(tot_h, 1), "blas": round(tot_b, 1), "best_of": round(tot_min, 1)}}))
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
