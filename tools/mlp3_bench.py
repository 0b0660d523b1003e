"""Standalone device time of the update's fused MLP kernels (csrc/mlp_fused.hip, csrc/gemm.hip
weight gradients) at the bench's shapes, one kernel at a time on an idle GPU (inside the update
they share the chip with the other stream's kernels, so the trace's per-kernel times are
inflated). Prints one JSON line per case.

    python tools/mlp3_bench.py [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools.gputime import time_launches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cases", default="", help="M,K1,N3,keep,groups;... (default: the bench's shapes)")
    a = ap.parse_args()
    import msacl_amd  # noqa: F401
    from msacl_amd.apprfunc import _fused as F

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H = 256

    def lin(n_out, n_in):
        return (torch.randn(n_out, n_in, device=dev) / n_in ** 0.5, torch.randn(n_out, device=dev) * 0.1)

    rows_out = []
    cases = [tuple(int(v) for v in c.split(",")) for c in a.cases.split(";") if c]
    for M, K1, N3, keep, groups in cases or ((5120, 16, 1, True, 2), (5120, 16, 1, False, 2), (10240, 12, 1, True, 1),
                                    (5120, 12, 256, True, 1), (5120, 12, 1, True, 1), (10240, 12, 256, True, 1),
                                    (5376, 12, 256, False, 1), (5120, 16, 1, True, 4)):
        keep = bool(keep)
        layers = (lin(H, K1), lin(H, H), lin(N3, H))
        x = torch.randn(M, K1, device=dev)
        if groups == 4:
            # the critics and the target critics as the two network sets of one launch (forward_pair)
            from msacl_amd.apprfunc._twin import TwinCritic
            from msacl_amd.apprfunc.mlp import ActionValue
            kw = dict(obs_dim=12, act_dim=4, hidden_sizes=[256, 256], hidden_activation="relu",
                      output_activation="linear")
            nets = [ActionValue(**kw).to(dev) for _ in range(4)]
            tc, tt = TwinCritic.build(nets[0], nets[1]), TwinCritic.build(nets[2], nets[3])
            xo = torch.randn(M, K1, device=dev)

            def fwd():
                tc.forward_pair(x, tt, xo)
        elif groups == 2:
            # the twin critics' joint buffers: group q's operands at q x the strides
            W1 = torch.stack([layers[0][0]] * 2)
            b1 = torch.stack([layers[0][1]] * 2)
            W2 = torch.stack([layers[1][0]] * 2)
            b2 = torch.stack([layers[1][1]] * 2)
            W3 = torch.stack([layers[2][0]] * 2)
            b3 = torch.stack([layers[2][1]] * 2)
            y = torch.empty(2, M, N3, device=dev)
            h = [torch.empty(2, M, H, device=dev) for _ in range(2)] if keep else None
            strides = (0, H * K1, H, H * H, H, N3 * H, N3, M * H, M * N3)

            def fwd():
                N = F._native()
                import ctypes
                gs = (ctypes.c_int64 * 9)(*strides)
                N.check(N.lib().mh_mlp3_forward(N.ptr(x), M, K1, x.stride(0), N.ptr(W1), N.ptr(b1), N.ptr(W2), N.ptr(b2),
                                                N.ptr(W3), N.ptr(b3), H, N3, 1, 1, 0,
                                                N.ptr(h[0]) if keep else None, N.ptr(h[1]) if keep else None, H,
                                                N.ptr(y), N3, 2, gs, N.stream_of(dev)), "mh_mlp3_forward")
        else:
            def fwd():
                F.mlp3_forward(x, layers, (1, 1, 0), keep)
        t = time_launches(fwd, reps=a.reps)
        flops = 2.0 * groups * M * (K1 * H + H * H + H * N3)
        rows_out.append({"kernel": "k_mlp3_fwd", "M": M, "K1": K1, "N3": N3, "keep": keep, "groups": groups,
                         "us": round(t * 1e3, 2), "f32_TFLOPs": round(flops / (t * 1e-3) / 1e12, 1)})
        print(json.dumps(rows_out[-1]), flush=True)

        if groups == 1 and keep:
            # per-layer path of the same forward (MSACL_MLP3=0)
            def per_layer():
                h1 = F.gemm(x, layers[0][0], layers[0][1], M, H, K1, K1, K1, 0, 1, act=1)
                h2 = F.gemm(h1, layers[1][0], layers[1][1], M, H, H, H, H, 0, 1, act=1)
                F.gemm(h2, layers[2][0], layers[2][1], M, N3, H, H, H, 0, 1, act=0)
            try:
                t2 = time_launches(per_layer, reps=a.reps)
                rows_out.append({"kernel": "per_layer_fwd", "M": M, "K1": K1, "N3": N3, "us": round(t2 * 1e3, 2)})
                print(json.dumps(rows_out[-1]), flush=True)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"kernel": "per_layer_fwd", "error": str(e)[:200]}), flush=True)
            # backward chain (input gradient + kept g2 / g1)
            y, h1, h2 = F.mlp3_forward(x, layers, (1, 1, 0), True)
            dy = torch.randn(M, N3, device=dev)
            g2 = torch.empty(M, H, device=dev)
            g1 = torch.empty(M, H, device=dev)
            dx = torch.empty(M, K1, device=dev)

            def bwd():
                N = F._native()
                N.check(N.lib().mh_mlp3_backward(N.ptr(dy), N3, N.ptr(h1), N.ptr(h2), H, N.ptr(layers[0][0]),
                                                 N.ptr(layers[1][0]), N.ptr(layers[2][0]), M, K1, H, N3, 1, 1,
                                                 N.ptr(g2), N.ptr(g1), H, N.ptr(dx), K1, 1, None, N.stream_of(dev)),
                        "mh_mlp3_backward")
            t3 = time_launches(bwd, reps=a.reps)
            rows_out.append({"kernel": "k_mlp3_bwd", "M": M, "K1": K1, "N3": N3, "us": round(t3 * 1e3, 2)})
            print(json.dumps(rows_out[-1]), flush=True)
            # the three weight gradients (mh_weight_grads)
            dW = [torch.empty(H, K1, device=dev), torch.empty(H, H, device=dev), torch.empty(N3, H, device=dev)]
            db = [torch.empty(H, device=dev), torch.empty(H, device=dev), torch.empty(N3, device=dev)]
            prods = [(dy, N3, h2, H, N3, H, dW[2], db[2]), (g2, H, h1, H, H, H, dW[1], db[1]),
                     (g1, H, x, K1, H, K1, dW[0], db[0])]
            prods = [p for p in prods if F.wgrad_ok(p[0], p[1], p[2], p[3], p[4], p[5], M)]
            t4 = time_launches(lambda: F.weight_grads(prods, M, dev), reps=a.reps)
            rows_out.append({"kernel": "weight_grads", "M": M, "K1": K1, "N3": N3, "products": len(prods),
                             "us": round(t4 * 1e3, 2)})
            print(json.dumps(rows_out[-1]), flush=True)


if __name__ == "__main__":
    main()
