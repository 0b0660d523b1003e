"""Standalone device time of the MSACL update's policy-head launches at the bench's 5,120 rows:
log_prob only (the Lyapunov step), rsample on given noise, rsample with the in-kernel draw
(mh_policy_head_sample), and the backward. One JSON line per case."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.gputime import time_launches  # noqa: E402


def main():
    import msacl_amd  # noqa: F401
    import msacl_amd._native as N
    M, A, D = 5120, 4, 12
    dev = torch.device("cuda", 0)
    raw = torch.randn(M, 2 * A, device=dev) * 0.7
    obs = torch.randn(M, D, device=dev)
    old = torch.rand(M, A, device=dev) * 1.8 - 0.9
    hi, lo = torch.ones(A, device=dev), -torch.ones(A, device=dev)
    eps = torch.randn(M, A, device=dev)
    xq = torch.empty(M, D + A, device=dev)
    nl, ol = torch.empty(M, device=dev), torch.empty(M, device=dev)
    ctr = torch.zeros(2, dtype=torch.int64, device=dev)
    st = N.stream_of(dev)
    L = N.lib()
    cases = {
        "log_prob": lambda: L.mh_policy_head(N.ptr(raw), None, None, N.ptr(old), N.ptr(hi), N.ptr(lo), M, A, 0, -20.0,
                                             1.0, None, None, N.ptr(ol), st),
        "rsample_eps": lambda: L.mh_policy_head(N.ptr(raw), N.ptr(eps), N.ptr(obs), None, N.ptr(hi), N.ptr(lo), M, A,
                                                D, -20.0, 1.0, N.ptr(xq), N.ptr(nl), None, st),
        "rsample_draw": lambda: L.mh_policy_head_sample(N.ptr(raw), N.ptr(obs), None, N.ptr(hi), N.ptr(lo), M, A, D,
                                                        -20.0, 1.0, 7, N.ptr(ctr), N.ptr(eps), N.ptr(xq), N.ptr(nl),
                                                        None, st),
        "rsample_draw_logprob": lambda: L.mh_policy_head_sample(N.ptr(raw), N.ptr(obs), N.ptr(old), N.ptr(hi),
                                                                N.ptr(lo), M, A, D, -20.0, 1.0, 7, N.ptr(ctr),
                                                                N.ptr(eps), N.ptr(xq), N.ptr(nl), N.ptr(ol), st),
    }
    for name, fn in cases.items():
        t = time_launches(fn, reps=50)
        print(json.dumps({"case": name, "rows": M, "us": round(t * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
