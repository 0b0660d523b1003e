"""GPU: the MSACL update's rsample noise drawn inside the policy-head kernel (mh_policy_head_sample).

The reference draws it with torch's generator (RL/utils/act_distribution_cls.py:45-49, rsample),
which no kernel can replay, so the draw is the engine's own and is pinned to the CPU oracle's
restatement of it (oracle/rng.py: Philox4x32-10 + Box-Muller, keyed by (seed, row, launch
counter), stream i / 4, component i % 4), and everything downstream of the draw must equal
mh_policy_head fed the same noise, bit for bit. The device counter must advance once per launch
(a graph replay draws new noise) and re-arm its arrival count.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import rng as R

pytestmark = pytest.mark.gpu


def _native():
    import msacl_amd._native as N
    return N


def _case(M=5120, A=4, D=12, seed=0x1234_5678_9ABC_DEF0):
    g = torch.Generator().manual_seed(3)
    raw = (torch.randn(M, 2 * A, generator=g) * 0.7).cuda()
    obs = torch.randn(M, D, generator=g).cuda()
    old = (torch.rand(M, A, generator=g) * 1.8 - 0.9).cuda()
    hi = torch.full((A,), 1.0).cuda()
    lo = torch.full((A,), -1.0).cuda()
    return raw, obs, old, hi, lo, seed


def _sample(raw, obs, old, hi, lo, seed, ctr):
    N = _native()
    M, A, D = raw.shape[0], raw.shape[1] // 2, obs.shape[1]
    eps = torch.empty(M, A, device="cuda")
    xq = torch.empty(M, D + A, device="cuda")
    nl = torch.empty(M, device="cuda")
    ol = torch.empty(M, device="cuda")
    N.check(N.lib().mh_policy_head_sample(N.ptr(raw), N.ptr(obs), N.ptr(old), N.ptr(hi), N.ptr(lo), M, A, D, -20.0,
                                          1.0, seed, N.ptr(ctr), N.ptr(eps), N.ptr(xq), N.ptr(nl), N.ptr(ol),
                                          N.stream_of(raw.device)), "mh_policy_head_sample")
    return eps, xq, nl, ol


def test_head_noise_matches_oracle_and_downstream_is_bitwise():
    raw, obs, old, hi, lo, seed = _case()
    M, A = raw.shape[0], raw.shape[1] // 2
    ctr = torch.zeros(2, dtype=torch.int64, device="cuda")
    eps0, xq0, nl0, ol0 = _sample(raw, obs, old, hi, lo, seed, ctr)
    eps1, *_ = _sample(raw, obs, old, hi, lo, seed, ctr)
    torch.cuda.synchronize()
    assert ctr.tolist() == [2, 0]  # one advance per launch, arrival count re-armed
    rows = np.arange(M)
    for launch, eps in ((0, eps0), (1, eps1)):
        want = np.empty((M, A))
        for s in range((A + 3) // 4):
            nv = R.box_muller(R.draw_words(seed, rows, np.full(M, launch), s))
            for i in range(4 * s, min(A, 4 * s + 4)):
                want[:, i] = nv[:, i - 4 * s]
        got = eps.cpu().numpy().astype(np.float64)
        # float32 Box-Muller (logf / sincosf) vs float64 on the same uniforms
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=2e-6 * np.abs(want).max())
    assert not torch.equal(eps0, eps1)
    # downstream of the draw: mh_policy_head on the same noise, bit for bit
    N = _native()
    D = obs.shape[1]
    xq = torch.empty(M, D + A, device="cuda")
    nl = torch.empty(M, device="cuda")
    ol = torch.empty(M, device="cuda")
    N.check(N.lib().mh_policy_head(N.ptr(raw), N.ptr(eps0), N.ptr(obs), N.ptr(old), N.ptr(hi), N.ptr(lo), M, A, D,
                                   -20.0, 1.0, N.ptr(xq), N.ptr(nl), N.ptr(ol), N.stream_of(raw.device)),
            "mh_policy_head")
    for a, b in ((xq, xq0), (nl, nl0), (ol, ol0)):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_head_noise_statistics_and_graph_replay():
    raw, obs, old, hi, lo, seed = _case(M=65536, A=8)
    ctr = torch.zeros(2, dtype=torch.int64, device="cuda")
    _sample(raw, obs, old, hi, lo, seed, ctr)  # warm
    outs = []
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eps, *_ = _sample(raw, obs, old, hi, lo, seed, ctr)
    for _ in range(3):
        g.replay()
        outs.append(eps.clone())
    torch.cuda.synchronize()
    assert ctr[1].item() == 0 and ctr[0].item() >= 4
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
    x = torch.cat(outs).double()
    assert abs(x.mean().item()) < 5e-3 and abs(x.std().item() - 1.0) < 5e-3
