#!/usr/bin/env python3
"""Per-kernel microbenchmarks of the engine: device time per launch with HIP
events (tools/gputime.py), algorithmic bytes per launch, achieved GB/s and the fraction of the
8 TB/s HBM peak.

  env_step      mh_env_step (k_rollout<Env>, injected in-box actions, no n-step ring) for
                the six envs at E = 65,536 and 4,194,304
  rollout       mh_rollout_step (TanhGauss sampling from logits + step + ring push) alone and
  +emit         followed by the fused window emission into an HBM store, E = 65,536
  gather        mh_replay_gather of B windows (random indices) from a 1M-window store
  msacl         q_target / lyapunov / stability_adv / ppo_clip at the replay batch B = 256, n = 20
  gae           mh_gae over [E][H] on-policy trajectory blocks (65,536 x 64 and 65,536 x 1,600)
  policy        fused f32-MFMA policy MLP forward vs the PyTorch GEMM path (TFLOP/s vs 157.3 peak)

Prints one JSON object per line; --out writes the list as JSON.
Usage: python tools/kernel_bench.py [--sizes 65536,4194304] [--reps 20] [--out file]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import msacl_amd  # noqa: E402,F401
import msacl_amd._native as N  # noqa: E402
from tools.gputime import time_launches  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E
ENVS = ["VanderPol", "Pendulum", "DuctedFan", "TwoLink", "SingleTrackCar", "QuadTracking"]


def row(kernel, env, units, unit_name, bytes_per_unit, ms, **extra):
    gbs = units * bytes_per_unit / (ms * 1e-3) / 1e9
    r = {"kernel": kernel, "env": env, unit_name: units, "bytes_per_unit": bytes_per_unit, "avg_us": round(ms * 1e3, 3),
         "GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
    r.update(extra)
    print(json.dumps(r), flush=True)
    return r


# SURVEY §8(d)'s algorithmic bytes per env-step (minimal f32 SoA: read state + step counter +
# action, write state + step counter + real_next_obs + reward + cost + term + trunc; Quad with
# Rd_last in f64), the figure the >= 40 % per-kernel HBM bar is quoted on
SURVEY_BYTES = {"VanderPol": 46, "Pendulum": 46, "DuctedFan": 98, "TwoLink": 74, "SingleTrackCar": 110,
                "QuadTracking": 370}


def env_step_bytes(info):
    S, XS, D, A = info.state_dim, info.xstate_dim, info.obs_dim, info.act_dim
    # read state/xstate/step + action; write state/xstate/step + obs + real_next_obs + reward + term + trunc
    return 2 * (S * 4 + XS * 8 + 4) + A * 4 + 2 * D * 4 + 4 + 2


def bench_env_step(name, E, reps, dev):
    info = N.env_info(name)
    D, A = info.obs_dim, info.act_dim
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS[name], E, 1234, ctypes.byref(h)), "create")
    try:
        lo = torch.tensor(list(info.act_low)[:A], device=dev)
        hi = torch.tensor(list(info.act_high)[:A], device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        act = (lo + (hi - lo) * torch.rand(E, A, device=dev, generator=g)).contiguous()
        obs, real = torch.empty(E, D, device=dev), torch.empty(E, D, device=dev)
        rew = torch.empty(E, device=dev)
        term = torch.empty(E, dtype=torch.uint8, device=dev)
        trunc = torch.empty_like(term)
        st = N.stream_of(dev)
        N.check(N.lib().mh_env_reset(h, None, N.ptr(obs), st), "reset")

        def fn():
            N.lib().mh_env_step(h, N.ptr(act), None, N.ptr(obs), N.ptr(real), N.ptr(rew), N.ptr(term),
                                N.ptr(trunc), st)

        ms = time_launches(fn, reps)
        sb = SURVEY_BYTES[name]
        return row("env_step", name, E, "env_steps", env_step_bytes(info), ms, survey_bytes_per_unit=sb,
                   survey_frac=round(E * sb / (ms * 1e-3) / 1e9 / PEAK, 4))
    finally:
        torch.cuda.synchronize()
        N.lib().mh_env_destroy(h)


def bench_rollout(name, E, reps, dev, n=20):
    from msacl_amd.trainer.buffer.device_nstep_replay_buffer import DeviceNstepReplayBuffer
    info = N.env_info(name)
    S, XS, D, A, F = info.state_dim, info.xstate_dim, info.obs_dim, info.act_dim, info.record_floats
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS[name], E, 99, ctypes.byref(h)), "create")
    out = []
    try:
        N.check(N.lib().mh_nstep_attach(h, n, 100.0, 100.0), "attach")
        N.check(N.lib().mh_nstep_set_log_std_clamp(h, 1, -20.0, 1.0), "clamp")
        store = E <= 1_000_000  # the window store path (fused / deferred emission) at <= 1M envs
        buf = DeviceNstepReplayBuffer(obs_dim=D, act_dim=A, buffer_max_size=1_000_000, n_step=n, device=dev) \
            if store else None
        obs = torch.empty(E, D, device=dev)
        st = N.stream_of(dev)
        N.check(N.lib().mh_env_reset(h, None, N.ptr(obs), st), "reset")
        logits = torch.zeros(E, 2 * A, device=dev)
        logits[:, A:] = -1.0  # log std
        # warm the rings so windows are emitted every step
        for _ in range(n):
            N.check(N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(obs),
                                            ctypes.byref(buf.ws) if store else None, None, None, st), "rollout")

        def fn_roll():
            N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(obs), None, None, None, st)

        def fn_pair():
            N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(obs), ctypes.byref(buf.ws), None, None, st)

        def fn_defer():
            N.lib().mh_rollout_step_deferred(h, N.ptr(logits), None, None, None, N.ptr(obs), ctypes.byref(buf.ws),
                                             None, None, st)

        ms_roll = time_launches(fn_roll, reps)
        b_roll = (S * 4 + XS * 8 + 4 + 2 * A * 4 + D * 4 + 8) + (S * 4 + XS * 8 + 4 + D * 4 + F * 4 + 8 + 4)
        out.append(row("rollout_step", name, E, "env_steps", b_roll, ms_roll))
        if not store:
            return out
        w0 = int(buf.cursor[2].item())
        ms_pair = time_launches(fn_pair, reps, warm=0)
        wins = (int(buf.cursor[2].item()) - w0) / reps
        ms_emit = max(ms_pair - ms_roll, 1e-6)
        b_win = n * F * 4 + n * (2 * D + A + 4) * 4
        out.append(row("window_emit(pair-minus-rollout)", name, round(wins, 1), "windows", b_win, ms_emit,
                       pair_us=round(ms_pair * 1e3, 3)))
        w1 = int(buf.cursor[2].item())
        ms_defer = time_launches(fn_defer, reps, warm=0)
        N.check(N.lib().mh_rollout_flush(h, st), "flush")
        torch.cuda.synchronize()
        wd = (int(buf.cursor[2].item()) - w1) / reps
        # per env-step bytes of the deferred kernel: the step + its share of the windows it emits
        out.append(row("rollout_emit(deferred)", name, E, "env_steps", b_roll + wd * b_win / E, ms_defer,
                       windows=round(wd, 1)))
        return out
    finally:
        torch.cuda.synchronize()
        N.lib().mh_env_destroy(h)


def bench_gather(name, B, reps, dev, n=20, M=1_000_000):
    from msacl_amd.trainer.buffer.device_nstep_replay_buffer import DeviceNstepReplayBuffer
    info = N.env_info(name)
    D, A = info.obs_dim, info.act_dim
    buf = DeviceNstepReplayBuffer(obs_dim=D, act_dim=A, buffer_max_size=M, n_step=n, device=dev)
    for v in buf.n_step_buf.values():
        v.uniform_()
    buf.cursor.copy_(torch.tensor([0, M, M, 0], dtype=torch.int64))
    idx = buf.sample_indices(B)
    outs = {k: torch.empty((B,) + tuple(v.shape[1:]), device=dev) for k, v in buf.n_step_buf.items()}
    st = N.stream_of(dev)
    keys = ["obs", "act", "rew", "cost", "obs2", "done", "logp"]

    def fn():
        N.lib().mh_replay_gather(ctypes.byref(buf.ws), n, D, A, N.ptr(idx), B, *[N.ptr(outs[k]) for k in keys], st)

    ms = time_launches(fn, reps)
    per = 2 * n * (2 * D + A + 4) * 4 + 8
    return row("replay_gather", name, B, "windows", per, ms)


def bench_msacl(reps, dev, B=256, n=20, D=12):
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    q1, q2, q1t, q2t, nlp, rew = r(B, n), r(B, n), r(B, n), r(B, n), r(B, n), r(B, n)
    done = (torch.rand(B, n, device=dev, generator=g) < 0.1).float()
    la = torch.tensor([0.3], device=dev)
    o = [torch.empty(B, n, device=dev) for _ in range(3)] + [torch.empty(1, device=dev), torch.empty(B, device=dev)]
    st = N.stream_of(dev)
    res = []

    def fq():
        N.lib().mh_msacl_q_target(*[N.ptr(t) for t in (q1, q2, q1t, q2t, nlp, rew, done, la)], None, 0.99, B, n,
                                  *[N.ptr(t) for t in o], st)
    ms = time_launches(fq, reps)
    res.append(row("msacl_q_target", "-", B, "windows", (9 * n) * 4 + (3 * n + 1) * 4, ms))
    obs, obs2 = r(B, n, D) * 0.5, r(B, n, D) * 0.5
    V, V2 = torch.rand(B, n, device=dev, generator=g), torch.rand(B, n, device=dev, generator=g)
    logp, old = r(B, n), r(B, n)
    k = torch.arange(1, n + 1, dtype=torch.float32, device=dev)
    s = (0.85 ** k).contiguous()                      # (1 - eta)^k, eta = 0.15
    c = (s * 2.0).sqrt().contiguous()                 # ((1 - eta)^k alpha2 / alpha1)^(1/2)
    w = (0.95 ** (k - 1) / (0.95 ** (k - 1)).sum()).contiguous()  # lambda^(k-1) / sum
    lo = [torch.empty(B, n, device=dev), torch.empty(B, n, device=dev), torch.empty(B, device=dev),
          torch.empty(1, device=dev), torch.empty(B, n, device=dev), torch.empty(B, n, device=dev)]

    def fl():
        N.lib().mh_msacl_lyapunov(*[N.ptr(t) for t in (logp, old, V, V2, obs, obs2, c, w, s)], 1.0, 2.0, 1.0, 10.0,
                                  B, n, D, *[N.ptr(t) for t in lo], st)
    ms = time_launches(fl, reps)
    res.append(row("msacl_lyapunov", "-", B, "windows", (4 * n + 2 * n * D) * 4 + (4 * n + 1) * 4, ms))
    V0 = torch.rand(B, device=dev, generator=g)
    adv_raw = torch.empty(B, device=dev)
    stats = torch.empty(2, dtype=torch.float64, device=dev)

    def fa():
        N.lib().mh_msacl_stability_adv(N.ptr(V0), N.ptr(V2), N.ptr(w), N.ptr(s), B, n, N.ptr(adv_raw), N.ptr(stats), st)
    ms = time_launches(fa, reps)
    res.append(row("msacl_stability_adv", "-", B, "windows", (1 + n) * 4 + 4, ms))
    ratio = 1.0 + 0.1 * r(B)
    adv, loss, dr = torch.empty(B, device=dev), torch.empty(1, device=dev), torch.empty(B, device=dev)

    def fp():
        N.lib().mh_msacl_ppo_clip(N.ptr(ratio), N.ptr(adv_raw), N.ptr(stats), float(B), 0.1, B, N.ptr(adv), N.ptr(loss),
                                  N.ptr(dr), st)
    ms = time_launches(fp, reps)
    res.append(row("msacl_ppo_clip", "-", B, "windows", 4 * 4, ms))
    return res


def bench_gae(E, H, reps, dev, p_done=0.02):
    """mh_gae over an [E][H] trajectory block (on-policy sampler, csrc/gae.hip)."""
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    val = torch.randn(E, H, device=dev, generator=g)
    val2 = torch.randn(E, H, device=dev, generator=g)
    rew = torch.randn(E, H, device=dev, generator=g)
    done = (torch.rand(E, H, device=dev, generator=g) < p_done).to(torch.uint8)
    adv, ret = torch.empty(E, H, device=dev), torch.empty(E, H, device=dev)
    st = N.stream_of(dev)

    def fn():
        N.lib().mh_gae(N.ptr(val), N.ptr(val2), N.ptr(rew), N.ptr(done), E, H, 0.99, 0.95, N.ptr(adv), N.ptr(ret), st)
    ms = time_launches(fn, reps)
    # val, rew, done in + adv, ret out, plus the bootstrap read at every segment end
    per = 4 + 4 + 1 + 4 + 4 + 4 * (p_done + 1.0 / H)
    return row("gae", "-", E * H, "steps", round(per, 3), ms, envs=E, horizon=H)


def bench_policy(E, reps, dev, D=12, A=4):
    """Sampler policy forward: fused f32-MFMA kernel (csrc/policy_mlp.hip) vs the PyTorch
    StochaPolicy MLP (hipBLASLt GEMMs, ReLU epilogues) on the same parameters."""
    import torch.nn as nn
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(D, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 2 * A)).to(dev)
    obs = torch.randn(E, D, device=dev)
    n = ctypes.c_int64()
    N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "size")
    P = torch.empty(n.value, device=dev)
    ps = [t.detach().contiguous() for t in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                            net[4].bias)]
    st = N.stream_of(dev)
    N.check(N.lib().mh_policy_pack(*[N.ptr(t) for t in ps], D, 256, 256, 2 * A, N.ptr(P), st), "pack")
    out = torch.empty(E, 2 * A, device=dev)

    def fused():
        N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, 2 * A, N.ptr(out), st)

    def torch_path():
        with torch.no_grad():
            h = torch._addmm_activation(net[0].bias, obs, net[0].weight.t())
            h = torch._addmm_activation(net[2].bias, h, net[2].weight.t())
            torch.addmm(net[4].bias, h, net[4].weight.t())

    flops = 2.0 * (D * 256 + 256 * 256 + 256 * 2 * A)
    rows = []
    for name, fn in (("policy_mlp_fused", fused), ("policy_mlp_torch", torch_path)):
        ms = time_launches(fn, reps)
        tf = E * flops / (ms * 1e-3) / 1e12
        r = {"kernel": name, "envs": E, "avg_us": round(ms * 1e3, 3), "TFLOPs": round(tf, 2),
             "frac_f32_mfma": round(tf / 157.3, 4)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    return rows


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", default="65536,4194304")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--envs", default=",".join(ENVS))
    p.add_argument("--skip", default="")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sizes = [int(x) for x in a.sizes.split(",")]
    skip = set(a.skip.split(","))
    rows = []
    if "env_step" not in skip:
        for name in a.envs.split(","):
            for E in sizes:
                rows.append(bench_env_step(name, E, a.reps, dev))
    if "rollout" not in skip:
        for name in a.envs.split(","):
            for E in sizes:
                rows += bench_rollout(name, E, a.reps, dev)
    if "gather" not in skip:
        for B in (256, 65536):
            rows.append(bench_gather("QuadTracking", B, a.reps, dev))
    if "msacl" not in skip:
        rows += bench_msacl(a.reps, dev)
    if "policy" not in skip:
        for E in (65536, 262144):
            rows += bench_policy(E, a.reps, dev)
    if "gae" not in skip:
        for E, H in ((65536, 64), (65536, 1600)):
            rows.append(bench_gae(E, H, a.reps, dev))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
