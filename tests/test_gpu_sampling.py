"""GPU: the in-kernel TanhGauss sampler of the rollout step (throughput mode) against
TanhGaussDistribution.sample (RL/utils/act_distribution_cls.py:45-57) restated by the oracle.

The reference draws its noise from torch's CPU generator, which no device can replay; the engine
draws it in-kernel from Philox keyed by (seed, env, the env's counter). oracle/rng.py replays those
draws from the seed and the counters (tests/test_gpu_rng.py pins them), so every sampled action and
log-prob is compared with the float64 TanhGauss of (the kernel's logits, the oracle's eps) at
rtol = atol = 1e-5 — every row, saturated actions included (|z| up to ~12). Also: the recovered
pre-tanh noise is standard normal, and StochaPolicy's std clamp (log_std in [-20, 1]) is applied
in-kernel."""
import ctypes

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle import rng as OR

pytestmark = pytest.mark.gpu


def _sample(name, E, seed=11, lo_ls=-3.0, hi_ls=0.5, mu_scale=1.0):
    info = N.env_info(name)
    D, A = info.obs_dim, info.act_dim
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS[name], E, seed, ctypes.byref(h)), "create")
    try:
        N.check(N.lib().mh_nstep_attach(h, 2, 1.0, 1.0), "attach")
        N.check(N.lib().mh_nstep_set_log_std_clamp(h, 1, -20.0, 1.0), "clamp")
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        mu = (torch.rand(E, A, device="cuda", generator=g) * 2 - 1) * mu_scale
        ls = lo_ls + (hi_ls - lo_ls) * torch.rand(E, A, device="cuda", generator=g)
        logits = torch.cat([mu, ls], dim=1).contiguous()
        obs = torch.empty(E, D, device="cuda")
        st = N.stream_of()
        N.check(N.lib().mh_env_reset(h, None, N.ptr(obs), st), "reset")
        ctr = torch.empty(E, dtype=torch.int32, device="cuda")
        N.check(N.lib().mh_env_get_counters(h, N.ptr(ctr), st), "counters")
        act, logp = torch.empty(E, A, device="cuda"), torch.empty(E, device="cuda")
        N.check(N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(obs), None, N.ptr(act), N.ptr(logp), st),
                "rollout")
        torch.cuda.synchronize()
    finally:
        N.lib().mh_env_destroy(h)
    lo = np.array(info.act_low[:A], np.float64)
    hi = np.array(info.act_high[:A], np.float64)
    # the oracle's TanhGauss of (these logits, the eps this env drew at its counter)
    eps = OR.action_normals(seed, np.arange(E), ctr.cpu().numpy().astype(np.int64) & 0xFFFFFFFF)
    a_o, lp_o = OR.tanh_gauss_sample(logits.cpu().numpy(), eps, lo, hi)
    return (mu.cpu().double().numpy(), ls.cpu().double().numpy(), act.cpu().double().numpy(),
            logp.cpu().double().numpy(), lo, hi, a_o, lp_o)


@pytest.mark.parametrize("regime", ["moderate", "saturating"])
@pytest.mark.parametrize("name", list(N.ENV_IDS))
def test_in_kernel_tanh_gauss_sample_matches_oracle(name, regime):
    """Every row at 1e-5: moderate logits (|z| < 2) and saturating ones (|mean| <= 4, std up to e,
    so |tanh z| reaches 1 - 1e-10 and the clip bites)."""
    kw = dict(lo_ls=-3.0, hi_ls=-1.5, mu_scale=0.5) if regime == "moderate" else dict(lo_ls=-1.0, hi_ls=1.0, mu_scale=4.0)
    _, _, act, logp, lo, hi, a_o, lp_o = _sample(name, 262144, **kw)
    # the action on the distribution's own scale, tanh(z) = (a - mid) / half (act_distribution_cls.py:
    # 47-50): when mean and std * eps nearly cancel, the float32 sample z itself carries ~1 ulp of
    # |mean| (the reference's as well as the kernel's), which the env's half-range (20 for TwoLink,
    # 42.5 for QuadTracking's thrust) then scales
    half, mid = (hi - lo) / 2, (hi + lo) / 2
    np.testing.assert_allclose((act - mid) / half, (a_o - mid) / half, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(act, a_o, rtol=1e-5, atol=1e-5 * np.maximum(1.0, half).max())
    np.testing.assert_allclose(logp, lp_o, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", ["QuadTracking", "DuctedFan", "VanderPol"])
def test_in_kernel_tanh_gauss_noise_is_standard_normal(name):
    """|mu| <= 0.5 and std <= e^-1.5 keep |z| < 2 (|tanh z| < 0.97) for |eps| < 6: the pre-tanh
    sample is recoverable from the action without truncating the eps distribution."""
    E = 262144
    mu, ls, act, logp, lo, hi, _, _ = _sample(name, E, lo_ls=-3.0, hi_ls=-1.5, mu_scale=0.5)
    sd = np.exp(np.clip(ls, -20, 1))
    th = (2 * act - (hi + lo)) / (hi - lo)
    z = np.arctanh(th)
    eps = (z - mu) / sd
    e = eps.reshape(-1)
    assert abs(e.mean()) < 0.01 and abs(e.std() - 1) < 0.01, (e.mean(), e.std())
    qs = np.quantile(e, [0.05, 0.25, 0.5, 0.75, 0.95])
    np.testing.assert_allclose(qs, [-1.6449, -0.6745, 0.0, 0.6745, 1.6449], atol=0.02)
    assert ((act >= lo) & (act <= hi)).all()


def test_in_kernel_std_clamp():
    """log_std below -20 is clamped (std = e^-20): the action is then tanh(mu) up to rounding."""
    mu, ls, act, logp, lo, hi, _, _ = _sample("VanderPol", 65536, lo_ls=-40.0, hi_ls=-30.0)
    expect = (hi - lo) / 2 * np.tanh(mu) + (hi + lo) / 2
    np.testing.assert_allclose(act, expect, rtol=1e-5, atol=1e-5)
    # z - mu is 0 or one float32 ulp of mu (std*eps is below half an ulp): the log-prob is then
    # +20 - 0.92 - log(5) + ... or hugely negative, exactly as float32 torch computes it
    assert np.isfinite(logp).all()
    assert (np.abs(logp - (20 - 0.5 * np.log(2 * np.pi) - np.log(5.0)
                           - np.log(1 + 1e-6 - np.tanh(mu[:, 0]) ** 2)) < 1e-3) | (logp < -10)).all()
