"""GPU: the in-kernel TanhGauss sampler of the fused rollout step (throughput mode) against
TanhGaussDistribution.sample's math (RL/utils/act_distribution_cls.py:45-57).

The policy's noise comes from torch's CPU generator in the reference and cannot be replayed on
the device, so the check is: (1) recover z = atanh((2a - (h+l)) / (h-l)) from every unclipped
action and require eps = (z - mu) / std to be standard normal (moments, quantiles); (2) the
kernel's log-prob equals Normal(mu, std).log_prob(z) - sum log(1 + 1e-6 - tanh(z)^2)
- sum log((h-l)/2) evaluated in float64 on the recovered z (tolerance from the atanh
conditioning, |tanh z| < 0.95 rows only); (3) the std clamp of StochaPolicy (log_std clamped to
[-20, 1]) is applied in-kernel."""
import ctypes

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N

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
        act, logp = torch.empty(E, A, device="cuda"), torch.empty(E, device="cuda")
        N.check(N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(obs), None, N.ptr(act), N.ptr(logp), st),
                "rollout")
        torch.cuda.synchronize()
    finally:
        N.lib().mh_env_destroy(h)
    lo = np.array(info.act_low[:A], np.float64)
    hi = np.array(info.act_high[:A], np.float64)
    return mu.cpu().double().numpy(), ls.cpu().double().numpy(), act.cpu().double().numpy(), logp.cpu().double().numpy(), lo, hi


@pytest.mark.parametrize("name", ["QuadTracking", "DuctedFan", "VanderPol"])
def test_in_kernel_tanh_gauss_sample(name):
    """|mu| <= 0.5 and std <= e^-1.5 keep |z| < 2 (|tanh z| < 0.97) for |eps| < 6: the pre-tanh
    sample is recoverable without truncating the eps distribution."""
    E = 262144
    mu, ls, act, logp, lo, hi = _sample(name, E, lo_ls=-3.0, hi_ls=-1.5, mu_scale=0.5)
    sd = np.exp(np.clip(ls, -20, 1))
    th = (2 * act - (hi + lo)) / (hi - lo)
    z = np.arctanh(th)
    eps = (z - mu) / sd
    ok = np.ones_like(eps, dtype=bool)
    e = eps.reshape(-1)
    assert abs(e.mean()) < 0.01 and abs(e.std() - 1) < 0.01, (e.mean(), e.std())
    qs = np.quantile(e, [0.05, 0.25, 0.5, 0.75, 0.95])
    np.testing.assert_allclose(qs, [-1.6449, -0.6745, 0.0, 0.6745, 1.6449], atol=0.02)
    # log-prob on the recovered pre-tanh sample (float64); the recovery through atanh of a
    # float32 action is good to ~1e-6 in z, i.e. ~1e-6 / std^2 * |z - mu| in the log-prob
    lp = (-((z - mu) ** 2) / (2 * sd ** 2) - np.log(sd) - 0.5 * np.log(2 * np.pi)).sum(1)
    lp = lp - np.log(1 + 1e-6 - np.tanh(z) ** 2).sum(1) - np.log((hi - lo) / 2).sum()
    np.testing.assert_allclose(logp, lp, rtol=1e-4, atol=5e-3)
    assert ((act >= lo) & (act <= hi)).all()


def test_in_kernel_std_clamp():
    """log_std below -20 is clamped (std = e^-20): the action is then tanh(mu) up to rounding."""
    mu, ls, act, logp, lo, hi = _sample("VanderPol", 65536, lo_ls=-40.0, hi_ls=-30.0)
    expect = (hi - lo) / 2 * np.tanh(mu) + (hi + lo) / 2
    np.testing.assert_allclose(act, expect, rtol=1e-5, atol=1e-5)
    # z - mu is 0 or one float32 ulp of mu (std*eps is below half an ulp): the log-prob is then
    # +20 - 0.92 - log(5) + ... or hugely negative, exactly as float32 torch computes it
    assert np.isfinite(logp).all()
    assert (np.abs(logp - (20 - 0.5 * np.log(2 * np.pi) - np.log(5.0)
                           - np.log(1 + 1e-6 - np.tanh(mu[:, 0]) ** 2)) < 1e-3) | (logp < -10)).all()
