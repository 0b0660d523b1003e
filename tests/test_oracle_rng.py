"""CPU: oracle/rng.py (the restatement of the engine's in-kernel draws) pinned without a GPU.

* Its Philox keying equals oracle/per.py's (itself pinned by the Random123 known-answer vectors,
  tests/test_per_oracle.py) for scalar ticks.
* The engine's CPU build (libmsacl_host.so) compiles the SAME reset_draw.h / philox.h as the gfx950
  kernels: its drawn resets equal the oracle's bit for bit (QuadTracking's float32 rotation within
  2e-7 of the oracle's float64 one) — the host half of tests/test_gpu_rng.py.
* The Box–Muller normals are standard normal; the stable TanhGauss log-Jacobian equals the direct
  float64 formula where that one has no cancellation.
"""
import ctypes

import numpy as np
import pytest

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle import per as OP
from oracle import rng as OR

SEED = 0x1234_5678_9ABC_DEF0


def test_draw_words_matches_per_oracle_keying():
    units = np.arange(1000)
    for tick in (0, 1, 77, 0xFFFFFFFF, 1 << 40):
        np.testing.assert_array_equal(OR.draw_words(SEED, units, np.full(1000, tick), 9),
                                      OP.draw_words(SEED, units, tick, 9))


@pytest.mark.parametrize("name", list(N.ENV_IDS))
def test_host_engine_reset_draws_equal_oracle(name):
    info = N.host_env_info(name)
    E = 4096
    h = ctypes.c_void_p()
    N.host_check(N.host_lib().mhh_env_create(N.ENV_IDS[name], E, SEED, ctypes.byref(h)), "create")
    try:
        obs = np.empty((E, info.obs_dim), np.float32)
        N.host_check(N.host_lib().mhh_env_reset(h, None, N.hptr(obs)), "reset")   # counters 0 -> 1
        N.host_check(N.host_lib().mhh_env_reset(h, None, N.hptr(obs)), "reset")   # draws at counter 1
        st = np.empty((E, info.state_dim), np.float32)
        N.host_check(N.host_lib().mhh_env_get_state(h, N.hptr(st), None, None), "state")
    finally:
        N.host_lib().mhh_env_destroy(h)
    want = OR.reset_draw(name, SEED, np.arange(E), np.ones(E, np.int64))
    if name == "QuadTracking":
        uni = np.r_[0:6, 15:18]
        np.testing.assert_array_equal(st[:, uni], want[:, uni])
        np.testing.assert_allclose(st[:, 6:15], want[:, 6:15], rtol=0, atol=2e-7)
        R = want[:, 6:15].reshape(E, 3, 3).astype(np.float64)
        assert np.abs(R @ np.transpose(R, (0, 2, 1)) - np.eye(3)).max() < 1e-6
    else:
        np.testing.assert_array_equal(st, want)


def test_action_normals_are_standard_normal():
    eps = OR.action_normals(SEED, np.arange(1 << 18), np.full(1 << 18, 5))
    e = eps.reshape(-1)
    assert abs(e.mean()) < 5e-3 and abs(e.std() - 1.0) < 5e-3
    np.testing.assert_allclose(np.quantile(e, [0.05, 0.25, 0.5, 0.75, 0.95]),
                               [-1.6449, -0.6745, 0.0, 0.6745, 1.6449], atol=0.01)
    # the four components are independent draws
    c = np.corrcoef(eps.T)
    assert np.abs(c - np.eye(4)).max() < 0.01


def test_tanh_gauss_stable_form_equals_direct_formula():
    rng = np.random.default_rng(0)
    n, A = 100000, 4
    logits = np.concatenate([rng.uniform(-2, 2, (n, A)), rng.uniform(-2, 0.5, (n, A))], 1).astype(np.float32)
    eps = rng.standard_normal((n, A))
    lo, hi = -np.ones(A), np.ones(A)
    act, lp = OR.tanh_gauss_sample(logits, eps, lo, hi)
    mu = logits[:, :A].astype(np.float64)
    c = np.clip(logits[:, A:], -20, 1).astype(np.float64)
    sd = np.exp(c).astype(np.float32).astype(np.float64)
    z = (mu + (sd * eps).astype(np.float32)).astype(np.float32).astype(np.float64)
    direct = (-((z - mu) ** 2) / (2 * sd * sd) - c - 0.5 * np.log(2 * np.pi)).sum(1)
    direct = direct - np.log(OR.ONE_PLUS_EPS - np.tanh(z) ** 2).sum(1)  # f64: <= 1e-10 of cancellation here
    np.testing.assert_allclose(lp, direct, rtol=1e-12, atol=1e-10)
    np.testing.assert_allclose(act, np.tanh(z), rtol=0, atol=1e-15)
