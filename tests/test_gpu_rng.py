"""GPU: the engine's in-kernel random draws against their restatement in oracle/rng.py.

The reference draws the TanhGauss noise from torch's CPU generator
(RL/utils/act_distribution_cls.py:46) and reset states from numpy's
(RL/env/<Env>.py reset(), e.g. VanderPol.py:79-82, QuadTracking.py:169-186); neither can be
replayed on a device, so the engine keys Philox4x32-10 by (seed, env, the env's counter)
(csrc/philox.h). Pinned here, through mh_rng_draw (the same inline draws the rollout and fused
sampler kernels make) and through the env batch itself:
  * the action normals equal the oracle's float64 Box–Muller of the same uniforms within a few
    float32 ulp of the Box–Muller radius (the kernel uses the hardware transcendentals);
  * every uniform reset component is BIT-EXACT; QuadTracking's rotation block within 2e-7;
  * mh_env_reset draws at each env's counter and advances it by one, for keys with high bits set.
"""
import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.env.hip_vector_env import HipVectorEnv
from oracle import rng as OR

pytestmark = pytest.mark.gpu
SEED = 0x1234_5678_9ABC_DEF0


def _draw(name, kind, env, ctr, seed=SEED):
    n = env.shape[0]
    width = 4 if kind == 0 else N.env_info(name).reset_dim
    out = torch.empty(n, width, device="cuda")
    e = torch.as_tensor(env, dtype=torch.int64, device="cuda")
    c = torch.as_tensor(ctr.astype(np.uint32).view(np.int32), device="cuda")
    N.check(N.lib().mh_rng_draw(N.ENV_IDS[name], kind, seed, N.ptr(e), N.ptr(c), n, N.ptr(out), N.stream_of()),
            "mh_rng_draw")
    return out.cpu().numpy()


def _keys(n, seed=7):
    rng = np.random.default_rng(seed)
    env = rng.integers(0, 1 << 40, size=n, dtype=np.int64)  # high words exercised
    env[:4096] = np.arange(4096)
    ctr = rng.integers(0, 1 << 32, size=n, dtype=np.int64)
    ctr[:16] = [0, 1, 2, 3, 0xFFFFFFFF, 0xFFFFFFFE, 1000, 1 << 31] + list(range(8))
    return env, ctr


def test_action_normals_match_oracle():
    env, ctr = _keys(1 << 20)
    got = _draw("QuadTracking", 0, env, ctr).astype(np.float64)
    q = OR.draw_words(SEED, env, ctr, 0)
    want = OR.box_muller(q)
    r = OR.box_muller_radius(q)
    err = np.abs(got - want) / np.maximum(r, 1.0)
    print("action normals: max |err| / max(1, radius) =", err.max(), "; max |err| =", np.abs(got - want).max())
    # v_log_f32 / v_sqrt_f32 / v_sin_f32 / v_cos_f32 (a few ulp each) on the exact uniforms
    assert err.max() < 6e-7, err.max()  # measured 2.5e-7 (1M draws)
    assert abs(got.mean()) < 5e-3 and abs(got.std() - 1.0) < 5e-3


@pytest.mark.parametrize("name", list(N.ENV_IDS))
def test_reset_draws_match_oracle(name):
    env, ctr = _keys(1 << 18, seed=11)
    got = _draw(name, 1, env, ctr)
    want = OR.reset_draw(name, SEED, env, ctr)
    if name == "QuadTracking":
        uni = np.r_[0:6, 15:18]
        np.testing.assert_array_equal(got[:, uni], want[:, uni])
        np.testing.assert_allclose(got[:, 6:15], want[:, 6:15], rtol=0, atol=2e-7)
    else:
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name", list(N.ENV_IDS))
def test_env_reset_draws_at_the_counters(name):
    """HipVectorEnv.reset() (mh_env_reset without states): env e restarts from the oracle's draw at
    its counter, and every counter advances by one."""
    E = 70000
    env = HipVectorEnv(name, E, seed=SEED)
    try:
        env.reset()
        c0 = env.get_counters().cpu().numpy()
        assert (c0 == 1).all()
        start = np.random.default_rng(3).integers(0, 1 << 32, size=E, dtype=np.int64)
        env.set_counters(torch.as_tensor(start.astype(np.uint32).view(np.int32)))
        env.reset()
        st, _, steps = env.get_state()
        want = OR.reset_draw(name, SEED, np.arange(E), start)
        got = st.cpu().numpy()
        if name == "QuadTracking":
            uni = np.r_[0:6, 15:18]
            np.testing.assert_array_equal(got[:, uni], want[:, uni])
            np.testing.assert_allclose(got[:, 6:15], want[:, 6:15], rtol=0, atol=2e-7)
        else:
            np.testing.assert_array_equal(got, want)
        assert (steps.cpu().numpy() == 0).all()
        np.testing.assert_array_equal(env.get_counters().cpu().numpy(), (start + 1) & 0xFFFFFFFF)
    finally:
        env.close()
