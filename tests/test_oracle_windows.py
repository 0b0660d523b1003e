"""CPU: the array form of the n-step window assembly (oracle.sampler.NStepWindows, used by the
65,536-env GPU parity tests) equals the per-env deque restatement (oracle.sampler.NStepRollout,
bit-exact against the reference's own _n_step traces in test_oracle_golden.py) window for
window, including clears on termination and truncation (RL/trainer/sampler/base.py:178-217)."""
import numpy as np
import pytest

from oracle import envs as OE
from oracle import sampler as OS


@pytest.mark.parametrize("name,n", [("Pendulum", 5), ("VanderPol", 3), ("DuctedFan", 20)])
def test_array_windows_equal_deque_windows(name, n):
    E, T = 48, 90
    cls = OE.ENVS[name]
    rng = np.random.default_rng(7)
    venv = OS.VectorEnv(name, E, lambda idx: cls.reset_draw(rng, len(idx)))
    ro = OS.NStepRollout(venv, n)
    venv.steps[:] = rng.integers(900, 999, size=E)  # truncations inside the run
    nw = OS.NStepWindows(E, n, cls.obs_dim, cls.act_dim)
    lo, hi = cls.act_low.astype(np.float64), cls.act_high.astype(np.float64)
    seen = dones = 0
    for _ in range(T):
        act = (lo + (hi - lo) * rng.uniform(size=(E, lo.size))).astype(np.float32)
        logp = rng.standard_normal(E).astype(np.float32)
        obs = np.float32(ro.obs).copy()
        wins, info = ro.step(act, logp)
        got = nw.push(obs, act, info["rew"], info["cost"], info["real_next_obs"], info["done"], logp)
        assert got[0].shape[0] == len(wins)
        for j in range(7):
            exp = np.stack([w[j] for w in wins]) if wins else np.zeros((0, n), np.float32)
            np.testing.assert_array_equal(got[j].reshape(exp.shape), exp)
        seen += len(wins)
        dones += int(info["done"].sum())
    assert seen > 0 and dones > 0
