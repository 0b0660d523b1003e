"""GPU: the env step at env counts that fill neither a wavefront nor a workgroup (E = 333, 1, 65)
through the C ABI, for every env: observation / real-next-observation rows (stored through the
per-wave LDS transpose for D >= 4, csrc/rollout.hip wave_store_rows) and rewards equal the
reference fixtures' rows (rtol = atol = 1e-5), and no output row at or beyond E is written
(the buffers carry sentinel rows past E)."""
import ctypes
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle import envs as OE

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = dict(rtol=1e-5, atol=1e-5)
SENTINEL = 7.25


@pytest.mark.parametrize("E", [333, 1, 65])
@pytest.mark.parametrize("name", list(OE.ENVS))
def test_env_step_ragged_counts_write_only_their_rows(name, E):
    g = np.load(os.path.join(G, f"env_{name}.npz"))
    dev = torch.device("cuda", 0)
    state = torch.tensor(g["state"][:E], device=dev)
    xstate = torch.tensor(g["xstate"][:E], device=dev) if "xstate" in g else None
    steps = torch.tensor(g["steps"][:E], dtype=torch.int32, device=dev)
    act = torch.tensor(g["act"][:E], device=dev).contiguous()
    D = g["obs"].shape[1]
    pad = 70  # more than one wavefront of sentinel rows past E
    nxt = torch.full((E + pad, D), SENTINEL, device=dev)
    real = torch.full((E + pad, D), SENTINEL, device=dev)
    rew = torch.full((E + pad,), SENTINEL, device=dev)
    term = torch.full((E + pad,), 9, dtype=torch.uint8, device=dev)
    trunc = torch.full((E + pad,), 9, dtype=torch.uint8, device=dev)
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS[name], E, 1234, ctypes.byref(h)), "mh_env_create")
    try:
        st = N.stream_of(dev)
        N.check(N.lib().mh_env_set_state(h, N.ptr(state), N.ptr(xstate) if xstate is not None else None,
                                         N.ptr(steps), st), "mh_env_set_state")
        N.check(N.lib().mh_env_step(h, N.ptr(act), None, N.ptr(nxt), N.ptr(real), N.ptr(rew), N.ptr(term),
                                    N.ptr(trunc), st), "mh_env_step")
        torch.cuda.synchronize()
    finally:
        N.lib().mh_env_destroy(h)
    real_np, rew_np = real.cpu().numpy(), rew.cpu().numpy()
    np.testing.assert_allclose(real_np[:E], g["obs"][:E], **TOL)
    np.testing.assert_allclose(rew_np[:E], g["reward"][:E].astype(np.float32), **TOL)
    done = g["terminated"][:E].astype(bool) | g["truncated"][:E].astype(bool)
    np.testing.assert_allclose(nxt.cpu().numpy()[:E][~done], g["obs"][:E][~done], **TOL)
    assert np.all(nxt.cpu().numpy()[E:] == SENTINEL) and np.all(real_np[E:] == SENTINEL)
    assert np.all(rew_np[E:] == SENTINEL)
    assert np.all(term.cpu().numpy()[E:] == 9) and np.all(trunc.cpu().numpy()[E:] == 9)


@pytest.mark.parametrize("E", [1000, 4099])
def test_car_kinematic_lanes_match_oracle(E):
    """SingleTrackCar's kinematic model (|v| < 0.1, SingleTrackCar.py:199-204, 259-277), which the
    reference fixtures (speeds drawn from the reset box) never reach: states with a third of the
    speeds near the switch (some crossing it inside the five substeps, so waves mix both models)
    against the oracle's env_step: real next observations, rewards and states of non-terminal
    envs at rtol = atol = 1e-5, termination away from the box boundary exactly."""
    name = "SingleTrackCar"
    rng = np.random.default_rng(E)
    cls = OE.ENVS[name]
    st = rng.uniform(0.8 * cls.obs_low, 0.8 * cls.obs_high, size=(E, 7)).astype(np.float32)
    near = rng.random(E) < 1 / 3
    st[near, 3] = rng.uniform(-1.0, -0.8, size=int(near.sum())).astype(np.float32)  # v = ve + 1 in [0, 0.2]
    act = rng.uniform(-5, 5, size=(E, 2)).astype(np.float32)
    steps = rng.integers(0, 998, size=E).astype(np.int32)
    s_o, _, o_o, r_o, te_o, tr_o = OE.env_step(name, st, act, None, steps)
    dev = torch.device("cuda", 0)
    state = torch.tensor(st, device=dev)
    k = torch.tensor(steps, device=dev)
    a = torch.tensor(act, device=dev)
    nxt, real = torch.empty(E, 7, device=dev), torch.empty(E, 7, device=dev)
    rew = torch.empty(E, device=dev)
    term = torch.empty(E, dtype=torch.uint8, device=dev)
    trunc = torch.empty(E, dtype=torch.uint8, device=dev)
    out_state = torch.empty(E, 7, device=dev)
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS[name], E, 99, ctypes.byref(h)), "mh_env_create")
    try:
        s_ = N.stream_of(dev)
        N.check(N.lib().mh_env_set_state(h, N.ptr(state), None, N.ptr(k), s_), "set_state")
        N.check(N.lib().mh_env_step(h, N.ptr(a), None, N.ptr(nxt), N.ptr(real), N.ptr(rew), N.ptr(term),
                                    N.ptr(trunc), s_), "mh_env_step")
        N.check(N.lib().mh_env_get_state(h, N.ptr(out_state), None, None, s_), "get_state")
        torch.cuda.synchronize()
    finally:
        N.lib().mh_env_destroy(h)
    np.testing.assert_allclose(real.cpu().numpy(), o_o, **TOL)
    np.testing.assert_allclose(rew.cpu().numpy(), r_o.astype(np.float32), **TOL)
    te = term.cpu().numpy().astype(bool)
    ok = ~np.any((np.abs(o_o - cls.obs_low) < 1e-4) | (np.abs(o_o - cls.obs_high) < 1e-4), axis=1)
    np.testing.assert_array_equal(te[ok], te_o[ok])
    np.testing.assert_array_equal(trunc.cpu().numpy().astype(bool), tr_o)
    done = te | tr_o
    np.testing.assert_allclose(out_state.cpu().numpy()[~done], s_o[~done], **TOL)
    np.testing.assert_allclose(nxt.cpu().numpy()[~done], o_o[~done], **TOL)
    # the kinematic model was exercised: some speeds were below the switch during the step
    assert (np.abs(st[:, 3] + 1.0) < 0.1).sum() > 10
