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
