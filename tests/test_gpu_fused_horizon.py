"""GPU: the fused horizon sampler (csrc/sample_fused.hip, mh_sample_horizon: the whole horizon in
one persistent kernel + one emission launch) against the per-lockstep kernels it replaces
(k_policy_forward_x3 + k_rollout<Env, true> with deferred emission), which
tests/test_gpu_sampler_oracle.py pins to the oracle lockstep by lockstep.

Both paths run the same arithmetic (the split-f16 policy's MFMA sequence, the env step, the
Philox draws), so after each sample() — eager, graph capture, graph replay — the replay store
(rows and order), its cursor, the observations and the env state must be identical BIT FOR BIT,
for all six envs, at 65,536 envs and at env counts that leave a partial workgroup / wave."""
import ctypes

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.utils.config import build_pipeline
from msacl_amd.create_pkg.create_buffer import create_buffer
from msacl_amd.create_pkg.create_envs import create_envs
from msacl_amd.create_pkg.create_sampler import create_sampler
from msacl_amd.trainer.buffer.device_nstep_replay_buffer import KEYS
from msacl_amd.utils.config import default_msacl_args
from msacl_amd.utils.init_args import init_args
from oracle import envs as OE

pytestmark = pytest.mark.gpu


def _pair(name, E, n, tmp, noise=None, hover=False, horizon=20):
    out = []
    for fused in (True, False):
        args = default_msacl_args(env_name=name, env_num=E, n_step=n, seed=0, env_seed=5, buffer_max_size=600_000,
                                  buffer_warm_size=0, save_folder=str(tmp / str(fused)), noise_params=noise,
                                  sampler_fused_horizon=fused, sample_batch_size=horizon)
        args = init_args(create_envs(**args), **args)
        s, b = create_sampler(**args), create_buffer(**args)
        s.bind_store(b)
        out.append((s, b))
    (a, ba), (b, bb) = out
    b.networks.load_state_dict(a.networks.state_dict())
    if hover:  # long episodes: every ring fills (bench.py --policy hover)
        from bench import set_hover_policy
        for s in (a, b):
            set_hover_policy(s.networks.policy, float(s.envs.single_action_space.high[0]) / 2)
    assert a.fused_horizon and not b.fused_horizon
    return a, ba, b, bb


def _fused_errors(s):
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    N.check(N.lib().mh_sample_horizon_errors(s._h, N.ptr(out), N.stream_of()), "errors")
    return int(out.item())


def _assert_same(a, ba, b, bb, where):
    torch.cuda.synchronize()
    assert _fused_errors(a) == 0, where
    assert torch.equal(ba.cursor, bb.cursor), (where, ba.cursor.tolist(), bb.cursor.tolist())
    total = int(ba.cursor[1])
    for k in KEYS:
        x, y = ba.n_step_buf[k][:total], bb.n_step_buf[k][:total]
        assert torch.equal(x, y), (where, k, int((x != y).sum()))
    bad = []
    for nm, u, v in zip(("obs", "state", "xstate", "steps"), (a.obs,) + tuple(a.envs.get_state()),
                        (b.obs,) + tuple(b.envs.get_state())):
        if u is not None and not torch.equal(u, v):
            rows = (u != v).reshape(u.shape[0], -1).any(1).nonzero().flatten()
            d = (u.double() - v.double()).abs().max().item()
            bad.append((nm, int(rows.numel()), rows[:8].tolist(), d))
    assert not bad, (where, bad)
    return total


CASES = [(nm, 65536, 20, False) for nm in OE.ENVS] + [("QuadTracking", 65536, 20, True), ("QuadTracking", 4000, 20, False),
                                                     ("DuctedFan", 300, 3, False), ("TwoLink", 777, 5, False),
                                                     # 3,125 waves (196 cells of 16) per lockstep: each cell sums the
                                                     # earlier cells' counts
                                                     ("VanderPol", 200000, 20, False),
                                                     # 4,688 waves per lockstep (293 cells > FUSED_EMIT_SCAN_CELLS):
                                                     # k_emit_prefix
                                                     ("VanderPol", 300000, 20, False)]


@pytest.mark.parametrize("name,E,n,hover", CASES, ids=[f"{c[0]}-{c[1]}-n{c[2]}{'-hover' if c[3] else ''}" for c in CASES])
def test_fused_horizon_equals_lockstep_kernels(name, E, n, hover, tmp_path):
    a, ba, b, bb = _pair(name, E, n, tmp_path, hover=hover)
    total = 0
    for it in range(4):  # eager, capture + replay, replays
        a.sample()
        b.sample()
        total = _assert_same(a, ba, b, bb, f"sample {it}")
    assert total > 0


def test_fused_horizon_with_exploration_noise(tmp_path):
    """GaussNoise: one scalar per lockstep (base.py:136-137) — both paths read the same H draws."""
    a, ba, b, bb = _pair("DuctedFan", 65536, 20, tmp_path, noise={"mean": 0.0, "std": 0.3})
    b._draw_noise = lambda: None  # b replays a's draws
    for it in range(3):
        a.sample()
        b._noise.copy_(a._noise)
        b.sample()
        _assert_same(a, ba, b, bb, f"sample {it}")


def test_emission_relaunch_rewrites_the_same_rows(tmp_path):
    """mh_sample_horizon_emit (the emission launch alone, bench.py's timing of it) on the last
    horizon rewrites exactly the rows that horizon's emission wrote — into a wiped store, bit for
    bit, cursor untouched — and reports the horizon's window count."""
    a, ba, b, bb = _pair("QuadTracking", 65536, 20, tmp_path, hover=True)
    c0 = int(ba.cursor[2])
    a.sample()
    a.sample()  # the second horizon is the one re-emitted
    torch.cuda.synchronize()
    c_before = int(ba.cursor[2])
    a.sample()
    torch.cuda.synchronize()
    won = int(ba.cursor[2]) - c_before
    assert won > 0 and c0 >= 0
    snap = {k: ba.n_step_buf[k].clone() for k in KEYS}
    cur = ba.cursor.clone()
    for k in KEYS:
        ba.n_step_buf[k].fill_(-7.0)
    wins = torch.zeros(1, dtype=torch.int64, device="cuda")
    N.check(N.lib().mh_sample_horizon_emit(a._h, a.horizon, ctypes.byref(ba.ws), N.ptr(wins), N.stream_of()),
            "mh_sample_horizon_emit")
    torch.cuda.synchronize()
    assert int(wins) == won
    assert torch.equal(ba.cursor, cur)
    M = ba.max_size
    start = (int(cur[0]) - won) % M
    rows = (start + torch.arange(won, device="cuda")) % M
    for k in KEYS:
        assert torch.equal(ba.n_step_buf[k][rows], snap[k][rows]), k
    untouched = torch.ones(M, dtype=torch.bool, device="cuda")
    untouched[rows] = False
    assert bool((ba.n_step_buf["rew"][untouched] == -7.0).all())
    # only that horizon can be re-emitted: another horizon length, or any stepping / resetting
    # call on the handle since (here mh_rollout_flush), is refused without a launch
    assert N.lib().mh_sample_horizon_emit(a._h, a.horizon - 1, ctypes.byref(ba.ws), None, N.stream_of()) != 0
    N.check(N.lib().mh_rollout_flush(a._h, N.stream_of()), "mh_rollout_flush")
    assert N.lib().mh_sample_horizon_emit(a._h, a.horizon, ctypes.byref(ba.ws), None, N.stream_of()) != 0


def test_fused_horizon_needs_reserved_rings():
    info = N.env_info("VanderPol")
    h = ctypes.c_void_p()
    N.check(N.lib().mh_env_create(N.ENV_IDS["VanderPol"], 1024, 1, ctypes.byref(h)), "create")
    try:
        N.check(N.lib().mh_nstep_attach(h, 4, 1.0, 1.0), "attach")
        obs = torch.zeros(1024, info.obs_dim, device="cuda")
        P = torch.zeros(1 << 20, device="cuda")
        rc = N.lib().mh_sample_horizon(h, N.ptr(P), info.obs_dim, 2 * info.act_dim, N.ptr(obs), 8, None, None, None,
                                       None, N.stream_of())
        assert rc == -4  # MH_ESTATE: rings of n slots cannot hold a horizon's windows
        N.check(N.lib().mh_nstep_reserve(h, 4 + 8 - 1), "reserve")
        assert N.lib().mh_sample_horizon(h, N.ptr(P), info.obs_dim + 1, 2 * info.act_dim, N.ptr(obs), 8, None, None,
                                         None, None, N.stream_of()) == -1  # shape mismatch
        assert N.lib().mh_nstep_reserve(h, 3) == -1  # fewer slots than n_step
    finally:
        N.lib().mh_env_destroy(h)


def test_fused_horizon_of_one_lockstep(tmp_path):
    """sample_batch_size = 1 (a horizon of one lockstep, which the reference accepts): the rings keep
    n slots (mh_nstep_reserve(n + 0)) but the horizon's window lists are still sized, so the fused
    path runs and equals the lockstep kernels."""
    a, ba, b, bb = _pair("DuctedFan", 65536, 5, tmp_path, horizon=1)
    total = 0
    for it in range(8):
        a.sample()
        b.sample()
        total = _assert_same(a, ba, b, bb, f"sample {it}")
    assert total > 0


def test_fused_horizon_timeouts_are_loud(tmp_path):
    """A policy-wave wait that gives up (forced here by a spin limit of 1 poll) leaves garbage
    logits: the sampler must not carry on silently. check_errors() raises, close() raises after
    releasing its resources, every later call raises, and the trainer raises at its log interval."""
    args = default_msacl_args(env_name="VanderPol", env_num=65536, n_step=4, seed=0, env_seed=5,
                              buffer_max_size=600_000, buffer_warm_size=0, save_folder=str(tmp_path / "s"),
                              sampler_spin_limit=1)
    args = init_args(create_envs(**args), **args)
    s, b = create_sampler(**args), create_buffer(**args)
    s.bind_store(b)
    assert s.fused_horizon
    s.sample()
    torch.cuda.synchronize()
    assert _fused_errors(s) > 0
    with pytest.raises(RuntimeError, match="timed out"):
        s.check_errors()
    with pytest.raises(RuntimeError, match="timed out"):
        s.close()
    with pytest.raises(RuntimeError, match="closed"):
        s.sample()
    s.close()  # idempotent once closed

    args = default_msacl_args(env_name="VanderPol", env_num=4096, n_step=4, buffer_warm_size=512, buffer_max_size=50000,
                              max_iteration=4, log_save_interval=2, eval_interval=100, save_folder=str(tmp_path / "t"),
                              seed=0, replay_batch_size=64, sampler_spin_limit=1)
    *_, trainer = build_pipeline(args)
    with pytest.raises(RuntimeError, match="timed out"):
        for _ in range(3):
            trainer.step()
            trainer.iteration += 1
    try:
        trainer.close()
    except RuntimeError:
        pass
