"""GPU parity of the n-step window path: fused rollout step (injected actions) + scan +
emission into the device store vs the reference's own _n_step traces (tests/golden/nstep_*),
FIFO wrap of the store, and the replay gather."""
import ctypes
import glob
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.env.hip_vector_env import HipVectorEnv
from msacl_amd.trainer.buffer.device_nstep_replay_buffer import KEYS, DeviceNstepReplayBuffer
from oracle import envs as OE

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
TOL = dict(rtol=1e-5, atol=1e-5)
TRACES = sorted(glob.glob(os.path.join(G, "nstep_*.npz")))


def _run_trace(path, capacity=None, tile=1, check_obs=False, deferred=False, g=None, ring_slots=None):
    """Replay a reference _n_step trace through the fused rollout (injected actions); deferred:
    through mh_rollout_step_deferred (each step's windows emitted by the next step's emitter
    waves) and a final mh_rollout_flush. `g` overrides the fixture (a sliced trace)."""
    g = np.load(path) if g is None else g
    name = os.path.basename(path)[6:-4].replace("_n20", "")
    # TwoLink's upright arm is open-loop unstable: under the trace's recorded (feedback) torques
    # replayed open loop, ulp-level differences grow ~e-fold every few steps (2e-5 by step 12 of
    # the n = 20 trace). Re-anchor its state (== obs) to the reference's after every step, so each
    # window entry is one kernel step from the reference's own state.
    anchor = name == "TwoLink" and n_of(g) == 20
    E0, T, n = g["init_reset"].shape[0], g["actions"].shape[0], int(g["n_step"])
    E = E0 * tile
    tl = lambda a: np.concatenate([a] * tile, axis=0)  # noqa: E731
    env = HipVectorEnv(name, E, seed=1)
    h = env.handle()
    N.check(N.lib().mh_nstep_attach(h, n, 100.0, 100.0), "attach")
    if ring_slots is not None:  # rings longer than n (the fused horizon sampler's layout)
        N.check(N.lib().mh_nstep_reserve(h, n + ring_slots), "reserve")
    obs, _ = env.reset(reset_states=tl(g["init_reset"]))
    env.set_state(None, None, tl(g["init_steps"]))
    total = int(g["counts"].sum()) * tile
    buf = DeviceNstepReplayBuffer(obs_dim=env.obs_dim, act_dim=env.act_dim, buffer_max_size=capacity or total + 7,
                                  n_step=n)
    dev = obs.device
    for t in range(T):
        act = torch.as_tensor(tl(g["actions"][t]), device=dev).contiguous()
        lp = torch.as_tensor(tl(g["logp"][t]), device=dev).contiguous()
        rs = torch.as_tensor(tl(g["resets"][t]), device=dev).contiguous()
        fn = N.lib().mh_rollout_step_deferred if deferred else N.lib().mh_rollout_step
        N.check(fn(h, None, N.ptr(act), N.ptr(lp), N.ptr(rs), N.ptr(obs), ctypes.byref(buf.ws), None, None,
                   N.stream_of(dev)), "rollout")
        if tile == 1:
            np.testing.assert_allclose(obs.cpu().numpy(), g["obs_trace"][t + 1], **TOL)
        elif check_obs:
            ref = torch.as_tensor(g["obs_trace"][t + 1], device=dev).repeat(tile, 1)
            assert ((obs - ref).abs() <= TOL["atol"] + TOL["rtol"] * ref.abs()).all(), f"obs at step {t}"
        if anchor:
            ref = torch.as_tensor(tl(g["obs_trace"][t + 1]), device=dev).contiguous()
            env.set_state(ref)
            obs.copy_(ref)
    N.check(N.lib().mh_rollout_flush(h, N.stream_of(dev)), "flush")
    torch.cuda.synchronize()
    return g, buf, total, tile


def _expected_windows(g, tile):
    """Window order of a tiled trace: per step, env-index order over the tiled envs."""
    if tile == 1:
        return {k: g["w_" + k] for k in KEYS}
    out = {k: [] for k in KEYS}
    off = 0
    for c in g["counts"]:
        for _ in range(tile):
            for k in KEYS:
                out[k].append(g["w_" + k][off:off + c])
        off += c
    return {k: np.concatenate(v) for k, v in out.items()}


@pytest.mark.parametrize("deferred", [False, True], ids=["immediate", "deferred"])
@pytest.mark.parametrize("path", TRACES, ids=os.path.basename)
def test_windows_match_reference_sampler(path, deferred):
    g, buf, total, _ = _run_trace(path, deferred=deferred)
    assert buf.size == total and int(buf.cursor[2]) == total
    for k in KEYS:
        np.testing.assert_allclose(buf.n_step_buf[k][:total].cpu().numpy(), g["w_" + k], **TOL, err_msg=k)
    assert not buf.n_step_buf["done"][:total, :-1].any()


@pytest.mark.parametrize("extra", [1, 19])
@pytest.mark.parametrize("deferred", [False, True], ids=["immediate", "deferred"])
@pytest.mark.parametrize("path", TRACES, ids=os.path.basename)
def test_windows_with_longer_rings(path, deferred, extra):
    """Rings of n + extra slots (mh_nstep_reserve) give the same windows, in the same order."""
    g, buf, total, _ = _run_trace(path, deferred=deferred, ring_slots=extra)
    assert buf.size == total and int(buf.cursor[2]) == total
    for k in KEYS:
        np.testing.assert_allclose(buf.n_step_buf[k][:total].cpu().numpy(), g["w_" + k], **TOL, err_msg=k)


@pytest.mark.parametrize("deferred", [False, True], ids=["immediate", "deferred"])
@pytest.mark.parametrize("path", TRACES[:2], ids=os.path.basename)
def test_windows_tiled_to_many_envs(path, deferred):
    g, buf, total, tile = _run_trace(path, tile=256, deferred=deferred)
    exp = _expected_windows(g, tile)
    for k in KEYS:
        np.testing.assert_allclose(buf.n_step_buf[k][:total].cpu().numpy(), exp[k], **TOL, err_msg=k)


@pytest.mark.parametrize("cap", [37, 100])
def test_store_fifo_wrap(cap):
    path = os.path.join(G, "nstep_VanderPol.npz")
    g, buf, total, _ = _run_trace(path, capacity=cap)
    assert buf.size == cap and buf.ptr == total % cap
    rows = (np.arange(total - cap, total)) % cap
    for k in KEYS:
        np.testing.assert_allclose(buf.n_step_buf[k].cpu().numpy()[rows], g["w_" + k][total - cap:], **TOL)


def test_replay_gather_and_indices():
    path = os.path.join(G, "nstep_DuctedFan.npz")
    g, buf, total, _ = _run_trace(path)
    idx = torch.tensor([0, 5, total - 1, 3, 3], device="cuda")
    out = buf.gather(idx)
    for k in KEYS:
        np.testing.assert_allclose(out[k].cpu().numpy(), g["w_" + k][idx.cpu().numpy()], **TOL)
    draws = buf.sample_indices(100000).cpu().numpy()
    assert draws.min() >= 0 and draws.max() < total
    counts = np.bincount(draws, minlength=total)
    assert counts.min() > 0.5 * 100000 / total  # roughly uniform
    batch = buf.sample_batch(256)
    assert batch["obs"].shape == (256, int(g["n_step"]), 6) and batch["rew"].shape == (256, int(g["n_step"]))
    assert "obs_act" not in batch and "v_in" not in batch  # the reference's seven keys unless asked


def test_replay_gather_joint_layouts():
    """mh_replay_gather_joint: the update's [obs | act] rows and [obs[:, 0]; obs2 rows] batch equal
    the torch.cat of the gathered arrays the update would otherwise form (msacl.py:236-238, 395-396),
    bit for bit, fresh and into static destinations (also with repeated / boundary indices)."""
    path = os.path.join(G, "nstep_DuctedFan.npz")
    g, buf, total, _ = _run_trace(path)
    idx = torch.tensor([0, 5, total - 1, 3, 3, total - 2], device="cuda")
    out = buf.gather(idx, joint=True)
    n, D = out["obs"].shape[1], out["obs"].shape[2]
    torch.testing.assert_close(out["obs_act"], torch.cat([out["obs"], out["act"]], -1), rtol=0, atol=0)
    torch.testing.assert_close(out["v_in"], torch.cat([out["obs"][:, 0], out["obs2"].reshape(-1, D)], 0),
                               rtol=0, atol=0)
    static = {k: torch.full_like(v, float("nan")) for k, v in out.items()}
    buf.gather(idx, out=static)
    for k in out:
        torch.testing.assert_close(static[k], out[k], rtol=0, atol=0)
    assert out["v_in"].shape == (6 + 6 * n, D)


@pytest.mark.parametrize("D,A,n", [(1, 1, 1), (2, 2, 1), (3, 1, 5), (6, 2, 3), (12, 4, 5), (7, 3, 20)])
@pytest.mark.parametrize("shift", [0, 1, 2], ids=["aligned", "off4B", "off8B"])
def test_replay_gather_layouts_over_chunks(D, A, n, shift):
    """The flat chunked gather (launch_gather: one workgroup per chunk of one output, batch rows
    straddling chunk edges) equals torch indexing of the store bit for bit, for every output, at
    batches spanning many chunks, into destinations offset by `shift` floats (the vector width
    falls back to what the pointers allow); the in-kernel draw writes the same indices to idx_out
    as the host-counter draw and gathers exactly those windows."""
    M, B = 911, 2500
    buf = DeviceNstepReplayBuffer(obs_dim=D, act_dim=A, buffer_max_size=M, n_step=n)
    gen = torch.Generator(device="cuda").manual_seed(D * 100 + A * 10 + n)
    for k in KEYS:
        buf.n_step_buf[k].copy_(torch.randn(buf.n_step_buf[k].shape, device="cuda", generator=gen))
    buf.cursor.copy_(torch.tensor([0, M, M, 0]))
    shapes = {"obs": (B, n, D), "act": (B, n, A), "rew": (B, n), "cost": (B, n), "obs2": (B, n, D),
              "done": (B, n), "logp": (B, n), "obs_act": (B, n, D + A), "v_in": (B + B * n, D)}

    def dests():
        out = {}
        for k, shp in shapes.items():
            flat = torch.full((int(np.prod(shp)) + shift,), float("nan"), device="cuda")
            out[k] = flat[shift:].view(shp)
        return out

    def expect(idx):
        ref = {k: buf.n_step_buf[k][idx] for k in KEYS}
        ref["obs_act"] = torch.cat([ref["obs"], ref["act"]], -1)
        ref["v_in"] = torch.cat([ref["obs"][:, 0], ref["obs2"].reshape(-1, D)], 0)
        return ref
    st = N.stream_of(buf.device)
    idx = torch.randint(0, M, (B,), device="cuda", generator=gen)
    out = dests()
    N.check(N.lib().mh_replay_gather_joint(ctypes.byref(buf.ws), n, D, A, N.ptr(idx), B,
                                           *[N.ptr(out[k]) for k in KEYS], N.ptr(out["obs_act"]),
                                           N.ptr(out["v_in"]), st), "gather_joint")
    ref = expect(idx)
    for k in shapes:
        assert torch.equal(out[k], ref[k]), k
    host = torch.empty(B, dtype=torch.int64, device="cuda")
    N.check(N.lib().mh_replay_sample_indices(ctypes.byref(buf.ws), buf.seed, 0, B, N.ptr(host), st), "draw")
    out = dests()
    idx_out = torch.full((B,), -1, dtype=torch.int64, device="cuda")
    N.check(N.lib().mh_replay_draw_gather(ctypes.byref(buf.ws), n, D, A, buf.seed, N.ptr(buf._draw_state), B,
                                          N.ptr(idx_out), *[N.ptr(out[k]) for k in KEYS], N.ptr(out["obs_act"]),
                                          N.ptr(out["v_in"]), st), "draw_gather")
    assert torch.equal(idx_out, host)
    assert buf.draws == 1 and int(buf._draw_state[1].item()) == 0  # advanced once; the ticket reset
    ref = expect(host)
    for k in shapes:
        assert torch.equal(out[k], ref[k]), k
    # indices only (every output null): the grid is the index segment alone
    N.check(N.lib().mh_replay_sample_indices(ctypes.byref(buf.ws), buf.seed, 1, B, N.ptr(host), st), "draw")
    N.check(N.lib().mh_replay_draw_gather(ctypes.byref(buf.ws), n, D, A, buf.seed, N.ptr(buf._draw_state), B,
                                          N.ptr(idx_out), *([None] * 9), st), "draw_only")
    assert torch.equal(idx_out, host) and buf.draws == 2


def test_device_draw_counter_and_one_launch_draw_gather():
    """The replay draw keyed by the buffer's DEVICE counter (mh_replay_sample_indices_dev) equals
    the host-counter entry at the same counters; the one-launch draw + gather
    (mh_replay_draw_gather, sample_batch with out / joint) equals the draw followed by the gather,
    bit for bit; and a captured draw + gather replays as the NEXT draw each time (the counter is
    advanced inside the launch), which is what lets the trainer put it inside the update graph."""
    import ctypes
    import msacl_amd._native as N
    path = os.path.join(G, "nstep_DuctedFan.npz")
    g, buf, total, _ = _run_trace(path)
    B = 300  # > 256: two workgroups share the counter's arrival ticket
    st = N.stream_of(buf.device)

    def host_draw(k):
        ref = torch.empty(B, dtype=torch.int64, device="cuda")
        N.check(N.lib().mh_replay_sample_indices(ctypes.byref(buf.ws), buf.seed, k, B, N.ptr(ref), st), "draw")
        return ref
    for k in range(3):
        got = buf.sample_indices(B)
        assert torch.equal(got, host_draw(k)), k
    assert buf.draws == 3
    ref = buf.gather(host_draw(3), joint=True)
    got = buf.sample_batch(B, joint=True)
    assert set(got) == set(ref)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k
    assert buf.draws == 4
    static = {k: torch.full_like(v, float("nan")) for k, v in got.items()}
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        buf.sample_batch(B, out=static)
    assert buf.draws == 4  # capture runs nothing
    for k in (4, 5):
        graph.replay()
        ref = buf.gather(host_draw(k), joint=True)
        for key in ref:
            assert torch.equal(static[key], ref[key]), (k, key)
        assert buf.draws == k + 1
    del graph


def n_of(g):
    return int(g["n_step"])


N20 = [os.path.join(G, f"nstep_{nm}_n20.npz") for nm in ("QuadTracking", "TwoLink", "DuctedFan")]


@pytest.mark.parametrize("path", N20, ids=os.path.basename)
def test_n20_windows_tiled_to_65536_envs(path):
    """The benchmark's n = 20 windows for configs 3 / 4 envs (QuadTracking, TwoLink, DuctedFan):
    the reference's 16-env _n_step trace tiled 4,096 times = 65,536 envs in lockstep; every
    step's observations and every emitted window (order: per step, env-index order) equal the
    reference's at rtol = atol = 1e-5, compared on the device."""
    g, buf, total, tile = _run_trace(path, tile=4096, check_obs=True)
    assert int(buf.cursor[2]) == total and g["counts"].sum() > 100
    counts = g["counts"]
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    idx = np.concatenate([np.tile(np.arange(o, o + c), tile) for o, c in zip(offs, counts)])
    idx = torch.as_tensor(idx, device="cuda")
    for k in KEYS:
        exp = torch.as_tensor(g["w_" + k], device="cuda")[idx]
        got = buf.n_step_buf[k][:total]
        bad = ((got - exp).abs() > TOL["atol"] + TOL["rtol"] * exp.abs()).sum().item()
        assert bad == 0, (k, bad)
    assert not buf.n_step_buf["done"][:total, :-1].any()


@pytest.mark.parametrize("path", TRACES, ids=os.path.basename)
def test_host_and_device_builds_agree(path):
    """Config 1's CPU build (libmsacl_host.so) and the gfx950 kernels run the same env math: the
    same injected trace through both gives the same windows (VanderPol bit-exact, the others at
    the north-star tolerance, their transcendentals coming from two libms)."""
    from test_host_engine import _cpu_trace
    g, dbuf, total, _ = _run_trace(path)
    _, hbuf = _cpu_trace(path)
    assert hbuf.size == dbuf.size == total
    for k in KEYS:
        d = dbuf.n_step_buf[k][:total].cpu().numpy()
        h = hbuf.n_step_buf[k][:total]
        if "VanderPol" in path:
            np.testing.assert_array_equal(h, d, err_msg=k)
        else:
            np.testing.assert_allclose(h, d, **TOL, err_msg=k)


@pytest.mark.parametrize("deferred", [False, True], ids=["immediate", "deferred"])
def test_single_env_vanderpol_windows(deferred):
    """Config 1's shape on the device (VanderPol, env_num = 1): env 0 of the reference's n = 20
    trace alone through the fused rollout; its windows equal the oracle's replay of the same
    single-env trace (the oracle is bit-exact against the reference's full trace,
    tests/test_oracle_golden.py; envs are independent, so env 0's slice is a valid trace)."""
    from oracle import sampler as OS
    path = os.path.join(G, "nstep_VanderPol_n20.npz")
    full = np.load(path)
    g = {k: full[k] for k in full.files}
    for k in ("init_reset", "init_steps"):
        g[k] = g[k][:1]
    for k in ("actions", "logp", "resets", "obs_trace"):
        g[k] = g[k][:, :1]
    t = {"t": -1}
    venv = OS.VectorEnv("VanderPol", 1, lambda idx: g["init_reset"][idx] if t["t"] < 0 else g["resets"][t["t"]][idx])
    ro = OS.NStepRollout(venv, int(g["n_step"]))
    venv.steps[:] = g["init_steps"]
    wins, counts = [], []
    for k in range(g["actions"].shape[0]):
        t["t"] = k
        w, _ = ro.step(g["actions"][k], g["logp"][k])
        counts.append(len(w))
        wins += w
    g["counts"] = np.array(counts)
    assert len(wins) > 0
    _, buf, total, _ = _run_trace(path, g=g, deferred=deferred)
    assert total == len(wins) and int(buf.cursor[2]) == total
    for j, k in enumerate(KEYS):
        np.testing.assert_array_equal(buf.n_step_buf[k][:total].cpu().numpy(), np.stack([w[j] for w in wins]),
                                      err_msg=k)


def test_single_env_vanderpol_pipeline_trains(tmp_path):
    """Config 1's plumbing on the device: the unchanged pipeline (create_envs -> create_sampler ->
    create_buffer -> create_alg -> trainer) with env_num = 1 trains a few MSACL iterations."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    args = default_msacl_args(env_name="VanderPol", env_num=1, buffer_warm_size=64, buffer_max_size=10000,
                              replay_batch_size=32, max_iteration=4, eval_interval=10 ** 6, save_folder=str(tmp_path),
                              seed=0, num_eval_episode=1)
    _, alg, sampler, buffer, _, trainer = build_pipeline(args)
    assert sampler.device.type == "cuda"
    trainer.train()
    torch.cuda.synchronize()
    assert buffer.size >= 64
    assert all(torch.isfinite(p).all() for p in alg.networks.parameters())
