"""GPU: the fused f32-MFMA policy forward (csrc/policy_mlp.hip) against the PyTorch StochaPolicy
MLP it replaces in the sampler (RL/apprfunc/mlp.py:111-136): same parameters, same observations,
raw head output (mean | log_std) within float32 summation-order rounding (K = 256 sums:
rtol 1e-5, atol 1e-5 of the output scale)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn as nn

import msacl_amd  # noqa: F401
from msacl_amd.utils.dist import cuda_graph
import msacl_amd._native as N

pytestmark = pytest.mark.gpu


def _mlp(D, A, seed):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(D, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 2 * A),
                         nn.Identity()).cuda()


def _fused(net, obs, D, N3):
    n = ctypes.c_int64()
    N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "size")
    P = torch.empty(n.value, device="cuda")
    ps = [net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight, net[4].bias]
    ps = [p.detach().contiguous() for p in ps]
    N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, N3, N.ptr(P), N.stream_of()), "pack")
    out = torch.empty(obs.shape[0], N3, device="cuda")
    N.check(N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), obs.shape[0], D, N3, N.ptr(out), N.stream_of()), "fwd")
    return out


@pytest.mark.parametrize("D,A,E", [(12, 4, 65536), (12, 4, 1000), (2, 1, 777), (6, 2, 4097), (7, 2, 64), (5, 8, 333),
                                   (16, 16, 96)])  # 2A <= 16: 16x16x1 4-block layer 3; 2A = 32: 32x32x2
def test_fused_policy_forward_matches_torch(D, A, E):
    net = _mlp(D, A, seed=D * 100 + A)
    g = torch.Generator(device="cuda").manual_seed(E)
    obs = (torch.randn(E, D, device="cuda", generator=g) * 2).contiguous()
    with torch.no_grad():
        ref = net(obs).double()
        # float64 reference for the tolerance: both float32 paths sit within a few ulps of it
        net64 = _mlp(D, A, seed=D * 100 + A).double()
        exact = net64(obs.double())
    got = _fused(net, obs, D, 2 * A).double()
    scale = exact.abs().max().item()
    np.testing.assert_allclose(got.cpu().numpy(), exact.cpu().numpy(), rtol=1e-5, atol=1e-5 * scale)
    np.testing.assert_allclose(got.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("obs_scale,w1_scale,w2_scale", [(1e3, 1.0, 1.0), (1e-3, 1.0, 1.0), (1.0, 30.0, 1e-4),
                                                    (1.0, 1e-3, 50.0), (20.0, 20.0, 20.0)])
def test_fused_policy_forward_scaled_operands(obs_scale, w1_scale, w2_scale):
    """The split-f16 layer 2 scales W2 and every env's layer-1 column by powers of two: across
    operand magnitudes far from 1 each logit stays within 2e-6 of the magnitude network
    sum |W3| (sum |W2| |H1| + |b2|) + |b3| (f64) of its float64 value."""
    D, A, E = 12, 4, 4096
    net = _mlp(D, A, seed=7)
    with torch.no_grad():
        net[0].weight.mul_(w1_scale)
        net[0].bias.mul_(w1_scale)
        net[2].weight.mul_(w2_scale)
    g = torch.Generator(device="cuda").manual_seed(3)
    obs = (torch.randn(E, D, device="cuda", generator=g) * obs_scale).contiguous()
    with torch.no_grad():
        n64 = [m.double() if isinstance(m, nn.Linear) else m for m in (net[0], net[2], net[4])]
        x = obs.double()
        h1 = torch.relu(x @ n64[0].weight.T + n64[0].bias)
        h2 = torch.relu(h1 @ n64[1].weight.T + n64[1].bias)
        exact = h2 @ n64[2].weight.T + n64[2].bias
        m2 = h1 @ n64[1].weight.abs().T + n64[1].bias.abs()
        mag = m2 @ n64[2].weight.abs().T + n64[2].bias.abs()
        for m in n64:
            m.float()
    got = _fused(net, obs, D, 2 * A).double()
    err = (got - exact).abs()
    assert torch.isfinite(got).all()
    assert (err <= 2e-6 * mag + 1e-30).all(), (err / mag).max().item()


def test_fused_policy_rejects_unsupported_shapes():
    n = ctypes.c_int64()
    assert N.lib().mh_policy_packed_size(17, ctypes.byref(n)) == -1
    z = torch.zeros(1, device="cuda")
    assert N.lib().mh_policy_pack(*[N.ptr(z)] * 6, 12, 128, 256, 8, N.ptr(z), N.stream_of()) == -1
    assert N.lib().mh_policy_pack(*[N.ptr(z)] * 6, 12, 256, 256, 40, N.ptr(z), N.stream_of()) == -1


def test_sampler_uses_fused_policy_and_matches_torch_path():
    """The n-step sampler picks the fused kernel for the default policy shape; its logits for
    the current observations equal the PyTorch path's."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        args = default_msacl_args(env_name="QuadTracking", env_num=4096, buffer_warm_size=0, max_iteration=0,
                                  save_folder=td, seed=0)
        _, alg, sampler, buffer, _, trainer = build_pipeline(args)
        assert sampler._fused_layers() is not None
        assert sampler._pack_policy()
        fused, raw = sampler._policy_fused()
        torch_logits, raw2 = sampler._policy_raw()
        assert raw and raw2
        np.testing.assert_allclose(fused.detach().cpu().numpy(), torch_logits.detach().cpu().numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("backend", ["auto", "hip", "blas"])
@pytest.mark.parametrize("act", [nn.ReLU, nn.Tanh, nn.Identity])
@pytest.mark.parametrize("rows", [5120 + 37, 256])
def test_fused_linear_act_forward_backward_matches_torch(act, backend, rows):
    """apprfunc/_fused.py LinearAct (GEMM epilogue activation, mh_act_grad_colsum backward) under
    each GEMM backend (mh_gemm_f32 / library / per-shape choice) vs the plain nn.Sequential
    forward/backward: outputs and every gradient (x, W, b) to float32 rounding; frozen parameters
    get no gradient."""
    from msacl_amd.apprfunc._fused import MLP, gemm_backend, set_gemm_backend
    prev = gemm_backend()
    set_gemm_backend(backend)
    try:
        _linear_act_case(MLP, act, rows)
    finally:
        set_gemm_backend(prev)


def _linear_act_case(MLP, act, rows):
    torch.manual_seed(3)
    layers = [nn.Linear(16, 256), act(), nn.Linear(256, 256), act(), nn.Linear(256, 3), nn.Identity()]
    fused = MLP(*layers).cuda()
    plain = nn.Sequential(*[type(m)() if not isinstance(m, nn.Linear) else m for m in layers]).cuda()
    plain.load_state_dict(fused.state_dict())
    x = torch.randn(rows, 16, device="cuda")
    outs, grads = [], []
    for net in (fused, plain):
        xi = x.clone().requires_grad_(True)
        y = net(xi)
        (y * torch.linspace(-1, 1, 3, device="cuda")).pow(2).sum().backward()
        outs.append(y.detach())
        grads.append([xi.grad] + [p.grad.clone() for p in net.parameters()])
        net.zero_grad(set_to_none=True)
    np.testing.assert_allclose(outs[0].cpu().numpy(), outs[1].cpu().numpy(), rtol=1e-5, atol=1e-5)
    for a, b in zip(*grads):
        scale = b.abs().max().item()
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-5 * scale)
    for p in fused[2].parameters():
        p.requires_grad_(False)
    xi = x.clone().requires_grad_(True)
    fused(xi).sum().backward()
    assert fused[2].weight.grad is None and fused[0].weight.grad is not None and xi.grad is not None


@pytest.mark.parametrize("backend", ["hip", "blas"])
def test_fused_mlp_empty_batch(backend):
    """Zero rows: empty outputs, zero weight and bias gradients (the empty sum), as nn.Sequential."""
    from msacl_amd.apprfunc._fused import MLP, gemm_backend, set_gemm_backend
    prev = gemm_backend()
    set_gemm_backend(backend)
    try:
        torch.manual_seed(0)
        net = MLP(nn.Linear(12, 256), nn.ReLU(), nn.Linear(256, 256), nn.Tanh(), nn.Linear(256, 8), nn.Identity()).cuda()
        y = net(torch.zeros(0, 12, device="cuda"))
        assert y.shape == (0, 8)
        y.sum().backward()
        for p in net.parameters():
            assert p.grad is not None and torch.equal(p.grad, torch.zeros_like(p))
    finally:
        set_gemm_backend(prev)


def test_policy_pack_and_forward_replayed_in_a_graph_equal_eager():
    """mh_policy_pack + mh_policy_forward captured in one HIP graph and replayed several times
    (the sampler packs at every sample()): every replay equals the eager result bit for bit,
    including the packed scale slots (they were once zeroed by a memset node that stayed dirty
    from the second replay on)."""
    D, A, E = 12, 4, 8192
    net = _mlp(D, A, seed=3)
    obs = torch.randn(E, D, device="cuda").contiguous()
    ref = _fused(net, obs, D, 2 * A)
    n = ctypes.c_int64()
    N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "size")
    P = torch.full((n.value,), float("nan"), device="cuda")
    out = torch.empty(E, 2 * A, device="cuda")
    ps = [p.detach().contiguous() for p in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                            net[4].bias)]
    g = torch.cuda.CUDAGraph()
    with cuda_graph(g):
        N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, 2 * A, N.ptr(P), N.stream_of()), "pack")
        N.check(N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, 2 * A, N.ptr(out), N.stream_of()), "fwd")
    for _ in range(4):
        P[-64:].fill_(-3.0e38)  # dirty slots between replays must not leak into the scales
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


@pytest.mark.parametrize("warm", [0, 3000])
def test_sampler_graph_replays_equal_eager_sampling(tmp_path, warm):
    """The n-step sampler's captured horizon (graph replays 1..4) and eager sampling from the same
    state give bit-identical observations and window stores."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args

    def pipe(graph, sub):
        torch.manual_seed(0)
        args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=warm, buffer_max_size=200000,
                                  max_iteration=0, eval_interval=10 ** 6, save_folder=str(tmp_path / sub), seed=0,
                                  num_eval_episode=1, sampler_use_graph=graph)
        return build_pipeline(args)
    A, B = pipe(True, "a"), pipe(False, "b")
    for _ in range(4):
        A[3].add_batch(A[2].sample()[0])
        B[3].add_batch(B[2].sample()[0])
        torch.cuda.synchronize()
        assert torch.equal(A[2].obs, B[2].obs)
        assert torch.equal(A[3].cursor, B[3].cursor)
        for k in A[3].n_step_buf:
            assert torch.equal(A[3].n_step_buf[k], B[3].n_step_buf[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("env_name,graph", [("QuadTracking", True), ("DuctedFan", False), ("VanderPol", True)])
def test_deferred_emission_equals_immediate_emission(tmp_path, env_name, graph):
    """mh_rollout_step_deferred (each lockstep's windows copied by the next lockstep's emitter
    waves, the last by mh_rollout_flush) and mh_rollout_step (a separate emission launch per
    step) leave bit-identical window stores, cursors and observations after every horizon;
    VanderPol's long episodes make every env emit every step (the heavy-emission case)."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args

    def pipe(deferred, sub):
        torch.manual_seed(0)
        args = default_msacl_args(env_name=env_name, env_num=4096, buffer_warm_size=0, buffer_max_size=150000,
                                  max_iteration=0, eval_interval=10 ** 6, save_folder=str(tmp_path / sub), seed=0,
                                  num_eval_episode=1, sampler_use_graph=graph, sampler_deferred_emission=deferred)
        return build_pipeline(args)
    A, B = pipe(True, "a"), pipe(False, "b")
    for _ in range(4):
        A[3].add_batch(A[2].sample()[0])
        B[3].add_batch(B[2].sample()[0])
        torch.cuda.synchronize()
        assert torch.equal(A[2].obs, B[2].obs)
        assert torch.equal(A[3].cursor, B[3].cursor)
        for k in A[3].n_step_buf:
            assert torch.equal(A[3].n_step_buf[k], B[3].n_step_buf[k]), k
    assert int(A[3].cursor[2]) > 0


@pytest.mark.gpu
def test_deferred_steps_interleaved_with_immediate_calls():
    """A pending deferred emission is flushed by every other call that steps or resets the
    handle: deferred, immediate and deferred steps, then an env reset, give the same store and
    cursor as immediate steps throughout (C ABI, injected actions)."""
    from msacl_amd.trainer.buffer.device_nstep_replay_buffer import DeviceNstepReplayBuffer
    from msacl_amd.env.hip_vector_env import HipVectorEnv
    E, n, name = 1000, 4, "TwoLink"
    dev = torch.device("cuda", 0)
    runs = []
    for mode in ("mixed", "immediate"):
        env = HipVectorEnv(name, E, seed=3)
        obs = env.reset()[0].contiguous()
        N.check(N.lib().mh_nstep_attach(env.handle(), n, 1.0, 1.0), "attach")
        buf = DeviceNstepReplayBuffer(obs_dim=env.obs_dim, act_dim=env.act_dim, buffer_max_size=5000, n_step=n,
                                      device=dev)
        g = torch.Generator(device="cpu").manual_seed(0)
        st = N.stream_of(dev)
        for t in range(13):
            act = (torch.rand(E, env.act_dim, generator=g) * 2 - 1).to(dev).contiguous()
            lp = torch.randn(E, generator=g).to(dev).contiguous()
            deferred = mode == "mixed" and t not in (5, 6)
            fn = N.lib().mh_rollout_step_deferred if deferred else N.lib().mh_rollout_step
            N.check(fn(env.handle(), None, N.ptr(act), N.ptr(lp), None, N.ptr(obs), ctypes.byref(buf.ws), None, None,
                       st), "step")
            if t == 9:
                N.check(N.lib().mh_env_reset(env.handle(), None, N.ptr(obs), st), "reset")
        N.check(N.lib().mh_rollout_flush(env.handle(), st), "flush")
        torch.cuda.synchronize()
        runs.append((obs.clone(), buf.cursor.clone(), {k: v.clone() for k, v in buf.n_step_buf.items()}))
    (oa, ca, sa), (ob, cb, sb) = runs
    assert torch.equal(oa, ob) and torch.equal(ca, cb)
    assert int(ca[2]) > 0
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
