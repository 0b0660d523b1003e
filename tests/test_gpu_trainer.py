"""GPU end-to-end: the reference's pipeline (create_* -> trainer.train()) on the HIP path,
uniform and prioritized replay, plus the device evaluator."""
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
from msacl_amd.utils.config import build_pipeline, default_msacl_args

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env_name,buffer_name", [("QuadTracking", "nstep_replay_buffer"),
                                                  ("DuctedFan", "prioritized_replay_buffer"),
                                                  ("VanderPol", "nstep_replay_buffer")])
def test_train_loop(tmp_path, env_name, buffer_name):
    args = default_msacl_args(env_name=env_name, env_num=2048, buffer_name=buffer_name, buffer_warm_size=3000,
                              buffer_max_size=200000, max_iteration=5, eval_interval=3, log_save_interval=2,
                              apprfunc_save_interval=4, save_folder=str(tmp_path), seed=0, num_eval_episode=4)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    assert buffer.size >= 3000
    trainer.train()
    torch.cuda.synchronize()
    assert trainer.iteration == 6
    assert os.path.exists(os.path.join(str(tmp_path), "apprfunc", "apprfunc_6.pkl"))
    for p in alg.networks.parameters():
        assert torch.isfinite(p).all()
    b = buffer.sample_batch(64)
    assert not b["done"][:, :-1].any()
    if buffer_name == "prioritized_replay_buffer":
        assert float(buffer.tree[1]) > 0 and "weight" in b
    sd = torch.load(os.path.join(str(tmp_path), "apprfunc", "apprfunc_6.pkl"), weights_only=True)
    assert set(sd) == set(alg.networks.state_dict())


def test_evaluator_runs_episodes(tmp_path):
    args = default_msacl_args(env_name="Pendulum", env_num=64, buffer_warm_size=0, max_iteration=0,
                              save_folder=str(tmp_path), seed=1, num_eval_episode=8)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    m, s, cm, cs = evaluator.run_evaluation(0)
    assert np.isfinite([m, s, cm, cs]).all() and cm >= 0


@pytest.mark.parametrize("alg_name,env_name", [("sac", "TwoLink"), ("lac", "Pendulum")])
def test_off_policy_train_loop(tmp_path, alg_name, env_name):
    """example/{sac,lac}_train.py's pipeline: off_sampler + replay_buffer + off_serial_trainer."""
    from msacl_amd.utils.config import default_lac_args, default_sac_args
    mk = default_sac_args if alg_name == "sac" else default_lac_args
    args = mk(env_name=env_name, env_num=1024, buffer_warm_size=4096, buffer_max_size=100000, max_iteration=6,
              eval_interval=3, log_save_interval=2, apprfunc_save_interval=3, save_folder=str(tmp_path), seed=0,
              num_eval_episode=4)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    assert type(buffer).__name__ == "ReplayBuffer" and type(sampler).__name__ == "OffSampler"
    assert buffer.size >= 4096
    trainer.train()
    torch.cuda.synchronize()
    assert trainer.iteration == 7
    for p in alg.networks.parameters():
        assert torch.isfinite(p).all()
    b = buffer.sample_batch(16)
    assert b["obs"].shape == (16, sampler.envs.obs_dim)


@pytest.mark.parametrize("alg_name", ["ppo", "polyc"])
def test_on_policy_train_loop(tmp_path, alg_name):
    """example/{ppo,polyc}_train.py's pipeline: on_sampler (+ GAE kernel) + on_serial_trainer."""
    from msacl_amd.utils.config import default_ppo_args
    args = default_ppo_args(algorithm=alg_name, env_name="DuctedFan", env_num=512, sample_batch_size=64,
                            num_mini_batch=4, mini_batch_size=16, max_iteration=16, eval_interval=8,
                            log_save_interval=8, apprfunc_save_interval=8, save_folder=str(tmp_path), seed=0,
                            num_eval_episode=4)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    assert buffer is None and type(sampler).__name__ == "OnSampler"
    trainer.train()
    torch.cuda.synchronize()
    assert trainer.global_iteration == 16
    for p in alg.networks.parameters():
        assert torch.isfinite(p).all()
    data, _ = sampler.sample()
    assert data["obs"].shape == (512 * 64, 6) and data["done"].dtype == torch.bool
    assert torch.isfinite(data["adv"]).all() and torch.isfinite(data["ret"]).all()


@pytest.mark.parametrize("name", ["VanderPol", "DuctedFan", "QuadTracking"])
def test_evaluator_matches_reference(tmp_path, name):
    """Parallel and sequential evaluation vs the reference Evaluator (tests/golden/eval_*.npz):
    same policy weights, same initial states. Deterministic mode() actions; the metric equals the
    reference's to 1e-4 relative (GPU vs CPU policy GEMMs differ in the last ulp and the
    reference accumulates in float32, the device in float64)."""
    from msacl_amd.create_pkg.create_evaluator import create_evaluator
    from msacl_amd.create_pkg.create_envs import create_envs
    from msacl_amd.utils.init_args import init_args
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"eval_{name}.npz"))
    E = g["init"].shape[0]
    args = default_msacl_args(env_name=name, env_num=4, save_folder=str(tmp_path), seed=0, num_eval_episode=E,
                              policy_hidden_sizes=[64, 64], value_hidden_sizes=[64, 64], lyapunov_hidden_sizes=[64, 64])
    args = init_args(create_envs(**args), **args)
    ev = create_evaluator(**args)
    ev.networks.policy.load_state_dict({k[7:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("policy/")})
    ev.networks.to(ev.device)
    par = ev.run_parallel_episodes(initial_states=g["init"])
    np.testing.assert_allclose(par, g["parallel"], rtol=1e-4, atol=1e-3)
    args1 = dict(args, is_parallel_eval=False)
    ev1 = create_evaluator(**args1)
    ev1.networks.load_state_dict(ev.networks.state_dict())
    ev1.networks.to(ev1.device)
    seq = ev1.run_n_episodes(3, 0, initial_states=g["seq_init"])
    np.testing.assert_allclose(seq, g["sequential"], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("buffer_name", ["nstep_replay_buffer", "prioritized_replay_buffer"])
def test_overlapped_sampling_equals_serial_order(tmp_path, buffer_name):
    """trainer_overlap_sampling (sampling of k + 1 beside the policy-free update of k on a second
    stream) gives bit-identical networks, window store and sampler state to the serial order.
    rocBLAS may use atomics in split-K GEMMs (run-to-run ulp noise), so both runs use PyTorch's
    deterministic mode, which turns them off."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        _overlap_vs_serial(tmp_path, buffer_name)
    finally:
        torch.use_deterministic_algorithms(prev)


def _overlap_vs_serial(tmp_path, buffer_name):
    def run(overlap, sub):
        torch.manual_seed(0)
        args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_name=buffer_name, buffer_warm_size=3000,
                                  buffer_max_size=60000, max_iteration=7, eval_interval=10 ** 6,
                                  log_save_interval=10 ** 6, apprfunc_save_interval=10 ** 6,
                                  save_folder=str(tmp_path / sub), seed=0, num_eval_episode=1,
                                  trainer_overlap_sampling=overlap)
        args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
        assert trainer.overlap == overlap
        trainer.train()
        torch.cuda.synchronize()
        sd = {k: v.detach().cpu().clone() for k, v in alg.networks.state_dict().items()}
        store = {k: v.cpu().clone() for k, v in buffer.n_step_buf.items()}
        return sd, store, buffer.cursor.cpu().clone(), sampler.obs.cpu().clone()
    a = run(True, "a")
    b = run(False, "b")
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    for k in a[1]:
        assert torch.equal(a[1][k], b[1][k]), k
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])


@pytest.mark.parametrize("buffer_name", ["nstep_replay_buffer", "prioritized_replay_buffer"])
def test_gather_into_update_inputs_equals_copy(tmp_path, monkeypatch, buffer_name):
    """The trainer gathers each replay batch straight into the replayed update graph's static
    inputs (MSACL.replay_inputs -> sample_batch(out=...)): bit-identical networks and buffer to
    gathering into fresh tensors that the update then copies in (deterministic GEMM mode, as
    above)."""
    from msacl_amd.algorithm.msacl import MSACL
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)

    def run(direct, sub):
        torch.manual_seed(0)
        args = default_msacl_args(env_name="DuctedFan", env_num=2048, buffer_name=buffer_name, buffer_warm_size=2000,
                                  buffer_max_size=60000, max_iteration=6, eval_interval=10 ** 6,
                                  log_save_interval=10 ** 6, apprfunc_save_interval=10 ** 6,
                                  save_folder=str(tmp_path / sub), seed=0, num_eval_episode=1)
        args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
        seen = []
        orig = buffer.sample_batch

        def spy(bs, out=None, **kw):
            r = orig(bs, out=out, **kw) if out is not None else orig(bs, **kw)
            seen.append(all(r[k].data_ptr() == alg._static[k].data_ptr() for k in ("obs", "rew"))
                        if alg._static is not None else False)
            return r
        buffer.sample_batch = spy
        if not direct:
            monkeypatch.setattr(MSACL, "replay_inputs", lambda self, b: None)
        trainer.train()
        monkeypatch.undo()
        torch.cuda.synchronize()
        sd = {k: v.detach().cpu().clone() for k, v in alg.networks.state_dict().items()}
        extra = buffer.tree.cpu().clone() if hasattr(buffer, "tree") else None
        return sd, extra, seen

    try:
        a = run(True, "a")
        b = run(False, "b")
    finally:
        torch.use_deterministic_algorithms(prev)
    assert any(a[2]) and not any(b[2])  # the direct path really gathered into the static inputs
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    if a[1] is not None:
        assert torch.equal(a[1], b[1])


@pytest.mark.parametrize("env_name", ["QuadTracking", "DuctedFan"])
def test_graphed_step_equals_separate_graphs(tmp_path, env_name):
    """trainer_graph_step (the iteration's sampling and update replayed as one graph, active with
    an unsynchronised sampler time; the policy pack skipped after a policy-free update) gives
    bit-identical networks, window store, replay cursor, sampler state and logged scalars to the
    sampler graph + update graph pair (deterministic GEMM mode, as above)."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)

    def run(graph_step, sub):
        torch.manual_seed(0)
        args = default_msacl_args(env_name=env_name, env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                                  max_iteration=9, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                                  apprfunc_save_interval=10 ** 6, save_folder=str(tmp_path / sub), seed=0,
                                  num_eval_episode=1, sampler_sync_timing=False, trainer_graph_step=graph_step)
        args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
        used = []
        orig = trainer._graph_step

        def spy():
            r = orig()
            used.append(r is not None)
            return r
        trainer._graph_step = spy
        while trainer.iteration <= trainer.max_iteration:
            trainer.step()
            trainer.iteration += 1
        torch.cuda.synchronize()
        sd = {k: v.detach().cpu().clone() for k, v in alg.networks.state_dict().items()}
        store = {k: v.cpu().clone() for k, v in buffer.n_step_buf.items()}
        ring = alg._tb_ring.cpu().clone() if getattr(alg, "_tb_ring", None) is not None else None  # logged scalars
        # graphs of policy iterations that reuse the packed policy of the policy-free step before
        skipped = any(not k[2] for k in trainer._step_graphs)
        out = (sd, store, buffer.cursor.cpu().clone(), sampler.obs.cpu().clone(), used, ring, skipped)
        trainer.close()
        return out

    try:
        a = run(True, "a")
        b = run(False, "b")
    finally:
        torch.use_deterministic_algorithms(prev)
    assert any(a[4]) and not any(b[4])  # the graphed step really ran (and never in the reference run)
    assert a[6]  # ... and skipped the redundant policy packs
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    for k in a[1]:
        assert torch.equal(a[1][k], b[1][k]), k
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
    assert a[5] is not None and torch.equal(a[5], b[5])


def test_pack_skip_sees_parameter_writes_outside_torch(tmp_path):
    """The graphed step skips the policy pack when the parameters cannot have changed since the
    last one; a write through `.data` (invisible to torch's version counters) followed by
    utils.dist.parameters_written() -- what broadcast_module does -- or by the sampler's
    invalidate_policy_pack() forces the next graphed step to pack again."""
    import msacl_amd.utils.dist as D
    args = default_msacl_args(env_name="QuadTracking", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                              max_iteration=12, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=str(tmp_path), seed=0,
                              num_eval_episode=1, sampler_sync_timing=False, trainer_graph_step=True)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    packs = {}
    orig = sampler.step_graph_parts

    def spy(pack=True):
        packs[trainer.iteration] = pack  # the last call of an iteration decides
        return orig(pack=pack)
    sampler.step_graph_parts = spy
    writes = {8: lambda: D.parameters_written(), 10: lambda: sampler.invalidate_policy_pack()}
    while trainer.iteration <= trainer.max_iteration:
        if trainer.iteration in writes:
            with torch.no_grad():
                for p in alg.networks.policy.parameters():
                    p.data.mul_(0.999)  # through .data: no version bump
            writes[trainer.iteration]()
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()
    trainer.close()
    # even iterations after a policy-free step skip the pack ...
    assert packs.get(6) is False, packs
    # ... unless the parameters were written outside torch's view and the writer said so
    assert packs.get(8) is True and packs.get(10) is True, packs
    assert packs.get(12) is False, packs
