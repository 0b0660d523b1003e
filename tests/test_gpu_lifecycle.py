"""GPU: deterministic release of the pipeline's device resources (captured HIP graphs, env handles,
streams) instead of whenever the garbage collector finalises them.

Background: round 2 saw an abort inside a graph capture when the cyclic collector finalised a
dead pipeline's graphs / events there (HIP calls illegal during a capture). The root fixes:
  * no reference cycles: a dropped MSACL / SAC pipeline is freed by reference counting at the
    `del`, outside any capture (UpdateGraph holds its algorithm's body weakly);
  * explicit close() on trainers, samplers, algorithms and evaluators (idempotent);
  * an env handle released from a finaliser during a capture is destroyed after it, not in it;
  * the collector stays paused while a graph captures (utils/dist.py).
"""
import gc
import weakref

import pytest
import torch

import msacl_amd  # noqa: F401
from msacl_amd.utils.config import build_pipeline, default_msacl_args, default_sac_args

pytestmark = pytest.mark.gpu


def _msacl(tmp, envs=2048, iters=4, warm=2000, **kw):
    args = default_msacl_args(env_name="DuctedFan", env_num=envs, buffer_warm_size=warm, buffer_max_size=60000,
                              max_iteration=iters, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=str(tmp), seed=0, num_eval_episode=1, **kw)
    return build_pipeline(args)


def _train(trainer, iters):
    for _ in range(iters):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()


@pytest.mark.parametrize("kind", ["msacl", "sac"])
def test_dropped_pipeline_is_freed_by_refcount(tmp_path, kind):
    """After training (sampler graph and update graphs captured), deleting the pipeline frees
    every part at once with the cyclic collector OFF: nothing waits for a collection."""
    if kind == "msacl":
        _, alg, sampler, buffer, evaluator, trainer = _msacl(tmp_path)
    else:
        args = default_sac_args(env_name="Pendulum", env_num=2048, buffer_warm_size=4096, max_iteration=4,
                                eval_interval=10 ** 6, log_save_interval=10 ** 6, apprfunc_save_interval=10 ** 6,
                                save_folder=str(tmp_path), seed=0, num_eval_episode=1)
        _, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    _train(trainer, 4)
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        refs = {n: weakref.ref(o) for n, o in (("alg", alg), ("sampler", sampler), ("buffer", buffer),
                                                 ("evaluator", evaluator), ("trainer", trainer),
                                                 ("networks", alg.networks))}
        del alg, sampler, buffer, evaluator, trainer
        alive = [n for n, r in refs.items() if r() is not None]
        assert not alive, f"kept alive by a reference cycle: {alive}"
    finally:
        if was:
            gc.enable()


def test_close_releases_device_resources_and_is_idempotent(tmp_path):
    _, alg, sampler, buffer, evaluator, trainer = _msacl(tmp_path)
    _train(trainer, 4)
    assert sampler._graph is not None and alg._graphs
    trainer.close()
    trainer.close()
    assert sampler._graph is None and sampler.envs._h is None and not alg._graphs and alg._static is None
    assert evaluator.envs._h is None


def _junk_pipeline(tmp):
    """A trained pipeline (graphs captured) left in a reference cycle."""
    _, alg, sampler, buffer, evaluator, trainer = _msacl(tmp, envs=512, iters=3, warm=600)
    _train(trainer, 3)
    trainer.cycle = trainer  # the hazard's shape: only the cyclic collector can free it
    return trainer


def test_gc_of_dead_pipelines_between_captures_and_replays_is_harmless(tmp_path):
    """Pipelines that died in reference cycles (with captured graphs) are collected between
    another pipeline's captures and replays: that pipeline's networks, window store and sampler
    state stay bit-identical to an undisturbed run (deterministic GEMM mode, as in
    test_gpu_trainer.py)."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)

    def run(disturb, sub):
        junk = [_junk_pipeline(tmp_path / f"{sub}_junk{i}") for i in range(3)] if disturb else []
        torch.manual_seed(0)
        _, alg, sampler, buffer, evaluator, trainer = _msacl(tmp_path / sub, iters=6)
        for it in range(6):  # iterations 0-1 eager, 2-3 capture, 4-5 replay (both update branches)
            trainer.step()
            trainer.iteration += 1
            if junk and it >= 1:  # between the eager runs, the captures and the replays
                junk.pop()
                assert gc.collect() > 0
        torch.cuda.synchronize()
        out = ({k: v.detach().cpu().clone() for k, v in alg.networks.state_dict().items()},
               {k: v.cpu().clone() for k, v in buffer.n_step_buf.items()}, buffer.cursor.cpu().clone(),
               sampler.obs.cpu().clone())
        trainer.close()
        return out

    try:
        a = run(False, "a")
        b = run(True, "b")
    finally:
        torch.use_deterministic_algorithms(prev)
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    for k in a[1]:
        assert torch.equal(a[1][k], b[1][k]), k
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])
