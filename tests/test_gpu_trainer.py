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
