"""CPU: the plugin surface mirrors the reference's registries (names, errors, dims)."""
import numpy as np
import pytest

import msacl_amd  # noqa: F401
from msacl_amd.create_pkg import create_alg, create_buffer, create_envs, create_sampler, create_trainer
from msacl_amd.utils.MyRL_path import underline2camel
from msacl_amd.utils.init_args import init_args


def test_underline2camel():
    assert underline2camel("nstep_off_sampler") == "NstepOffSampler"
    assert underline2camel("hip_nstep_off_sampler") == "HipNstepOffSampler"
    assert underline2camel("msacl_x", first_upper=True) == "MSACLX"


def test_registries_discover_plugins():
    assert {"nstep_off_sampler", "hip_nstep_off_sampler"} <= set(create_sampler.registry.specs)
    assert {"nstep_replay_buffer", "device_nstep_replay_buffer", "prioritized_replay_buffer"} <= set(create_buffer.registry.specs)
    assert "msacl" in create_alg.registry.specs
    assert "nstep_off_serial_trainer" in create_trainer.registry.specs


def test_unknown_ids_raise_keyerror():
    with pytest.raises(KeyError, match="No registered sampler with id"):
        create_sampler.create_sampler(sampler_name="nope")
    with pytest.raises(KeyError, match="No registered buffer with id"):
        create_buffer.create_buffer(buffer_name="nope", trainer="nstep_off_serial_trainer")
    with pytest.raises(KeyError, match="No registered algorithm with id"):
        create_alg.create_alg(algorithm="nope")
    with pytest.raises(RuntimeError):
        create_alg.create_alg(algorithm="msacl", trainer="weird_trainer")


def test_on_policy_trainer_gets_no_buffer():
    assert create_buffer.create_buffer(buffer_name="nstep_replay_buffer", trainer="on_serial_trainer") is None


def test_create_envs_and_init_args_without_gpu(tmp_path):
    envs = create_envs.create_envs(env_name="QuadTracking", env_num=4, env_seed=1)
    assert envs.single_observation_space.shape == (12,)
    args = init_args(envs, trainer="nstep_off_serial_trainer", sample_batch_size=20, save_folder=str(tmp_path),
                     env_name="QuadTracking", algorithm="msacl", lya_eta=0.15, n_step=20, seed=3, enable_cuda=True)
    assert args["obs_dim"] == 12 and args["act_dim"] == 4
    np.testing.assert_allclose(args["action_high_limit"], [4.34 * 9.8 * 2, 10, 10, 10], rtol=1e-6)
    assert (tmp_path / "config.json").exists()
    with pytest.raises(ValueError):
        create_envs.create_envs(env_name="CartPole", env_num=1, env_seed=0)


def test_approx_container_builds_on_cpu():
    """The networks (PyTorch) build through create_apprfunc with the reference's kwargs; the
    state_dict keys equal the reference ApproxContainer's (checkpoint compatibility)."""
    import torch
    from msacl_amd.algorithm.msacl import ApproxContainer
    from msacl_amd.utils.config import default_msacl_args
    a = default_msacl_args(obs_dim=12, act_dim=4, action_type="continu",
                           action_high_limit=np.array([85.064, 10, 10, 10], np.float32),
                           action_low_limit=np.array([0, -10, -10, -10], np.float32))
    net = ApproxContainer(**a)
    obs = torch.randn(5, 12)
    logits = net.policy(obs)
    assert logits.shape == (5, 8) and (logits[:, 4:] > 0).all()
    d = net.create_action_distributions(logits)
    act, lp = d.sample()
    assert act.shape == (5, 4) and lp.shape == (5,)
    assert torch.allclose(d.log_prob(act), lp, atol=1e-2)
    assert net.q1(obs, act).shape == (5,) and net.lyapunov(obs).shape == (5,)
    keys = set(net.state_dict())
    assert {"log_alpha", "policy.act_high_lim", "q1.q.0.weight", "q2_target.q.4.bias", "lyapunov.lya.4.weight",
            "policy.policy.4.weight"} <= keys


def test_hip_vector_env_exposes_the_vector_env_api():
    """The device vector env's gym-like surface (no GPU needed to inspect it)."""
    from msacl_amd.env.hip_vector_env import HipVectorEnv
    for m in ("reset", "step", "get_state", "set_state", "close", "handle"):
        assert callable(getattr(HipVectorEnv, m, None)), m
