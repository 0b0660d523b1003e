"""Default MSACL configuration = the argparse defaults of example/msacl_train.py:24-170, plus the
device-engine keys (env_num is per GPU; device/buffer names select the HIP path)."""


def default_msacl_args(**overrides):
    a = dict(
        env_name="QuadTracking", algorithm="msacl", enable_cuda=True,
        env_num=4, env_seed=1, capture_vedio=False, is_adversary=False, is_render=False, target_value=0.0,
        reward_scale=100.0, cost_scale=100.0,
        value_func_name="ActionValue", value_func_type="MLP", value_hidden_sizes=[256, 256],
        value_hidden_activation="relu", value_output_activation="linear",
        lyapunov_func_name="LyapunovValue", lyapunov_func_type="MLP", lyapunov_hidden_sizes=[256, 256],
        lyapunov_hidden_activation="tanh", lyapunov_output_dim=256, lyapunov_output_activation="linear",
        lyapunov_single_input_dim=False,
        policy_func_name="StochaPolicy", policy_func_type="MLP", policy_act_distribution="TanhGaussDistribution",
        policy_hidden_sizes=[256, 256], policy_hidden_activation="relu", policy_min_log_std=-20, policy_max_log_std=1,
        q_learning_rate=1e-3, lyapunov_learning_rate=1e-3, policy_learning_rate=3e-4, alpha_learning_rate=1e-3,
        lya_diff_scale=10.0, lya_zero_scale=1.0, lya_positive_scale=1.0, gamma=0.99, retrace_lambda=0.95, tau=0.005,
        disable_auto_alpha=False, alpha=1.0, set_alpha_bound=False, alpha_bound=2.0, n_step=20, policy_frequency=2,
        target_network_frequency=1, anneal_lr=False, alpha1=1, alpha2=2, lya_eta=0.15, clip_coef=0.1,
        trainer="nstep_off_serial_trainer", max_iteration=1000000, ini_network_dir=None,
        sampler_name="nstep_off_sampler", sample_interval=1, sample_batch_size=20, noise_params=None,
        buffer_name="nstep_replay_buffer", buffer_warm_size=int(5e3), buffer_max_size=int(1e6), replay_batch_size=256,
        eval_env_seed=2, is_parallel_eval=True, evaluator_name="evaluator", num_eval_episode=5, eval_interval=1000,
        eval_save=False, save_folder=None, apprfunc_save_interval=50000, log_save_interval=50000,
    )
    a.update(overrides)
    return a


_COMMON = dict(
    enable_cuda=True, env_seed=1, capture_vedio=False, is_adversary=False, is_render=False, target_value=0.0,
    reward_scale=100.0, cost_scale=100.0, value_func_type="MLP", value_hidden_sizes=[256, 256],
    value_hidden_activation="relu", value_output_activation="linear", policy_func_name="StochaPolicy",
    policy_func_type="MLP", policy_act_distribution="TanhGaussDistribution", policy_hidden_sizes=[256, 256],
    policy_hidden_activation="relu", policy_min_log_std=-20, policy_max_log_std=1, ini_network_dir=None,
    sample_interval=1, noise_params=None, eval_env_seed=2, is_parallel_eval=True, evaluator_name="evaluator",
    num_eval_episode=5, eval_interval=1000, eval_save=False, save_folder=None, apprfunc_save_interval=50000,
    log_save_interval=50000, max_iteration=1000000,
)


def default_sac_args(**overrides):
    """argparse defaults of example/sac_train.py."""
    a = dict(_COMMON)
    a.update(env_name="TwoLink", algorithm="sac", env_num=4, value_func_name="ActionValue", q_learning_rate=1e-3,
             policy_learning_rate=3e-4, alpha_learning_rate=1e-3, gamma=0.99, tau=0.005, alpha=1.0, auto_alpha=True,
             bound=True, policy_frequency=2, target_network_frequency=1, trainer="off_serial_trainer",
             sampler_name="off_sampler", sample_batch_size=20, buffer_name="replay_buffer", buffer_warm_size=int(5e3),
             buffer_max_size=int(1e6), replay_batch_size=256)
    a.update(overrides)
    return a


def default_lac_args(**overrides):
    """argparse defaults of example/lac_train.py."""
    a = dict(_COMMON)
    a.update(env_name="Pendulum", algorithm="lac", env_num=4, value_func_name="ActionValue", l_learning_rate=1e-3,
             policy_learning_rate=3e-4, alpha_learning_rate=1e-3, beta_learning_rate=1e-3, gamma=0.99, tau=0.005,
             alpha=1.0, beta=1.0, auto_alpha=True, bound=True, alpha3=0.01, policy_frequency=2,
             target_network_frequency=1, trainer="off_serial_trainer", sampler_name="off_sampler", sample_batch_size=20,
             buffer_name="replay_buffer", buffer_warm_size=int(5e3), buffer_max_size=int(1e6), replay_batch_size=256)
    a.update(overrides)
    return a


def default_ppo_args(**overrides):
    """argparse defaults of example/ppo_train.py (algorithm="polyc" gives polyc_train.py's)."""
    a = dict(_COMMON)
    a.update(env_name="Pendulum", algorithm="ppo", env_num=1, value_func_name="StateValue",
             lyapunov_func_name="LyapunovValue", lyapunov_func_type="MLP", lyapunov_hidden_sizes=[256, 256],
             lyapunov_hidden_activation="tanh", lyapunov_output_dim=256, lyapunov_output_activation="linear",
             lyapunov_single_input_dim=False, learning_rate=1e-3, policy_learning_rate=3e-4, loss_coefficient_value=1.0,
             loss_coefficient_entropy=0.01, loss_coefficient_kl=0.0, loss_value_clip=False, value_clip=10,
             lya_diff_sacle=1.0, lya_zero_sacle=10.0, lya_positive_scale=1.0, beta=0.01, gamma=0.99, gae_lambda=0.95,
             tau=0.005, schedule_adam="None", schedule_clip="None", clip=0.1, trainer="on_serial_trainer",
             num_repeat=2, num_mini_batch=25, mini_batch_size=64, num_epoch=50, sampler_name="on_sampler",
             sample_batch_size=1600, buffer_name="replay_buffer", buffer_warm_size=1000, buffer_max_size=50000)
    a.update(overrides)
    if a["algorithm"] == "polyc" and "buffer_max_size" not in overrides:
        a["buffer_max_size"] = 100000
    return a


def build_pipeline(args):
    """create_envs -> init_args -> create_alg/sampler/buffer/evaluator/trainer, exactly the
    sequence of example/msacl_train.py:175-193."""
    from ..create_pkg.create_alg import create_alg
    from ..create_pkg.create_buffer import create_buffer
    from ..create_pkg.create_envs import create_envs
    from ..create_pkg.create_evaluator import create_evaluator
    from ..create_pkg.create_sampler import create_sampler
    from ..create_pkg.create_trainer import create_trainer
    from .init_args import init_args
    envs = create_envs(**args)
    args = init_args(envs, **args)
    alg = create_alg(**args)
    sampler = create_sampler(**args)
    buffer = create_buffer(**args)
    evaluator = create_evaluator(**args)
    trainer = create_trainer(alg, sampler, buffer, evaluator, **args)
    return args, alg, sampler, buffer, evaluator, trainer
