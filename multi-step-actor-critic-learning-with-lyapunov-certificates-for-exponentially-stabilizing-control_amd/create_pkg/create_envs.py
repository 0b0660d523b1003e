"""create_envs (RL/create_pkg/create_envs.py:9-35): returns the device lockstep vector env
(the engine's CPU build for an explicit device="cpu", BASELINE.json config 1)."""
from ..env.host_vector_env import make_vector_env


def create_envs(**args):
    env_id = args.get("env_name")
    return make_vector_env(env_id, int(args.get("env_num") or 1), seed=int(args.get("env_seed") or 0),
                           device=args.get("device"))
