"""create_envs (RL/create_pkg/create_envs.py:9-35): returns the device lockstep vector env."""
from ..env.hip_vector_env import HipVectorEnv


def create_envs(**args):
    env_id = args.get("env_name")
    envs = HipVectorEnv(env_id, int(args.get("env_num") or 1), seed=int(args.get("env_seed") or 0),
                        device=args.get("device"))
    return envs
