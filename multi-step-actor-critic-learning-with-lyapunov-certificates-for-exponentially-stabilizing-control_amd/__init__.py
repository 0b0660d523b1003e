"""MI355X-native MSACL rollout + update engine.

Hand-written gfx950 HIP kernels (csrc/) for the six MSACL control environments, the n-step
window assembly and the MSACL target/certificate math, behind the reference's plugin surface
(create_envs / create_alg / create_sampler / create_buffer / create_evaluator / create_trainer).
The actor / critic / Lyapunov MLPs stay PyTorch-ROCm modules.
Import as `msacl_amd` (see /msacl_amd.py at the repository root).
"""
__version__ = "0.1.0"

PACKAGE_NAME = __name__
