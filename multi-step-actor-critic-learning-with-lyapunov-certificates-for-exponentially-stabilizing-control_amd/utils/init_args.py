"""init_args (RL/utils/init_args.py:11-76): derive dims/limits from the env spaces, pick the
device, seed everything, create the save folder and dump config.json."""
import copy
import datetime
import json
import os
import warnings

import numpy as np
import torch

from .common_utils import change_type, seed_everything


def init_args(envs, **args):
    threads = args.get("num_threads_main")
    if threads is None:
        threads = 4 if "serial" in args["trainer"] else 1
    torch.set_num_threads(threads)

    dev = args.get("device")
    cpu_build = dev is not None and torch.device(dev).type == "cpu"  # config 1: the engine's CPU build
    if args.get("enable_cuda", True) and torch.cuda.is_available() and not cpu_build:
        args["use_gpu"] = True
        # GEMM library behind the PyTorch MLPs of the update: rocBLAS measured 6 % faster than
        # hipBLASLt on the MSACL update shapes (the weight-gradient GEMMs, K = B * n = 5,120 with a
        # 256 x 256 output, get split-K kernels). "hipblaslt" / None keep PyTorch's choice.
        blas = args.get("blas_backend", "rocblas")
        if blas in ("rocblas", "hipblaslt"):
            torch.backends.cuda.preferred_blas_library("cublas" if blas == "rocblas" else "cublaslt")
        # the MLP layers' GEMMs: "auto" = mh_gemm_f32 (csrc/gemm.hip) on the shapes where it beats
        # the library above, "hip" / "blas" = one of the two everywhere
        from ..apprfunc._fused import set_gemm_backend
        set_gemm_backend(args.get("update_gemm", "auto"))
    else:
        if args.get("enable_cuda", True) and not cpu_build:
            warnings.warn("HIP device is not available, use CPU instead")
        args["use_gpu"] = False
    args["batch_size_per_sampler"] = args["sample_batch_size"]

    obs_shape = envs.single_observation_space.shape
    args["obs_dim"] = obs_shape[0] if len(obs_shape) == 1 else obs_shape
    act_shape = envs.single_action_space.shape
    args["action_type"] = "continu"
    args["act_dim"] = act_shape[0] if len(act_shape) == 1 else act_shape
    args["action_high_limit"] = np.asarray(envs.single_action_space.high, np.float32)
    args["action_low_limit"] = np.asarray(envs.single_action_space.low, np.float32)

    if args.get("save_folder") is None:
        stamp = datetime.datetime.now().strftime("%y%m%d-%H%M%S")
        base = os.path.join(os.getcwd(), "results", args["env_name"])
        if args["algorithm"] == "msacl":
            args["save_folder"] = os.path.join(base, "n_step_results",
                                               f"msacl_{stamp}_{args['lya_eta']}_n={args['n_step']}")
        else:
            args["save_folder"] = os.path.join(base, f"{args['algorithm']}_{stamp}")
    os.makedirs(os.path.join(args["save_folder"], "apprfunc"), exist_ok=True)

    args["seed"] = seed_everything(args.get("seed", None))
    print("Set the global seed: {}".format(args["seed"]))
    with open(os.path.join(args["save_folder"], "config.json"), "w", encoding="utf-8") as f:
        json.dump(change_type(copy.deepcopy({k: v for k, v in args.items() if k != "device"})), f,
                  ensure_ascii=False, indent=4)
    return args
