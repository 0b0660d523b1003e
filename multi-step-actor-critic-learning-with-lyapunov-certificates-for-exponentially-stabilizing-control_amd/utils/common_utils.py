"""Seeding, apprfunc config assembly, activations, device context (RL/utils/common_utils.py)."""
import random
import sys
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from .act_distribution_cls import DiracDistribution, GaussDistribution, TanhGaussDistribution  # noqa: F401

_DISTS = {"TanhGaussDistribution": TanhGaussDistribution, "GaussDistribution": GaussDistribution,
          "DiracDistribution": DiracDistribution}


def seed_everything(seed: Optional[int] = None) -> int:
    """Seed python, numpy and torch (all devices); draws a uint32 seed when None (:12-27)."""
    if seed is None:
        seed = random.randint(0, np.iinfo(np.uint32).max)
    seed = int(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


def change_type(obj):
    """NumPy scalars/arrays -> JSON-able Python values (the reference's version touches
    np.float_, removed in NumPy 2; this one does not)."""
    if isinstance(obj, np.integer):
        return int(obj)
    if isinstance(obj, type):
        return str(obj)
    if isinstance(obj, np.floating):
        return float(obj)
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: change_type(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [change_type(o) for o in obj]
    if isinstance(obj, torch.device):
        return str(obj)
    return obj


def get_apprfunc_dict(key: str, **kwargs):
    """Constructor kwargs for the `key` ("value" / "lyapunov" / "policy") network (:66-114)."""
    var = {
        "apprfunc": kwargs[key + "_func_type"],
        "name": kwargs[key + "_func_name"],
        "obs_dim": kwargs["obs_dim"],
        "min_log_std": kwargs.get(key + "_min_log_std", float("-20")),
        "max_log_std": kwargs.get(key + "_max_log_std", float("1.0")),
    }
    if key == "lyapunov":
        var["input_dim"] = 1 if kwargs[key + "_single_input_dim"] else kwargs["obs_dim"]
        var["output_dim"] = kwargs[key + "_output_dim"]
    if kwargs[key + "_func_type"] != "MLP":
        raise NotImplementedError(kwargs[key + "_func_type"])
    var["hidden_sizes"] = kwargs[key + "_hidden_sizes"]
    var["hidden_activation"] = kwargs[key + "_hidden_activation"]
    var["output_activation"] = kwargs.get(key + "_output_activation", "linear")
    if kwargs["action_type"] != "continu":
        raise NotImplementedError("Only continuous action space is supported")
    var["act_dim"] = kwargs["act_dim"]
    var["act_high_lim"] = np.array(kwargs["action_high_limit"])
    var["act_low_lim"] = np.array(kwargs["action_low_limit"])
    choice = kwargs["policy_act_distribution"]
    if choice == "default":
        var["action_distribution_cls"] = {"StochaPolicy": GaussDistribution,
                                          "DetermPolicy": DiracDistribution}.get(kwargs["policy_func_name"])
    else:
        var["action_distribution_cls"] = _DISTS.get(choice) or getattr(sys.modules[__name__], choice)
    return var


_ACTS = {"relu": nn.ReLU, "elu": nn.ELU, "gelu": nn.GELU, "selu": nn.SELU, "sigmoid": nn.Sigmoid,
         "tanh": nn.Tanh, "linear": nn.Identity}


def get_activation_func(key: str):
    assert isinstance(key, str)
    if key not in _ACTS:
        print("Can not identify activation name:" + key)
        raise RuntimeError
    return _ACTS[key]


class ModuleOnDevice:
    """Temporarily move a module to `device` (restored on exit) — the reference trainer wraps
    sampling in it (nstep_off_serial_trainer.py:78); the device sampler asks for its own device."""

    def __init__(self, module, device):
        self.module = module
        self.prev_device = next(module.parameters()).device.type
        self.new_device = torch.device(device).type
        self.different_device = self.prev_device != self.new_device

    def __enter__(self):
        if self.different_device:
            self.module.to(self.new_device)

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self.different_device:
            self.module.to(self.prev_device)
