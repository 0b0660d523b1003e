"""ctypes binding of include/msacl_hip.h (the engine's C ABI) and include/msacl_host.h (its CPU
build, config 1: host_lib()).

The library is built in-tree by `make -C csrc` (or __graft_entry__.build()) into
<repo>/lib/libmsacl_hip.so. There is no CPU fallback anywhere in the product path: if the
library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("MSACL_HIP_LIB", os.path.join(_REPO, "lib", "libmsacl_hip.so"))

ENV_IDS = {
    "VanderPol": 0,
    "Pendulum": 1,
    "DuctedFan": 2,
    "TwoLink": 3,
    "SingleTrackCar": 4,
    "QuadTracking": 5,
}

c_vp = ctypes.c_void_p
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double


class EnvInfo(ctypes.Structure):
    _fields_ = [
        ("obs_dim", c_i32), ("act_dim", c_i32), ("state_dim", c_i32), ("xstate_dim", c_i32),
        ("reset_dim", c_i32), ("control_step", c_i32), ("max_step", c_i32), ("record_floats", c_i32),
        ("obs_low", c_f32 * 16), ("obs_high", c_f32 * 16), ("act_low", c_f32 * 4), ("act_high", c_f32 * 4),
    ]


class AdamTensor(ctypes.Structure):
    """mh_adam_tensor_t (include/msacl_hip.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("step", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class PolyakTensor(ctypes.Structure):
    """mh_polyak_tensor_t (include/msacl_hip.h)."""
    _fields_ = [("target", ctypes.c_void_p), ("source", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class Wgrad(ctypes.Structure):
    """mh_wgrad_t (include/msacl_hip.h)."""
    _fields_ = [("g", ctypes.c_void_p), ("ld_g", ctypes.c_int64), ("x", ctypes.c_void_p), ("ld_x", ctypes.c_int64),
                ("n_out", ctypes.c_int64), ("n_in", ctypes.c_int64), ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p)]


class TrajStore(ctypes.Structure):
    _fields_ = [
        ("obs", c_vp), ("act", c_vp), ("rew", c_vp), ("cost", c_vp), ("obs2", c_vp), ("done", c_vp),
        ("logp", c_vp), ("horizon", c_i32),
    ]


class WindowStore(ctypes.Structure):
    _fields_ = [
        ("obs", c_vp), ("act", c_vp), ("rew", c_vp), ("cost", c_vp), ("obs2", c_vp), ("done", c_vp),
        ("logp", c_vp), ("capacity", c_i64), ("cursor", c_vp),
    ]


# name -> (restype, argtypes)
_PROTOS = {
    "mh_abi_version": (ctypes.c_int, []),
    "mh_last_error": (ctypes.c_char_p, []),
    "mh_env_info": (ctypes.c_int, [c_i32, ctypes.POINTER(EnvInfo)]),
    "mh_env_create": (ctypes.c_int, [c_i32, c_i64, c_u64, ctypes.POINTER(c_vp)]),
    "mh_env_destroy": (ctypes.c_int, [c_vp]),
    "mh_env_reset": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mh_env_step": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_env_get_state": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_env_set_state": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_nstep_attach": (ctypes.c_int, [c_vp, c_i32, c_f32, c_f32]),
    "mh_rollout_step": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(WindowStore), c_vp, c_vp, c_vp]),
    "mh_rollout_step_deferred": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(WindowStore), c_vp, c_vp,
                                                c_vp]),
    "mh_rollout_flush": (ctypes.c_int, [c_vp, c_vp]),
    "mh_nstep_set_log_std_clamp": (ctypes.c_int, [c_vp, c_i32, c_f32, c_f32]),
    "mh_env_set_reward_cost_scale": (ctypes.c_int, [c_vp, c_f32, c_f32]),
    "mh_env_set_action_noise": (ctypes.c_int, [c_vp, c_vp]),
    "mh_rollout_set_trace": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_rollout_set_trace_state": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_capture_unjoined": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int32, c_vp]),
    "mh_nstep_reserve": (ctypes.c_int, [c_vp, c_i32]),
    "mh_sample_horizon_windows": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_sample_horizon_errors": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_sample_horizon_set_spin_limit": (ctypes.c_int, [c_vp, ctypes.c_uint32]),
    "mh_env_get_counters": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_env_set_counters": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_rng_draw": (ctypes.c_int, [c_i32, c_i32, c_u64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "mh_sample_horizon_debug_logits": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mh_sample_horizon": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(WindowStore), c_vp,
                                         c_vp, c_vp, c_vp]),
    "mh_sample_horizon_emit": (ctypes.c_int, [c_vp, c_i32, ctypes.POINTER(WindowStore), c_vp, c_vp]),
    "mh_rollout_traj_step": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(TrajStore), c_i32,
                                            c_vp, c_vp, c_vp]),
    "mh_policy_packed_size": (ctypes.c_int, [c_i32, ctypes.POINTER(c_i64)]),
    "mh_policy_pack": (ctypes.c_int, [c_vp] * 6 + [c_i32] * 4 + [c_vp, c_vp]),
    "mh_policy_forward": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mh_act_grad_chunks": (ctypes.c_int, [c_i64, ctypes.POINTER(c_i32)]),
    "mh_act_grad_colsum": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_policy_head": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_f32, c_vp,
                                      c_vp, c_vp, c_vp]),
    "mh_policy_head_backward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32,
                                               c_f32, c_f32, c_vp, c_vp]),
    "mh_policy_head_sample": (ctypes.c_int, [c_vp] * 5 + [c_i64, c_i32, c_i32, c_f32, c_f32, c_u64] + [c_vp] * 6),
    "mh_dx_narrow": (ctypes.c_int, [c_vp, c_vp, c_i32, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mh_square_sum": (ctypes.c_int, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mh_square_sum_backward": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mh_head_backward_workspace": (ctypes.c_int, [c_i64, c_i32, c_i32, ctypes.POINTER(c_i64)]),
    "mh_head_backward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_linear_backward_plan": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "mh_linear_backward": (ctypes.c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp,
                                          c_vp]),
    "mh_msacl_policy_loss": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_vp, c_vp, c_vp]),
    "mh_msacl_policy_loss_backward": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mh_msacl_ratio0": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "mh_msacl_ratio0_backward": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp]),
    "mh_msacl_policy_objective": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f64, c_f32, c_i32,
                                                 c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_msacl_policy_objective_step": (ctypes.c_int, [c_vp] * 8 + [c_f64, c_f32, c_i32, c_i32] + [c_vp] * 11
                                       + [c_f32, c_vp, c_vp]),
    "mh_msacl_policy_objective_backward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                                                          c_vp, c_vp, c_vp, c_vp]),
    "mh_msacl_policy_combine": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "mh_msacl_alpha_grad": (ctypes.c_int, [c_vp, c_vp, c_f32, c_vp, c_vp]),
    "mh_polyak_multi": (ctypes.c_int, [c_vp, c_i32, ctypes.c_double, c_vp]),
    "mh_adam_multi": (ctypes.c_int, [c_vp, c_i32, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                     c_vp, c_vp]),
    "mh_adam_multi_lr": (ctypes.c_int, [c_vp, c_i32, c_vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_vp,
                                        c_vp]),
    "mh_gemm_workspace": (ctypes.c_int, [c_i64, c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "mh_gemm_f32": (ctypes.c_int, [c_vp] * 4 + [c_i64] * 6 + [c_i32] * 3 + [c_vp, c_vp]),
    "mh_gemm_f32_grouped": (ctypes.c_int, [c_vp] * 4 + [c_i64] * 6 + [c_i32] * 4 + [c_i64] * 4 + [c_vp]),
    "mh_linear_backward_grouped": (ctypes.c_int, [c_vp, c_vp, c_i32, c_vp, c_vp] + [c_i64] * 6 + [c_i32] + [c_i64] * 6
                                   + [c_vp] * 5),
    "mh_head_backward_grouped": (ctypes.c_int, [c_vp] * 3 + [c_i64, c_i32, c_i32, c_i64, c_i64, c_i32] + [c_i64] * 6
                                 + [c_vp] * 5),
    "mh_mlp3_forward": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i64] + [c_vp] * 6 + [c_i32] * 5
                        + [c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mh_mlp3_forward_pair": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_i32, c_i32] + [c_i32] * 3
                             + [c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mh_mlp3_forward_sqsum": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i64, c_vp] + [c_i32] * 5
                              + [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "mh_mlp3_backward_sqsum": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64]
                               + [c_i32] * 5 + [c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mh_mlp3_backward": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64] + [c_i32] * 5
                         + [c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mh_mlp3_set_row_tiles": (ctypes.c_int, [c_i32]),
    "mh_mlp3_backward_w3_workspace": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, ctypes.POINTER(c_i64)]),
    "mh_mlp3_backward_w3": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64] + [c_i32] * 5
                            + [c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "mh_weight_grads_workspace": (ctypes.c_int, [c_vp, c_i32, c_i64, ctypes.POINTER(c_i64)]),
    "mh_weight_grads": (ctypes.c_int, [c_vp, c_i32, c_i64, c_vp, c_vp]),
    "mh_stocha_head": (ctypes.c_int, [c_vp, c_i64, c_i32, c_f32, c_f32, c_vp, c_vp]),
    "mh_stocha_head_backward": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_f32, c_vp, c_vp]),
    "mh_tanh_gauss_rsample": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_i32, c_vp, c_vp, c_vp]),
    "mh_tanh_gauss_rsample_backward": (ctypes.c_int, [c_vp] * 6 + [c_i64, c_i32, c_vp, c_vp]),
    "mh_tanh_gauss_log_prob": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_i32, c_vp, c_vp]),
    "mh_tanh_gauss_log_prob_backward": (ctypes.c_int, [c_vp] * 5 + [c_i64, c_i32, c_vp, c_vp]),
    "mh_gae": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f64, c_f64, c_vp, c_vp, c_vp]),
    "mh_env_set_timing": (ctypes.c_int, [c_vp, c_i32]),
    "mh_env_read_timing": (ctypes.c_int, [c_vp, ctypes.POINTER(c_f64), ctypes.POINTER(c_i64), c_i32]),
    "mh_replay_gather": (ctypes.c_int, [ctypes.POINTER(WindowStore), c_i32, c_i32, c_i32, c_vp, c_i64,
                                        c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mh_replay_gather_joint": (ctypes.c_int, [ctypes.POINTER(WindowStore), c_i32, c_i32, c_i32, c_vp, c_i64]
                               + [c_vp] * 10),
    "mh_replay_sample_indices": (ctypes.c_int, [ctypes.POINTER(WindowStore), c_u64, c_u64, c_i64, c_vp, c_vp]),
    "mh_replay_sample_indices_dev": (ctypes.c_int, [ctypes.POINTER(WindowStore), c_u64, c_vp, c_i64, c_vp, c_vp]),
    "mh_replay_draw_gather": (ctypes.c_int, [ctypes.POINTER(WindowStore), c_i32, c_i32, c_i32, c_u64, c_vp, c_i64]
                              + [c_vp] * 10 + [c_vp]),
    "mh_msacl_q_target": (ctypes.c_int, [c_vp] * 9 + [c_f32, c_i32, c_i32] + [c_vp] * 5 + [c_vp]),
    "mh_msacl_q_target_stats": (ctypes.c_int, [c_vp] * 9 + [c_f32, c_i32, c_i32] + [c_vp] * 6 + [c_vp]),
    "mh_msacl_tb_pack": (ctypes.c_int, [c_vp] * 7 + [c_vp]),
    "mh_msacl_tb_pack_ring": (ctypes.c_int, [c_vp] * 8 + [c_i32, c_vp]),
    "mh_msacl_lyapunov": (ctypes.c_int, [c_vp] * 9 + [c_f32] * 4 + [c_i32] * 3 + [c_vp] * 6 + [c_vp]),
    "mh_msacl_stability_adv": (ctypes.c_int, [c_vp] * 4 + [c_i32, c_i32, c_vp, c_vp, c_vp]),
    "mh_msacl_ppo_clip": (ctypes.c_int, [c_vp, c_vp, c_vp, c_f64, c_f32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mh_per_update": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_f32, c_f32, c_vp, c_vp]),
    "mh_per_set_new": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "mh_per_sample": (ctypes.c_int, [c_vp, c_i64, c_vp, c_u64, c_u64, c_i64, c_f32, c_vp, c_vp, c_vp]),
}

_lib = None


def lib():
    """Load the engine library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"MSACL HIP engine library not found at {LIB_PATH}; build it with "
                f"`make -C {os.path.join(_HERE, 'csrc')}` (or __graft_entry__.build()). "
                "There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        # A/B runs load older builds (MSACL_HIP_LIB plus MSACL_HIP_LIB_AB=1): an entry point they
        # lack is left unbound there (listed on stderr; a call then raises). Every other library,
        # an MSACL_HIP_LIB override included, must export every entry point, checked here at load.
        ab = os.environ.get("MSACL_HIP_LIB_AB", "") == "1"
        missing = [name for name in _PROTOS if not hasattr(L, name)]
        if missing and not ab:
            raise RuntimeError(f"{LIB_PATH} lacks {len(missing)} entry point(s) of include/msacl_hip.h: "
                               f"{', '.join(missing[:8])}{' ...' if len(missing) > 8 else ''} (stale build?)")
        if missing:
            print(f"[msacl] A/B library {LIB_PATH}: {len(missing)} entry point(s) unbound: {', '.join(missing)}",
                  file=sys.stderr)
        for name, (res, args) in _PROTOS.items():
            if name in missing:
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.mh_abi_version() != 1:
            raise RuntimeError("libmsacl_hip ABI version mismatch")
        _lib = L
    return _lib


def exported_symbols():
    return list(_PROTOS)


# ------------------------------------------------------------------ CPU build (config 1)
HOST_LIB_PATH = os.environ.get("MSACL_HOST_LIB", os.path.join(_REPO, "lib", "libmsacl_host.so"))
_HOST_PROTOS = {
    "mhh_abi_version": (ctypes.c_int, []),
    "mhh_last_error": (ctypes.c_char_p, []),
    "mhh_env_info": (ctypes.c_int, [c_i32, ctypes.POINTER(EnvInfo)]),
    "mhh_env_create": (ctypes.c_int, [c_i32, c_i64, c_u64, ctypes.POINTER(c_vp)]),
    "mhh_env_destroy": (ctypes.c_int, [c_vp]),
    "mhh_env_reset": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "mhh_env_step": (ctypes.c_int, [c_vp] * 8),
    "mhh_env_get_state": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mhh_env_set_state": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "mhh_msacl_q_target": (ctypes.c_int, [c_vp] * 9 + [c_f32, c_i32, c_i32] + [c_vp] * 5),
    "mhh_msacl_lyapunov": (ctypes.c_int, [c_vp] * 9 + [c_f32] * 4 + [c_i32] * 3 + [c_vp] * 6),
    "mhh_msacl_stability_adv": (ctypes.c_int, [c_vp] * 4 + [c_i32, c_i32, c_vp, c_vp]),
    "mhh_msacl_ppo_clip": (ctypes.c_int, [c_vp, c_vp, c_vp, c_f64, c_f32, c_i32, c_vp, c_vp, c_vp]),
    "mhh_msacl_policy_loss": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_vp, c_vp]),
    "mhh_msacl_policy_loss_backward": (ctypes.c_int, [c_vp] * 4 + [c_i64, c_vp, c_vp, c_vp]),
    "mhh_msacl_ratio0": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp]),
    "mhh_msacl_ratio0_backward": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp]),
}
_host = None


def host_lib():
    """Load the engine's CPU build (raises if it has not been built). Selected explicitly by
    device="cpu"; the GPU path never falls back to it."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise RuntimeError(f"MSACL host engine library not found at {HOST_LIB_PATH}; build it with "
                               f"`make -C {os.path.join(_HERE, 'csrc')}` (or __graft_entry__.build()).")
        L = ctypes.CDLL(HOST_LIB_PATH)
        for name, (res, args) in _HOST_PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.mhh_abi_version() != 1:
            raise RuntimeError("libmsacl_host ABI version mismatch")
        _host = L
    return _host


def host_env_info(name_or_id):
    eid = ENV_IDS[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)
    info = EnvInfo()
    host_check(host_lib().mhh_env_info(eid, ctypes.byref(info)), "mhh_env_info")
    return info


def host_exported_symbols():
    return list(_HOST_PROTOS)


def host_check(rc, what=""):
    if rc != 0:
        msg = host_lib().mhh_last_error()
        raise RuntimeError(f"{what} failed (code {rc}): {msg.decode() if msg else ''}")


def hptr(t):
    """Host pointer of a contiguous CPU tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        if t.device.type != "cpu" or not t.is_contiguous():
            raise ValueError("the host engine takes contiguous CPU tensors")
        return ctypes.c_void_p(t.data_ptr())
    if not t.flags["C_CONTIGUOUS"]:
        raise ValueError("the host engine takes C-contiguous arrays")
    return ctypes.c_void_p(t.ctypes.data)


def check(rc, what=""):
    if rc != 0:
        msg = lib().mh_last_error()
        raise RuntimeError(f"{what} failed (code {rc}): {msg.decode() if msg else ''}")


def env_info(name_or_id):
    eid = ENV_IDS[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)
    info = EnvInfo()
    check(lib().mh_env_info(eid, ctypes.byref(info)), "mh_env_info")
    return info


# ------------------------------------------------------------------ torch plumbing helpers
def ptr(t):
    """Device pointer of a contiguous tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("tensor passed to the HIP engine must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t, name, dtype=None, numel=None, device=None):
    """Host-side shape/dtype/device checks before any kernel touches `t`."""
    import torch
    if t is None:
        return
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a device tensor (got {t.device})")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name} must have {numel} elements (got {t.numel()})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    _ = torch
