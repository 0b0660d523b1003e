"""Device time of the fused horizon kernel (k_sample_fused<Env>, mh_sample_horizon without emission)
at the bench configuration, for the library MSACL_HIP_LIB points at (tools/fused_variants.sh).
Prints one JSON line: {"lib", "env", "envs", "us_per_horizon", "us_per_lockstep"}.
Usage (GPU box): python tools/fused_ab.py [--env QuadTracking] [--envs 65536] [--reps 5]"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--env", default="QuadTracking")
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import torch
    import msacl_amd  # noqa: F401
    import msacl_amd._native as N
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    from tools.gputime import time_launches
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    cfg = default_msacl_args(env_name=a.env, env_num=a.envs, env_seed=1, seed=0, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=0,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), num_eval_episode=1,
                             sampler_sync_timing=False, device=dev)
    _args, _alg, sampler, buffer, _ev, _tr = build_pipeline(cfg)
    for _ in range(3):
        buffer.add_batch(sampler.sample()[0])
    torch.cuda.synchronize()
    h, st, H = sampler.envs.handle(), N.stream_of(dev), sampler.horizon
    noise = N.ptr(sampler._noise) if sampler._noise is not None else None

    def k_fused():
        N.lib().mh_sample_horizon(h, N.ptr(sampler._packed), sampler.envs.obs_dim, 2 * sampler.envs.act_dim,
                                  N.ptr(sampler.obs), H, None, noise, None, None, st)

    ts = [time_launches(k_fused, a.reps) * 1e3 for _ in range(a.rounds)]
    err = torch.zeros(4, dtype=torch.int64, device=dev)
    N.lib().mh_sample_horizon_errors(h, N.ptr(err), st)
    torch.cuda.synchronize()
    t = min(ts)
    print(json.dumps({"lib": os.environ.get("MSACL_HIP_LIB", "build"), "env": a.env, "envs": a.envs,
                      "us_per_horizon": round(t, 2), "us_per_lockstep": round(t / H, 3),
                      "all_us": [round(x, 2) for x in ts], "err_words": err.tolist()}), flush=True)


if __name__ == "__main__":
    main()
