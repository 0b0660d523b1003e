"""Overlap divergence: concurrency or ordering? Variants of the overlapped trainer order."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402


def trace(overlap, mode=None):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                              max_iteration=7, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=overlap)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    orig = sampler.sample
    if mode == "sync_after_sample":
        def s():
            r = orig()
            torch.cuda.synchronize()
            return r
        sampler.sample = s
    if mode == "sync_before_sample":
        def s():
            torch.cuda.synchronize()
            return orig()
        sampler.sample = s
    out = []
    for it in range(5):
        trainer.step()
        trainer.iteration += 1
        trainer.finish_pending() if it == 4 else None
        torch.cuda.synchronize()
        out.append((it, sampler.obs.double().sum().item(),
                    torch.cat([p.detach().flatten() for p in alg.networks.parameters()]).double().sum().item()))
    return out


if len(sys.argv) > 1 and sys.argv[1] == "det":
    torch.use_deterministic_algorithms(True, warn_only=True)  # rocBLAS without atomics
base = trace(False)
for ov, mode in ((False, None), (True, None), (True, "sync_after_sample"), (True, "sync_before_sample")):
    t = trace(ov, mode)
    print(ov, mode, ["SAME" if x == y else "DIFF" for x, y in zip(base, t)], flush=True)
