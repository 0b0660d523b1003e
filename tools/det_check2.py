"""Per-iteration divergence probe of serial vs overlapped trainer order."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402


def trace(overlap):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                              max_iteration=7, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=overlap)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    out = []
    for it in range(8):
        trainer.step()
        trainer.iteration += 1
        torch.cuda.synchronize()
        pol = torch.cat([p.detach().flatten() for p in alg.networks.policy.parameters()]).double().sum().item()
        q = torch.cat([p.detach().flatten() for p in alg.networks.q1.parameters()]).double().sum().item()
        st = buffer.n_step_buf["obs"].double().sum().item()
        out.append((it, int(buffer.cursor[2]), sampler.obs.double().sum().item(), st, pol, q))
    return out


a, b = trace(False), trace(True)
for x, y in zip(a, b):
    print("serial ", x)
    print("overlap", y, "SAME" if x == y else "DIFF")
