"""Determinism probe: the same seeded training run twice (serial / overlapped) -> which tensors differ."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402


def run(overlap, buffer_name="nstep_replay_buffer", **kw):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_name=buffer_name, buffer_warm_size=3000,
                              buffer_max_size=60000, max_iteration=7, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=overlap, **kw)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    trainer.train()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu().clone() for k, v in alg.networks.state_dict().items()}
    store = {k: v.cpu().clone() for k, v in buffer.n_step_buf.items()}
    return sd, store


def diff(a, b, tag):
    bad = [k for k in a[0] if not torch.equal(a[0][k], b[0][k])]
    bads = [k for k in a[1] if not torch.equal(a[1][k], b[1][k])]
    print(tag, "params differing:", len(bad), bad[:6], "store differing:", bads, flush=True)


for kw in ({}, {"alg_twin_streams": False, "alg_concurrent_streams": False}, {"alg_use_graph": False}):
    s1, s2, o1 = run(False, **kw), run(False, **kw), run(True, **kw)
    diff(s1, s2, f"serial vs serial {kw}")
    diff(s1, o1, f"serial vs overlap {kw}")
