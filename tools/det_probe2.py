"""Timing sensitivity of the sampler and of the update, separately (deterministic GEMM mode)."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

torch.use_deterministic_algorithms(True, warn_only=True)


PERT = int(sys.argv[1]) if len(sys.argv) > 1 else 1
GRAPH = (sys.argv[2] != "0") if len(sys.argv) > 2 else True


def pipe():
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                              max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=False,
                              sampler_use_graph=GRAPH)
    return build_pipeline(args)


side = torch.cuda.Stream()


def perturb(n):
    with torch.cuda.stream(side):
        x = torch.ones(4096, 4096, device="cuda")
        for _ in range(n):
            x = torch.tanh(x @ x * 1e-4)


A, B = pipe(), pipe()
_, _, sa, ba, _, ta = A
_, algb, sb, bb, _, tb = B
alga = A[1]
for k in range(4):
    da, _ = sa.sample()
    ba.add_batch(da)
    if PERT:
        perturb(2 + k)
    db, _ = sb.sample()
    bb.add_batch(db)
    torch.cuda.synchronize()
    same_obs = torch.equal(sa.obs, sb.obs)
    same_store = all(torch.equal(ba.n_step_buf[x], bb.n_step_buf[x]) for x in ba.n_step_buf)
    print("sample", k, "obs", same_obs, "store", same_store, "cursor", ba.cursor.tolist(), bb.cursor.tolist(), flush=True)
# update on identical batches
batch = ba.sample_batch(256)
batch = {x: v.clone() for x, v in batch.items()}
for k in range(4):
    torch.manual_seed(100 + k)
    alga.model_update(batch, k)
    torch.cuda.synchronize()
    torch.manual_seed(100 + k)
    perturb(3)
    algb.model_update(batch, k)
    torch.cuda.synchronize()
    sda, sdb = alga.networks.state_dict(), algb.networks.state_dict()
    bad = [x for x in sda if not torch.equal(sda[x], sdb[x])]
    print("update", k, "differing", len(bad), bad[:4], flush=True)
