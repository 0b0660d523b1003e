"""Two identical pipelines alive together: sampler graph replays, interleaved or not."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402


def pipe(graph=True):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                              max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=False, sampler_use_graph=graph)
    return build_pipeline(args)


def cmp(tag, A, B):
    sa, ba, sb, bb = A[2], A[3], B[2], B[3]
    print(tag, "obs", torch.equal(sa.obs, sb.obs),
          "store", all(torch.equal(ba.n_step_buf[x], bb.n_step_buf[x]) for x in ba.n_step_buf), flush=True)


mode = sys.argv[1]
if mode == "seq":
    A = pipe()
    for _ in range(3):
        A[3].add_batch(A[2].sample()[0])
    torch.cuda.synchronize()
    B = pipe()
    for _ in range(3):
        B[3].add_batch(B[2].sample()[0])
    torch.cuda.synchronize()
    cmp("seq (A done before B built)", A, B)
elif mode == "both":
    A, B = pipe(), pipe()
    cmp("after build", A, B)
    for _ in range(3):
        A[3].add_batch(A[2].sample()[0])
    for _ in range(3):
        B[3].add_batch(B[2].sample()[0])
    torch.cuda.synchronize()
    cmp("both alive, not interleaved", A, B)
elif mode == "ge":
    A, B = pipe(True), pipe(False)
    cmp("after build g/e", A, B)
    for _ in range(3):
        A[3].add_batch(A[2].sample()[0])
        B[3].add_batch(B[2].sample()[0])
    torch.cuda.synchronize()
    cmp("graph vs eager", A, B)
