"""Graph (A) vs eager (B) sampler, horizon 1: first diverging lockstep and what diverges."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 1
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 0
CAP = int(sys.argv[3]) if len(sys.argv) > 3 else 600000


def pipe(graph):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=WARM, buffer_max_size=CAP,
                              max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=False, sampler_use_graph=graph,
                              sample_batch_size=H)
    return build_pipeline(args)


A, B = pipe(True), pipe(False)
sa, ba, sb, bb = A[2], A[3], B[2], B[3]
for t in range(8):
    ba.add_batch(sa.sample()[0])
    bb.add_batch(sb.sample()[0])
    torch.cuda.synchronize()
    st_a, x_a, k_a = sa.envs.get_state()
    st_b, x_b, k_b = sb.envs.get_state()
    eq = dict(obs=torch.equal(sa.obs, sb.obs), state=torch.equal(st_a, st_b), steps=torch.equal(k_a, k_b),
              store=all(torch.equal(ba.n_step_buf[x], bb.n_step_buf[x]) for x in ba.n_step_buf),
              cursor=torch.equal(ba.cursor, bb.cursor))
    print(t, eq, flush=True)
    if not all(eq.values()):
        d = (sa.obs != sb.obs).any(1).nonzero().flatten()
        print("envs differing:", d.numel(), d[:10].tolist())
        if d.numel():
            i = d[0].item()
            print("A obs", sa.obs[i].tolist(), "\nB obs", sb.obs[i].tolist(), "steps", k_a[i].item(), k_b[i].item())
        break
