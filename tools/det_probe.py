"""Which part is timing-dependent: the MSACL update or the sampler? Same inputs, perturbed timing."""
import copy
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=60000,
                          max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                          apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0, num_eval_episode=1,
                          **dict(a.split("=") for a in sys.argv[1:]))
for k in ("alg_twin_streams", "alg_concurrent_streams", "alg_use_graph"):
    if k in args:
        args[k] = args[k] == "1"
args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
torch.manual_seed(5)
batch = buffer.sample_batch(256)
batch = {k: v.clone() for k, v in batch.items()}
sd0 = copy.deepcopy(alg.networks.state_dict())
opt0 = [copy.deepcopy(o.state_dict()) for o in (alg.networks.q1_optimizer, alg.networks.q2_optimizer,
                                                  alg.networks.lyapunov_optimizer, alg.networks.policy_optimizer,
                                                  alg.networks.alpha_optimizer)]
side = torch.cuda.Stream()


def run(perturb):
    alg.networks.load_state_dict(sd0)
    for o, s in zip((alg.networks.q1_optimizer, alg.networks.q2_optimizer, alg.networks.lyapunov_optimizer,
                     alg.networks.policy_optimizer, alg.networks.alpha_optimizer), opt0):
        o.load_state_dict(s)
    torch.manual_seed(11)
    for it in range(4):
        if perturb:
            with torch.cuda.stream(side):
                torch.cuda._sleep(int(perturb * (it + 1)))
                x = torch.randn(2048, 2048, device="cuda", generator=torch.Generator("cuda").manual_seed(it))
                for _ in range(3):
                    x = x @ x * 1e-3
        alg.model_update(batch, 100 + it)
    torch.cuda.synchronize()
    return {k: v.detach().clone() for k, v in alg.networks.state_dict().items()}


ref = run(0)
for p in (0, 1000, 50000, 0, 200000):
    got = run(p)
    bad = [k for k in ref if not torch.equal(ref[k], got[k])]
    print("update perturb", p, "differing:", len(bad), bad[:5], flush=True)
