"""Sampler divergence: packed params, logits, rollout step."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402

torch.use_deterministic_algorithms(True, warn_only=True)


def pipe(warm):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=warm, buffer_max_size=60000,
                              max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=False)
    return build_pipeline(args)


A, B = pipe(0), pipe(0)
sa, sb = A[2], B[2]
pa = [p.detach() for p in sa.networks.policy.parameters()]
pb = [p.detach() for p in sb.networks.policy.parameters()]
print("params equal", all(torch.equal(x, y) for x, y in zip(pa, pb)))
print("obs equal at start", torch.equal(sa.obs, sb.obs))
with torch.no_grad():
    sa._pack_policy()
    sb._pack_policy()
    torch.cuda.synchronize()
    print("packed equal", torch.equal(sa._packed, sb._packed), sa._packed.numel())
    if not torch.equal(sa._packed, sb._packed):
        d = (sa._packed != sb._packed).nonzero().flatten()
        print("first differing packed index", d[:10].tolist(), d.numel())
    la, _ = sa._policy_fused()
    lb, _ = sb._policy_fused()
    torch.cuda.synchronize()
    print("logits equal", torch.equal(la, lb))
    for rep in range(5):
        l2, _ = sa._policy_fused()
        torch.cuda.synchronize()
        print("logits repeat equal", rep, torch.equal(la, l2))

# rollout + emission with identical logits, B perturbed by concurrent work
import ctypes  # noqa: E402

import msacl_amd._native as N  # noqa: E402

side = torch.cuda.Stream()
ba, bb = A[3], B[3]
sa.bind_store(ba)
sb.bind_store(bb)
for t in range(6):
    with torch.no_grad():
        la, _ = sa._policy_fused()
    lb = la.clone()
    N.check(N.lib().mh_nstep_set_log_std_clamp(sa._h, 0, -20.0, 1.0), "c")
    N.check(N.lib().mh_nstep_set_log_std_clamp(sb._h, 0, -20.0, 1.0), "c")
    sa._lockstep(ba, logits=la)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        x = torch.ones(4096, 4096, device="cuda")
        for _ in range(3):
            x = torch.tanh(x @ x * 1e-4)
    sb._lockstep(bb, logits=lb)
    torch.cuda.synchronize()
    st_a, _, k_a = sa.envs.get_state()
    st_b, _, k_b = sb.envs.get_state()
    print("step", t, "obs", torch.equal(sa.obs, sb.obs), "state", torch.equal(st_a, st_b), "steps", torch.equal(k_a, k_b),
          "store", all(torch.equal(ba.n_step_buf[x], bb.n_step_buf[x]) for x in ba.n_step_buf),
          "cursor", ba.cursor.tolist(), bb.cursor.tolist(), flush=True)
