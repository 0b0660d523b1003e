"""Per-lockstep logits and obs inside sample(): graph (A) vs eager (B), after a warm-up."""
import sys
import tempfile

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
from msacl_amd.utils.config import build_pipeline, default_msacl_args  # noqa: E402


def pipe(graph):
    torch.manual_seed(0)
    args = default_msacl_args(env_name="DuctedFan", env_num=4096, buffer_warm_size=3000, buffer_max_size=600000,
                              max_iteration=100, eval_interval=10 ** 6, log_save_interval=10 ** 6,
                              apprfunc_save_interval=10 ** 6, save_folder=tempfile.mkdtemp(), seed=0,
                              num_eval_episode=1, trainer_overlap_sampling=False, sampler_use_graph=graph)
    return build_pipeline(args)


A, B = pipe(True), pipe(False)
sa, sb = A[2], B[2]
print("after build obs equal", torch.equal(sa.obs, sb.obs), "eager calls", sa._eager_calls, sb._eager_calls)
rec = {"A": [], "B": []}


def hook(s, key):
    orig = s._lockstep

    def f(store, logits=None, **kw):
        if logits is not None:
            rec[key].append((logits.clone(), s.obs.clone()))
        return orig(store, logits=logits, **kw)
    s._lockstep = f


hook(sa, "A")
hook(sb, "B")
sa._graph = None  # recapture with the hook inside
for call in range(2):
    rec["A"].clear() if call == 0 else None
    A[3].add_batch(sa.sample()[0])
    B[3].add_batch(sb.sample()[0])
    torch.cuda.synchronize()
    ra, rb = rec["A"][-20:], rec["B"][-20:]
    for t in range(20):
        la, oa = ra[t]
        lb, ob = rb[t]
        if not (torch.equal(la, lb) and torch.equal(oa, ob)):
            print("call", call, "lockstep", t, "logits equal", torch.equal(la, lb), "obs-in equal", torch.equal(oa, ob),
                  "max logit diff", (la - lb).abs().max().item())
            break
    else:
        print("call", call, "all 20 locksteps equal")
pa, pb = sa._packed, sb._packed
print("packed equal (excluding unused scal slots)", torch.equal(pa[:-56], pb[:-56]))
if not torch.equal(pa[:-56], pb[:-56]):
    d = (pa[:-56] != pb[:-56]).nonzero().flatten()
    print("differing", d.numel(), "first", d[:8].tolist(), "last", d[-4:].tolist(), "total len", pa.numel())
    print("scal A", pa[-64:-56].tolist(), "\nscal B", pb[-64:-56].tolist())
