"""Graph replay vs eager: policy pack+forward, and the rollout step, separately."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import msacl_amd  # noqa: F401,E402
import msacl_amd._native as N  # noqa: E402

D, N3, E = 6, 4, 4096
torch.manual_seed(0)
net = torch.nn.Sequential(torch.nn.Linear(D, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                          torch.nn.Linear(256, N3)).cuda()
n = ctypes.c_int64()
N.check(N.lib().mh_policy_packed_size(D, ctypes.byref(n)), "size")
ps = [p.detach().contiguous() for p in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                        net[4].bias)]
obs = torch.randn(E, D, device="cuda")


def fwd(P, out):
    N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, N3, N.ptr(P), N.stream_of()), "pack")
    N.check(N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, N3, N.ptr(out), N.stream_of()), "fwd")


P1 = torch.empty(n.value, device="cuda")
ref = torch.empty(E, N3, device="cuda")
fwd(P1, ref)
P2 = torch.zeros(n.value, device="cuda")
out = torch.zeros(E, N3, device="cuda")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fwd(P2, out)
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("graph policy replay", r, "equal", torch.equal(out, ref),
          "maxdiff", (out - ref).abs().max().item(), "packed equal (first 268352)", torch.equal(P1[:268352], P2[:268352]),
          flush=True)
    if not torch.equal(P1[:268352], P2[:268352]):
        d = (P1[:268352] != P2[:268352]).nonzero().flatten()
        print("  packed diff idx", d[:8].tolist(), d.numel())
