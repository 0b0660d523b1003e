"""Is the fused policy forward bit-stable when other kernels share the GPU? (race probe)"""
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
P = torch.empty(n.value, device="cuda")
ps = [p.detach().contiguous() for p in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                        net[4].bias)]
N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, N3, N.ptr(P), N.stream_of()), "pack")
obs = torch.randn(E, D, device="cuda")
ref = torch.empty(E, N3, device="cuda")
N.check(N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, N3, N.ptr(ref), N.stream_of()), "fwd")
torch.cuda.synchronize()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
a = torch.randn(4096, 4096, device="cuda")
bad = 0
for it in range(50):
    out = torch.empty(E, N3, device="cuda")
    with torch.cuda.stream(s1):
        for _ in range(3):
            a = torch.tanh(a @ a * 1e-3)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(it * 2000)
        N.check(N.lib().mh_policy_forward(N.ptr(P), N.ptr(obs), E, D, N3, N.ptr(out), N.stream_of()), "fwd")
        # re-pack too (the sampler packs every sample())
        N.check(N.lib().mh_policy_pack(*[N.ptr(p) for p in ps], D, 256, 256, N3, N.ptr(P), N.stream_of()), "pack")
    torch.cuda.synchronize()
    if not torch.equal(out, ref):
        bad += 1
        print("iter", it, "max diff", (out - ref).abs().max().item(), flush=True)
print("policy forward: differing runs", bad, "of 50")
