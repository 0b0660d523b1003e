"""GPU: HipAdam (mh_adam_multi, csrc/optim.hip) against torch.optim.Adam(fused=True,
capturable=True) — the optimiser every algorithm used before — over several steps of random
gradients on an MLP's parameters (ragged sizes, a scalar parameter, a parameter without a
gradient). Same scalars as PyTorch (1 - beta and the bias corrections formed in double from the
Python floats); the element math differs from PyTorch's kernel in float32 rounding only.
Tolerance: parameters within 1e-4 lr per step of PyTorch's (the update is O(lr) per step),
moments rtol 1e-5 / atol 1e-6 of their scale; step counters equal."""
import pytest
import torch

import msacl_amd  # noqa: F401
from msacl_amd.utils.dist import cuda_graph
from msacl_amd.algorithm._update_graph import HipAdam

pytestmark = pytest.mark.gpu


def _params(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    shapes = [(256, 16), (256,), (256, 256), (256,), (1, 256), (1,), (), (37, 5)]
    return [torch.nn.Parameter(torch.randn(s, device="cuda", generator=g) * 0.1) for s in shapes]


@pytest.mark.parametrize("lr", [3e-4, 1e-2])
def test_hip_adam_matches_torch_fused(lr):
    a = _params(1)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    oa = HipAdam(a, lr=lr)
    ob = torch.optim.Adam(b, lr=lr, fused=True, capturable=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    for it in range(6):
        for i, (pa, pb) in enumerate(zip(a, b)):
            if i == 7 and it % 2 == 0:  # no gradient on some steps: skipped, its step not advanced
                pa.grad = pb.grad = None
                continue
            gr = torch.randn(pa.shape, device="cuda", generator=g) * (10.0 ** (i % 3 - 1))
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        sa, sb = oa.state[pa], ob.state[pb]
        assert float(sa["step"]) == float(sb["step"])
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=0, atol=1e-4 * lr * 6)
        for key in ("exp_avg", "exp_avg_sq"):
            scale = float(sb[key].abs().max()) + 1e-30
            torch.testing.assert_close(sa[key], sb[key], rtol=1e-5, atol=1e-6 * scale)


def test_hip_adam_state_dict_round_trip_and_graph_capture():
    a = _params(2)
    opt = HipAdam(a, lr=1e-3)
    for p in a:
        p.grad = torch.ones_like(p)
    opt.step()
    sd = opt.state_dict()
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    opt2 = torch.optim.Adam(b, lr=1e-3, capturable=True)
    opt2.load_state_dict(sd)  # same state layout as torch's capturable Adam
    assert float(opt2.state[b[0]]["step"]) == 1.0
    # captured step replays advance the device step counter
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        opt.step()
    torch.cuda.current_stream().wait_stream(s)
    gph = torch.cuda.CUDAGraph()
    with cuda_graph(gph):
        opt.step()
    for _ in range(3):
        gph.replay()
    torch.cuda.synchronize()
    assert float(opt.state[a[0]]["step"]) == 5.0  # 1 eager + 1 warm-up + 3 replays (capture runs nothing)


def test_adam_steps_mixed_learning_rates_equal_separate_steps():
    """adam_steps over optimisers with different learning rates (the policy and alpha Adams:
    mh_adam_multi_lr, one launch) equals each optimiser's own step bit for bit."""
    from msacl_amd.algorithm._update_graph import adam_steps
    a1, a2 = _params(3), [torch.nn.Parameter(torch.tensor(1.0, device="cuda"))]
    b1 = [torch.nn.Parameter(p.detach().clone()) for p in a1]
    b2 = [torch.nn.Parameter(p.detach().clone()) for p in a2]
    oa1, oa2, ob1, ob2 = HipAdam(a1, lr=3e-4), HipAdam(a2, lr=1e-2), HipAdam(b1, lr=3e-4), HipAdam(b2, lr=1e-2)
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(4):
        for pa, pb in zip(a1 + a2, b1 + b2):
            gr = torch.randn(pa.shape, device="cuda", generator=g)
            pa.grad, pb.grad = gr.clone(), gr.clone()
        adam_steps(oa1, oa2)
        ob1.step()
        ob2.step()
    for oa, ob, pa_l, pb_l in ((oa1, ob1, a1, b1), (oa2, ob2, a2, b2)):
        for pa, pb in zip(pa_l, pb_l):
            assert torch.equal(pa.detach(), pb.detach())
            for key in ("step", "exp_avg", "exp_avg_sq"):
                assert torch.equal(oa.state[pa][key], ob.state[pb][key])


def test_polyak_kernel_matches_foreach_bit_exact():
    """mh_polyak_multi (algorithm/_update_graph.py polyak_) vs the multi-tensor PyTorch ops it
    replaces, p_t.mul_(1 - tau); p_t.add_(tau * p): the same two float32 roundings, bit-exact."""
    from msacl_amd.algorithm._update_graph import polyak_
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 256), torch.nn.ReLU(), torch.nn.Linear(256, 1)).cuda()
    targ = torch.nn.Sequential(torch.nn.Linear(16, 256), torch.nn.ReLU(), torch.nn.Linear(256, 1)).cuda()
    ref = [p.detach().clone() for p in targ.parameters()]
    for _ in range(3):
        polyak_(net, targ, 0.005)
        with torch.no_grad():
            torch._foreach_mul_(ref, 1 - 0.005)
            torch._foreach_add_(ref, torch._foreach_mul([p.data for p in net.parameters()], 0.005))
    for a, b in zip(targ.parameters(), ref):
        assert torch.equal(a.detach(), b)
