"""GPU: the fused MSACL policy-loss pieces (csrc/msacl_kernels.hip k_policy_loss / k_ratio0,
used by algorithm/msacl.py `_policy_update`, reference msacl.py:383-405) against the PyTorch
expressions they replace, forward and backward:
  loss = (min(q1, q2) - exp(log_alpha) * logp).mean(), entropy = -logp.mean()
  is_ratio = exp(logp_new - old_logp)[:, 0]
Tolerance: the loss/entropy sums run in double on the device (torch: float32 tree), so they
agree to 1e-6 relative of sum|terms|; element-wise gradients are bit-exact except the step-0
ratio gradient (one float32 multiply of the same values: exact as well)."""
import pytest
import torch

import msacl_amd  # noqa: F401
from msacl_amd.algorithm.msacl import _PolicyQLoss, _Ratio0

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,n", [(256, 20), (1, 1), (3, 7), (1000, 33)])
def test_policy_q_loss_matches_torch(B, n):
    g = torch.Generator(device="cuda").manual_seed(B * 31 + n)
    q1 = torch.randn(B, n, device="cuda", generator=g)
    q2 = torch.randn(B, n, device="cuda", generator=g)
    q2[:, ::3] = q1[:, ::3]  # ties: autograd gives each input half the gradient
    lp = torch.randn(B, n, device="cuda", generator=g)
    log_alpha = torch.tensor(-0.7, device="cuda")
    a = [t.clone().requires_grad_(True) for t in (q1, q2, lp)]
    b = [t.clone().requires_grad_(True) for t in (q1, q2, lp)]
    loss, ent = _PolicyQLoss.apply(a[0], a[1], a[2], log_alpha)
    ref = (torch.min(b[0], b[1]) - log_alpha.exp() * b[2]).mean()
    ref_ent = -b[2].mean().detach()
    scale = float((torch.min(q1, q2).abs() + lp.abs() * log_alpha.exp()).mean()) + 1e-30
    assert abs(float(loss) - float(ref)) <= 1e-6 * scale
    assert abs(float(ent) - float(ref_ent)) <= 1e-6 * (float(lp.abs().mean()) + 1e-30)
    assert not ent.requires_grad
    up = torch.tensor(-1.3, device="cuda")
    torch.autograd.backward([loss], [up])
    torch.autograd.backward([ref], [up])
    for x, y in zip(a, b):
        torch.testing.assert_close(x.grad, y.grad, rtol=0, atol=0)


def test_policy_q_loss_nan_propagates():
    q1 = torch.tensor([[1.0, float("nan")]], device="cuda")
    q2 = torch.tensor([[0.5, 2.0]], device="cuda")
    lp = torch.zeros(1, 2, device="cuda")
    loss, _ = _PolicyQLoss.apply(q1, q2, lp, torch.tensor(0.0, device="cuda"))
    assert torch.isnan(loss)


@pytest.mark.parametrize("B,n", [(256, 20), (1, 1), (17, 5)])
def test_ratio0_matches_torch(B, n):
    g = torch.Generator(device="cuda").manual_seed(B + n)
    lp = (torch.randn(B, n, device="cuda", generator=g) * 0.3).requires_grad_(True)
    old = torch.randn(B, n, device="cuda", generator=g) * 0.3
    lp2 = lp.detach().clone().requires_grad_(True)
    r = _Ratio0.apply(lp, old)
    ref = torch.exp(lp2 - old)[:, 0]
    assert torch.equal(r, ref)
    up = torch.randn(B, device="cuda", generator=g)
    torch.autograd.backward([r], [up])
    torch.autograd.backward([ref], [up])
    assert torch.equal(lp.grad, lp2.grad)


@pytest.mark.parametrize("B", [256, 1, 300])
def test_policy_combine_matches_torch(B):
    """mh_msacl_policy_combine: loss_policy = -loss_q - loss_ppo and -d_ratio, bit-exact with the
    PyTorch expressions it replaces (msacl.py:401-405)."""
    import msacl_amd._native as N
    g = torch.Generator(device="cuda").manual_seed(B)
    lq = torch.randn(1, device="cuda", generator=g)
    lppo = torch.randn(1, device="cuda", generator=g)
    dr = torch.randn(B, device="cuda", generator=g)
    lp, neg = torch.empty(1, device="cuda"), torch.empty(B, device="cuda")
    N.check(N.lib().mh_msacl_policy_combine(N.ptr(lq), N.ptr(lppo), N.ptr(dr), B, N.ptr(lp), N.ptr(neg),
                                            N.stream_of(lq.device)), "mh_msacl_policy_combine")
    assert torch.equal(lp[0], -lq[0] - lppo[0])
    assert torch.equal(neg, -dr)


@pytest.mark.parametrize("log_alpha,entropy,target", [(1.0, 3.7, -5.0), (-2.3, -6.1, -4.0), (0.0, 0.0, 0.0)])
def test_alpha_grad_matches_autograd(log_alpha, entropy, target):
    """mh_msacl_alpha_grad equals autograd's gradient of exp(log_alpha) * (entropy - target)
    w.r.t. log_alpha (msacl.py:429-437), bit for bit."""
    import msacl_amd._native as N
    la = torch.tensor(log_alpha, device="cuda", requires_grad=True)
    ent = torch.tensor(entropy, device="cuda")
    (la.exp() * (ent - target)).backward()
    out = torch.empty((), device="cuda")
    N.check(N.lib().mh_msacl_alpha_grad(N.ptr(la.detach()), N.ptr(ent), float(target), N.ptr(out),
                                        N.stream_of(ent.device)), "mh_msacl_alpha_grad")
    assert torch.equal(out, la.grad)


@pytest.mark.parametrize("B,n", [(256, 20), (3, 5), (1100, 2)])
def test_policy_objective_equals_separate_kernels(B, n):
    """mh_msacl_policy_objective[_backward] (the policy step's whole objective in one launch each way)
    equals the policy-loss, ratio, PPO-clip and combine kernels with their autograd seeds (-1 and
    -d_ratio) bit for bit: loss, entropy, advantage, d_ratio and every input gradient."""
    import msacl_amd._native as N
    from msacl_amd.algorithm.msacl import _PolicyObjective, _Scratch
    g = torch.Generator(device="cuda").manual_seed(B * 7 + n)
    q1 = torch.randn(B, n, device="cuda", generator=g)
    q2 = torch.randn(B, n, device="cuda", generator=g)
    q2[:, ::3] = q1[:, ::3]
    lp = torch.randn(B, n, device="cuda", generator=g)
    lp_new = torch.randn(B, n, device="cuda", generator=g) * 0.1
    old = lp_new + torch.randn(B, n, device="cuda", generator=g) * 0.1
    log_alpha = torch.tensor(0.3, device="cuda")
    adv_raw = torch.randn(B, device="cuda", generator=g)
    stats = torch.stack([adv_raw.double().sum(), (adv_raw.double() ** 2).sum()])
    st = N.stream_of(q1.device)

    s = _Scratch(B, n, q1.device)
    s.adv_raw.copy_(adv_raw)
    s.stats.copy_(stats)
    a = [t.clone().requires_grad_(True) for t in (q1, q2, lp, lp_new)]
    loss, ent = _PolicyObjective.apply(a[0], a[1], a[2], a[3], old, log_alpha, s, float(B), 0.1)
    torch.autograd.backward([loss], [torch.tensor(1.0, device="cuda")])

    b = [t.clone().requires_grad_(True) for t in (q1, q2, lp, lp_new)]
    lq, ent2 = _PolicyQLoss.apply(b[0], b[1], b[2], log_alpha)
    ratio = _Ratio0.apply(b[3], old)
    adv, lppo, dr = torch.empty(B, device="cuda"), torch.empty(1, device="cuda"), torch.empty(B, device="cuda")
    N.check(N.lib().mh_msacl_ppo_clip(N.ptr(ratio.detach().contiguous()), N.ptr(adv_raw), N.ptr(stats), float(B), 0.1, B,
                                      N.ptr(adv), N.ptr(lppo), N.ptr(dr), st), "ppo_clip")
    lpol, neg = torch.empty(1, device="cuda"), torch.empty(B, device="cuda")
    N.check(N.lib().mh_msacl_policy_combine(N.ptr(lq.detach()), N.ptr(lppo), N.ptr(dr), B, N.ptr(lpol), N.ptr(neg), st),
            "combine")
    torch.autograd.backward([lq, ratio], [torch.tensor(-1.0, device="cuda"), neg])
    assert torch.equal(loss.detach(), lpol[0]) and torch.equal(ent, ent2)
    assert torch.equal(s.adv, adv) and torch.equal(s.d_ratio, dr) and torch.equal(s.loss_ppo, lppo)
    for x, y in zip(a, b):
        assert torch.equal(x.grad, y.grad)


@pytest.mark.parametrize("B,n", [(256, 20), (3, 5), (1100, 2)])
@pytest.mark.parametrize("with_alpha", [True, False])
def test_policy_objective_step_equals_objective_and_backward(B, n, with_alpha):
    """mh_msacl_policy_objective_step (objective + its backward for the unit seed + the alpha
    gradient, one launch) equals _PolicyObjective forward / backward with seed 1 and
    mh_msacl_alpha_grad bit for bit."""
    import msacl_amd._native as N
    from msacl_amd.algorithm.msacl import _PolicyObjective, _Scratch, _policy_objective_step
    g = torch.Generator(device="cuda").manual_seed(B * 11 + n)
    q1 = torch.randn(B, n, device="cuda", generator=g)
    q2 = torch.randn(B, n, device="cuda", generator=g)
    q2[:, ::4] = q1[:, ::4]
    lp = torch.randn(B, n, device="cuda", generator=g)
    lp_new = torch.randn(B, n, device="cuda", generator=g) * 0.1
    old = lp_new + torch.randn(B, n, device="cuda", generator=g) * 0.1
    log_alpha = torch.tensor(-0.4, device="cuda")
    adv_raw = torch.randn(B, device="cuda", generator=g)
    stats = torch.stack([adv_raw.double().sum(), (adv_raw.double() ** 2).sum()])
    target = -4.0

    s1 = _Scratch(B, n, q1.device)
    s1.adv_raw.copy_(adv_raw)
    s1.stats.copy_(stats)
    a = [t.clone().requires_grad_(True) for t in (q1, q2, lp, lp_new)]
    loss, ent = _PolicyObjective.apply(a[0], a[1], a[2], a[3], old, log_alpha, s1, float(B), 0.2)
    torch.autograd.backward([loss], [torch.tensor(1.0, device="cuda")])
    ag_ref = torch.full((), 7.0, device="cuda")
    N.check(N.lib().mh_msacl_alpha_grad(N.ptr(log_alpha), N.ptr(ent.contiguous()), target, N.ptr(ag_ref),
                                        N.stream_of(q1.device)), "alpha_grad")

    s2 = _Scratch(B, n, q1.device)
    s2.adv_raw.copy_(adv_raw)
    s2.stats.copy_(stats)
    ag = torch.full((), 7.0, device="cuda")
    loss2, ent2, seeds = _policy_objective_step(q1, q2, lp, lp_new, old, log_alpha, s2, float(B), 0.2, target,
                                                ag if with_alpha else None)
    torch.cuda.synchronize()
    assert torch.equal(loss.detach(), loss2) and torch.equal(ent, ent2)
    assert torch.equal(s1.adv, s2.adv) and torch.equal(s1.d_ratio, s2.d_ratio) and torch.equal(s1.ratio, s2.ratio)
    for x, d in zip(a, seeds):
        assert torch.equal(x.grad, d)
    if with_alpha:
        assert torch.equal(ag, ag_ref)
    else:
        assert ag.item() == 7.0
