"""GPU: TanhGaussDistribution.rsample / log_prob on HIP float32 logits run as single kernels
(csrc/dist_kernels.hip); checked against the same distribution evaluated with PyTorch ops
(RL/utils/act_distribution_cls.py:15-85 math), forward values and gradients w.r.t. the logits.
Tolerance: against a float64 evaluation of the same expressions, every element of the kernels'
result (values and gradients) is within 1e-5 + 1e-5 |x| of it, or no further from it than 4x
PyTorch's own float32 error on that element, or — where tanh(z) is saturated (1 - tanh(z)^2 <
1e-3, so 1 + 1e-6 - tanh(z)^2 keeps only a few float32 digits, in PyTorch's evaluation as in the
kernel's) — no further than 4x PyTorch's worst float32 error over the saturated elements."""
import numpy as np
import pytest
import torch
import torch.distributions.normal as tdn

import msacl_amd  # noqa: F401
from msacl_amd.utils.act_distribution_cls import TanhGaussDistribution, _independent_normal, EPS

pytestmark = pytest.mark.gpu


def _torch_rsample(logits, eps, hi, lo):
    mean, std = torch.chunk(logits, 2, dim=-1)
    z = mean + eps * std
    g = _independent_normal(mean, std)
    act = (hi - lo) / 2 * torch.tanh(z) + (hi + lo) / 2
    logp = (g.log_prob(z) - torch.log(1 + EPS - torch.pow(torch.tanh(z), 2)).sum(-1)
            - torch.log((hi - lo) / 2).sum(-1))
    return act, logp


def _torch_log_prob(logits, a, hi, lo):
    mean, std = torch.chunk(logits, 2, dim=-1)
    z = torch.atanh((1 - EPS) * (2 * a - (hi + lo)) / (hi - lo))
    return _independent_normal(mean, std).log_prob(z) - torch.log(
        (hi - lo) / 2 * (1 + EPS - torch.pow(torch.tanh(z), 2))).sum(-1)


def _close(fused, torch32, ref64, sat=None, rtol=1e-5, atol=1e-5):
    """Elementwise: |fused - ref64| <= atol + rtol |ref64|  or  <= 4 |torch32 - ref64|  or, on
    saturated elements (`sat`), <= 4 max_sat |torch32 - ref64|."""
    assert fused.shape == torch32.shape == ref64.shape
    ef = (fused.double() - ref64).abs()
    et = (torch32.double() - ref64).abs()
    ok = (ef <= atol + rtol * ref64.abs()) | (ef <= 4 * et)
    if sat is not None and bool(sat.any()):
        ok = ok | (sat & (ef <= 4 * et[sat].max()))
    assert bool(ok.all()), (f"{int((~ok).sum())} / {ok.numel()} elements off: max fused err "
                            f"{float(ef.max()):.3e}, max torch err {float(et.max()):.3e}")


def _case(shape, A, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mean = torch.randn(*shape, A, device="cuda", generator=g) * 0.8
    std = torch.rand(*shape, A, device="cuda", generator=g) * 0.9 + 0.05
    logits = torch.cat([mean, std], -1)
    hi = torch.rand(A, device="cuda", generator=g) * 3 + 0.5
    lo = -torch.rand(A, device="cuda", generator=g) * 3 - 0.5
    eps = torch.randn(*shape, A, device="cuda", generator=g)
    return logits, hi, lo, eps


def _saturated(z64):
    """Per action dim: 1 - tanh(z)^2 < 1e-3; (dims, rows, logits columns)."""
    sat = (1 - torch.tanh(z64) ** 2) < 1e-3
    return sat, sat.any(-1), torch.cat([sat, sat], -1)


def _dist(logits, hi, lo):
    d = TanhGaussDistribution(logits)
    d.act_high_lim, d.act_low_lim = hi, lo
    return d


@pytest.mark.parametrize("shape,A", [((4096,), 4), ((256, 5), 4), ((1000,), 1), ((333,), 2), ((7, 3), 8), ((1,), 3)])
def test_rsample_matches_torch(monkeypatch, shape, A):
    logits, hi, lo, eps = _case(shape, A, seed=A * 31 + len(shape))
    monkeypatch.setattr(tdn, "_standard_normal", lambda s, dtype, device: eps.clone())
    l1 = logits.clone().requires_grad_(True)
    act, logp = _dist(l1, hi, lo).rsample()
    l2 = logits.clone().requires_grad_(True)
    act_r, logp_r = _torch_rsample(l2, eps, hi, lo)
    l3 = logits.double().requires_grad_(True)
    act_d, logp_d = _torch_rsample(l3, eps.double(), hi.double(), lo.double())
    _, sat_row, sat_col = _saturated(logits.double()[..., :A] + eps.double() * logits.double()[..., A:])
    assert act.shape == act_r.shape and logp.shape == logp_r.shape
    _close(act, act_r, act_d.detach())
    _close(logp, logp_r, logp_d.detach(), sat_row)
    g = torch.Generator(device="cuda").manual_seed(99)
    w = torch.randn(act.shape, device="cuda", generator=g)
    v = torch.randn(logp.shape, device="cuda", generator=g)
    ((act * w).sum() + (logp * v).sum()).backward()
    ((act_r * w).sum() + (logp_r * v).sum()).backward()
    ((act_d * w.double()).sum() + (logp_d * v.double()).sum()).backward()
    _close(l1.grad, l2.grad, l3.grad, sat_col)


def test_rsample_logp_only_and_act_only_grads(monkeypatch):
    logits, hi, lo, eps = _case((2048,), 4, seed=5)
    monkeypatch.setattr(tdn, "_standard_normal", lambda s, dtype, device: eps.clone())
    _, _, sat_col = _saturated(logits.double()[..., :4] + eps.double() * logits.double()[..., 4:])
    for use in ("act", "logp"):
        l1 = logits.clone().requires_grad_(True)
        l2 = logits.clone().requires_grad_(True)
        l3 = logits.double().requires_grad_(True)
        a1, p1 = _dist(l1, hi, lo).rsample()
        a2, p2 = _torch_rsample(l2, eps, hi, lo)
        a3, p3 = _torch_rsample(l3, eps.double(), hi.double(), lo.double())
        (a1.sum() if use == "act" else p1.sum()).backward()
        (a2.sum() if use == "act" else p2.sum()).backward()
        (a3.sum() if use == "act" else p3.sum()).backward()
        _close(l1.grad, l2.grad, l3.grad, sat_col)


@pytest.mark.parametrize("shape,A", [((4096,), 4), ((128, 5), 4), ((999,), 1), ((64,), 8)])
def test_log_prob_matches_torch(shape, A):
    logits, hi, lo, eps = _case(shape, A, seed=A * 7 + 1)
    with torch.no_grad():
        act, _ = _torch_rsample(logits, eps, hi, lo)
    l1 = logits.clone().requires_grad_(True)
    lp = _dist(l1, hi, lo).log_prob(act)
    l2 = logits.clone().requires_grad_(True)
    lp_r = _torch_log_prob(l2, act, hi, lo)
    l3 = logits.double().requires_grad_(True)
    lp_d = _torch_log_prob(l3, act.double(), hi.double(), lo.double())
    z64 = torch.atanh((1 - EPS) * (2 * act.double() - (hi + lo).double()) / (hi - lo).double())
    _, sat_row, sat_col = _saturated(z64)
    assert lp.shape == lp_r.shape
    _close(lp, lp_r, lp_d.detach(), sat_row)
    w = torch.randn(lp.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(98))
    (lp * w).sum().backward()
    (lp_r * w).sum().backward()
    (lp_d * w.double()).sum().backward()
    _close(l1.grad, l2.grad, l3.grad, sat_col)


def test_empty_batch():
    """No rows: empty outputs, no launch (PyTorch's Independent.log_prob raises on this shape)."""
    logits, hi, lo, _ = _case((0,), 3, seed=2)
    act, logp = _dist(logits.requires_grad_(True), hi, lo).rsample()
    assert act.shape == (0, 3) and logp.shape == (0,)
    assert _dist(logits, hi, lo).log_prob(act.detach()).shape == (0,)


def test_fused_path_is_taken(monkeypatch):
    """The kernels (not the PyTorch expression) produce the result on HIP float32 logits."""
    import msacl_amd._native as N
    calls = []
    lib = N.lib()
    orig = lib.mh_tanh_gauss_rsample

    class Spy:
        def __getattr__(self, name):
            return getattr(lib, name)

        def mh_tanh_gauss_rsample(self, *a):
            calls.append(1)
            return orig(*a)

    monkeypatch.setattr(N, "lib", lambda: Spy())
    logits, hi, lo, _ = _case((64,), 4, seed=1)
    _dist(logits, hi, lo).rsample()
    assert calls == [1]
    np.testing.assert_equal(len(calls), 1)


def test_stocha_head_matches_torch():
    """StochaPolicy head (mh_stocha_head[_backward]) vs chunk + clamp + exp + cat under autograd,
    including log_std exactly at and beyond the clamp bounds (the gradient mask is inclusive)."""
    from msacl_amd.apprfunc._fused import StochaHead
    lo, hi = -20.0, 1.0
    g = torch.Generator(device="cuda").manual_seed(11)
    raw = torch.randn(5120, 8, device="cuda", generator=g) * 3
    raw[0, 4:] = torch.tensor([lo, hi, lo - 1, hi + 1], device="cuda")
    r1 = raw.clone().requires_grad_(True)
    r2 = raw.clone().requires_grad_(True)
    y1 = StochaHead.apply(r1, lo, hi)
    mean, ls = torch.chunk(r2, 2, dim=-1)
    y2 = torch.cat((mean, torch.clamp(ls, lo, hi).exp()), dim=-1)
    torch.testing.assert_close(y1, y2, rtol=2.5e-7, atol=0)
    w = torch.randn(y1.shape, device="cuda", generator=g)
    (y1 * w).sum().backward()
    (y2 * w).sum().backward()
    torch.testing.assert_close(r1.grad, r2.grad, rtol=5e-7, atol=0)
    assert float(r1.grad[0, 6]) == 0.0 and float(r1.grad[0, 7]) == 0.0 and float(r1.grad[0, 4]) != 0.0


@pytest.mark.parametrize("R,A,D", [(5120, 4, 12), (257, 1, 3), (1000, 8, 9)])
def test_policy_head_equals_separate_kernels(R, A, D):
    """mh_policy_head (MSACL's policy step head: StochaPolicy std + TanhGauss rsample into the
    critic input [obs | act] + its log-prob + log_prob(old_act)) and its backward equal the
    separate StochaHead / rsample / concat / log_prob autograd chain bit for bit, with log-stds on
    both sides of the clamp bounds."""
    from msacl_amd.algorithm.msacl import _PolicyHead
    from msacl_amd.apprfunc._fused import StochaHead
    from msacl_amd.utils.act_distribution_cls import TanhGaussDistribution
    g = torch.Generator(device="cuda").manual_seed(R + A + D)
    raw = torch.randn(R, 2 * A, device="cuda", generator=g)
    raw[:, A:] = raw[:, A:] * 3.0 - 1.0
    raw[::7, A] = 1.5   # above max_log_std = 1 (clamped: no gradient)
    raw[::11, A] = -25.0  # below min_log_std = -20
    eps = torch.randn(R, A, device="cuda", generator=g)
    obs = torch.randn(R, D, device="cuda", generator=g)
    hi = torch.linspace(1.0, 3.0, A, device="cuda")
    lo = -hi * 0.5
    old_act = lo + (hi - lo) * torch.rand(R, A, device="cuda", generator=g)
    d_xq = torch.randn(R, D + A, device="cuda", generator=g)
    d_new = torch.randn(R, device="cuda", generator=g)
    d_old = torch.randn(R, device="cuda", generator=g)

    r1 = raw.clone().requires_grad_(True)
    xq, new_lp, old_lp = _PolicyHead.apply(r1, eps, obs, old_act, hi, lo, -20.0, 1.0)
    torch.autograd.backward([xq, new_lp, old_lp], [d_xq, d_new, d_old])

    r2 = raw.clone().requires_grad_(True)
    logits = StochaHead.apply(r2, -20.0, 1.0)
    dist = TanhGaussDistribution(logits)
    dist.act_high_lim, dist.act_low_lim = hi, lo
    import torch.distributions.normal as tdn
    orig = tdn._standard_normal
    tdn._standard_normal = lambda shape, dtype, device: eps.reshape(shape)
    try:
        act, lp = dist.rsample()
    finally:
        tdn._standard_normal = orig
    xq_ref = torch.cat([obs, act], -1)
    olp_ref = dist.log_prob(old_act)
    torch.autograd.backward([xq_ref, lp, olp_ref], [d_xq, d_new, d_old])
    assert torch.equal(xq, xq_ref)
    assert torch.equal(new_lp, lp)
    assert torch.equal(old_lp, olp_ref)
    torch.testing.assert_close(r1.grad, r2.grad, rtol=0, atol=0)
