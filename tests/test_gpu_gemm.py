"""GPU: mh_gemm_f32 (csrc/gemm.hip, f32 MFMA) against a float64 product of the same float32
operands, for the update's layer shapes (B x n = 5,120 and 256 rows; 256-wide hidden layers;
1- and 8-wide heads; the transposed weight-gradient form with K = 5,120, which takes the
cross-workgroup split + reduce launch) and ragged edges. Tolerance: f32 accumulation over K terms,
|err| <= 2e-6 * sqrt(K) * sum_k |a_k b_k| + 1e-6 (the k-ordered fma chain's bound with margin)."""
import ctypes

import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from msacl_amd.apprfunc._fused import gemm

pytestmark = pytest.mark.gpu


def _op(t, trans):
    return t.t() if trans else t


def _ref(a, b, bias, ta, tb, act):
    A = _op(a.double(), ta)
    B = _op(b.double(), tb)
    c = A @ B
    mag = A.abs() @ B.abs()
    if bias is not None:
        c = c + bias.double()
        mag = mag + bias.double().abs()
    if act == 1:
        c = torch.relu(c)
    elif act == 2:
        c = torch.tanh(c)
    return c, mag


SHAPES = [  # (M, N, K)
    (5120, 256, 16), (5120, 256, 256), (5120, 1, 256), (5120, 8, 256), (256, 256, 256), (256, 256, 12),
    (256, 8, 256), (256, 256, 5120), (8, 256, 5120), (1, 256, 5120), (16, 256, 5120), (256, 16, 5120),
    (333, 77, 45), (1, 1, 1), (65, 33, 129), (7, 300, 1000), (4097, 1, 300), (256, 1, 1000), (2048, 1, 3),
    # tall products (k_gemm_tall when op(A) is A: M >= 2,048, N % 64 == 0, K % 4 == 0)
    (5120, 256, 12), (5120, 64, 4), (3001, 128, 20), (2048, 192, 36), (4100, 256, 256),
    # short-K products (k_gemm_shortk: op(A) = A, op(B) = B^T, K <= 32)
    (10240, 256, 12), (5376, 256, 16), (300, 100, 32), (257, 64, 1), (1000, 130, 7),
    # more short-K shapes: several 64-column tiles, ragged last tile
    (700, 300, 20), (3000, 512, 5), (9000, 256, 28),
]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_matches_f64(M, N, K, ta, tb):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K + 10 * ta + tb)
    a = torch.randn(*((K, M) if ta else (M, K)), device="cuda", generator=g)
    b = torch.randn(*((N, K) if tb else (K, N)), device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    act = (M + N + K) % 3
    lda = a.shape[1]
    ldb = b.shape[1]
    c = gemm(a, b, bias, M, N, K, lda, ldb, ta, tb, act)
    ref, mag = _ref(a, b, bias, ta, tb, act)
    err = (c.double() - ref).abs()
    tol = 2e-6 * (K ** 0.5) * mag + 1e-6
    assert bool((err <= tol).all()), f"max err {float(err.max()):.3e}"


@pytest.mark.parametrize("lda_pad,a_off,act", [(0, 0, 2), (4, 0, 1), (3, 0, 0), (0, 1, 2), (4, 4, 2)])
def test_shortk_strided_and_offset_operands(lda_pad, a_off, act):
    """Short-K path (K <= 32, op(B) = B^T) on views: padded leading dimensions (float4 row loads
    only when lda % 4 == 0 and A is 16-byte aligned) and a misaligned start."""
    g = torch.Generator(device="cuda").manual_seed(17 + lda_pad + 5 * a_off + act)
    M, N, K = 5120, 256, 12
    abuf = torch.randn(M * (K + lda_pad) + a_off, device="cuda", generator=g)
    a = abuf[a_off:].reshape(M, K + lda_pad)[:, :K]
    b = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    c = gemm(abuf[a_off:], b, bias, M, N, K, K + lda_pad, K, 0, 1, act)  # pointer + lda (a 1-D view)
    ref, mag = _ref(a.contiguous(), b, bias, 0, 1, act)
    err = (c.double() - ref).abs()
    assert bool((err <= 2e-6 * (K ** 0.5) * mag + 1e-6).all()), f"max err {float(err.max()):.3e}"


def test_gemm_weight_gradient_form_is_deterministic():
    """dW = g^T x (op(A) transposed, K = 5,120 rows): the split partials are summed in split
    order, so repeated launches agree bit for bit."""
    gen = torch.Generator(device="cuda").manual_seed(3)
    gr = torch.randn(5120, 256, device="cuda", generator=gen)
    x = torch.randn(5120, 256, device="cuda", generator=gen)
    c1 = gemm(gr, x, None, 256, 256, 5120, 256, 256, 1, 0)
    c2 = gemm(gr, x, None, 256, 256, 5120, 256, 256, 1, 0)
    assert torch.equal(c1, c2)
    ref = gr.double().t() @ x.double()
    assert float((c1.double() - ref).abs().max()) < 1e-3


def test_gemm_asymmetric_exact_integers():
    """Exact small-integer data: catches any row/column swap of the MFMA C map."""
    M, N, K = 96, 80, 64
    a = (torch.arange(M * K, device="cuda") % 7 - 3).float().reshape(M, K)
    b = (torch.arange(K * N, device="cuda") % 5 - 2).float().reshape(K, N) * (1 + torch.arange(N, device="cuda")) % 4
    c = gemm(a, b.contiguous(), None, M, N, K, K, N, 0, 0)
    assert torch.equal(c, a @ b)


def test_gemm_rejects_bad_leading_dimension():
    a = torch.zeros(4, 4, device="cuda")
    out = torch.empty(4, 4, device="cuda")
    rc = N.lib().mh_gemm_f32(N.ptr(a), N.ptr(a), None, N.ptr(out), 4, 4, 4, 2, 4, 4, 0, 0, 0, None, N.stream_of())
    assert rc != 0 and b"leading dimension" in N.lib().mh_last_error()


def test_gemm_workspace_query():
    wf = ctypes.c_int64()
    assert N.lib().mh_gemm_workspace(256, 256, 5120, ctypes.byref(wf)) == 0
    assert wf.value > 0 and wf.value % (256 * 256) == 0
    assert N.lib().mh_gemm_workspace(5120, 256, 256, ctypes.byref(wf)) == 0
    assert wf.value == 0


@pytest.mark.parametrize("tb", [0, 1])
def test_tall_gemm_strided_operands(tb):
    """Tall path with leading dimensions larger than the row (views into wider buffers)."""
    g = torch.Generator(device="cuda").manual_seed(11 + tb)
    M, N, K = 5120, 128, 64
    abuf = torch.randn(M, K + 12, device="cuda", generator=g)
    bbuf = torch.randn(*((N, K + 8) if tb else (K, N + 64)), device="cuda", generator=g)
    a = abuf[:, :K]
    b = bbuf[:, :K] if tb else bbuf[:, :N]
    bias = torch.randn(N, device="cuda", generator=g)
    c = gemm(abuf, bbuf, bias, M, N, K, abuf.shape[1], bbuf.shape[1], 0, tb, 1)
    ref, mag = _ref(a.contiguous(), b.contiguous(), bias, 0, tb, 1)
    err = (c.double() - ref).abs()
    assert bool((err <= 2e-6 * (K ** 0.5) * mag + 1e-6).all()), f"max err {float(err.max()):.3e}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 5120), (256, 256, 10240), (64, 128, 1000), (128, 64, 3000),
                                   (256, 192, 1088)])
def test_deep_gemm_weight_gradient(M, N, K):
    """k_gemm_deep (A^T B, K >> M, N: the weight gradients): K split over workgroups, partials
    added in split order; ragged K (k rows past K read 0) and a strided B."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(K, M, device="cuda", generator=g)
    bbuf = torch.randn(K, N + 8, device="cuda", generator=g)
    c = gemm(a, bbuf, None, M, N, K, M, N + 8, 1, 0)
    ref, mag = _ref(a, bbuf[:, :N].contiguous(), None, 1, 0, 0)
    err = (c.double() - ref).abs()
    assert bool((err <= 2e-6 * (K ** 0.5) * mag + 1e-6).all()), f"max err {float(err.max()):.3e}"
    assert torch.equal(c, gemm(a, bbuf, None, M, N, K, M, N + 8, 1, 0))
