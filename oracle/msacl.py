"""CPU ORACLE — test infrastructure only.

NumPy restatement of the MSACL target / certificate math between the network evaluations
(RL/algorithm/msacl.py), with the gradients the fused kernels hand to autograd:
  q_target     msacl.py:242-257  backup, twin-MSE loss, dloss/dq1, dloss/dq2
  lyapunov     msacl.py:279-332  is_clip (cumprod), ESL, lya_diff, loss, dloss/dV(obs), dloss/dV(obs2)
  stability    msacl.py:383-405  advantage, normalisation, PPO-clip loss, dloss/dratio
torch.maximum/minimum split the gradient in half on ties; clamp passes it on the closed box.
Pinned against the reference through tests/golden/msacl_update.npz (full model_update runs).
"""
import numpy as np

F32 = np.float32


def coefficients(n, lya_eta=0.15, alpha1=1.0, alpha2=2.0, lam=0.95):
    k = np.arange(1, n + 1)
    c = ((F32(1 - lya_eta) ** k) * F32(alpha2 / alpha1)) ** F32(0.5)
    w = F32(lam) ** np.arange(n)
    w = (w / w.sum()).astype(F32)
    s = (F32(1 - lya_eta) ** k).astype(F32)
    return c.astype(F32), w, s


def _relu_grad(a):
    return np.where(a > 0, 1.0, np.where(a == 0, 0.5, 0.0)).astype(F32)


def q_target(q1, q2, q1t, q2t, nlogp, rew, done, alpha, gamma, weight=None):
    nq = np.minimum(q1t, q2t)
    backup = (rew + (F32(1) - done) * F32(gamma) * (nq - F32(alpha) * nlogp)).astype(F32)
    N = q1.size
    w = np.ones(q1.shape[0], F32) if weight is None else weight.astype(F32)
    e1, e2 = q1 - backup, q2 - backup
    loss = float((w[:, None] * e1.astype(np.float64) ** 2).sum() / N + (w[:, None] * e2.astype(np.float64) ** 2).sum() / N)
    d1 = (2 * e1 / N * w[:, None]).astype(F32)
    d2 = (2 * e2 / N * w[:, None]).astype(F32)
    abs_td = (0.5 * (np.abs(e1) + np.abs(e2))).mean(1).astype(F32)
    return backup, loss, d1, d2, abs_td


def lyapunov(logp, old_logp, V, V2, obs, obs2, c, w, s, alpha1=1.0, alpha2=2.0, pos_scale=1.0, diff_scale=1.0):
    B, n = V.shape
    N = B * n
    ratio = np.exp(logp - old_logp)
    is_clip = np.cumprod(np.clip(ratio, 0, 1), axis=1).astype(F32)
    pw = (obs ** 2).sum(-1)
    l1, l2 = alpha1 * pw - V, V - alpha2 * pw
    bound = (np.maximum(l1, 0).astype(np.float64).sum() + np.maximum(l2, 0).astype(np.float64).sum()) / N
    start = np.sqrt((obs[:, 0, :] ** 2).sum(-1))
    diff = start[:, None] * c[None, :] - np.sqrt((obs2 ** 2).sum(-1))
    esl = np.where(diff >= 0, F32(1), F32(-1))
    t = esl * (V2 - V[:, :1] * s[None, :])
    lya_diff = (w[None, :] * is_clip * np.maximum(t, 0)).sum(1).astype(F32)
    loss = bound * pos_scale + float(lya_diff.astype(np.float64).mean()) * diff_scale
    dV = (pos_scale / N * (-_relu_grad(l1) + _relu_grad(l2))).astype(F32)
    gt = diff_scale / B * w[None, :] * is_clip * _relu_grad(t)
    dV2 = (gt * esl).astype(F32)
    dV[:, 0] += (gt * esl * (-s[None, :])).sum(1)
    return is_clip, esl, lya_diff, loss, dV, dV2


def stability(V0, V2, ratio, w, s, clip=0.1):
    adv_raw = (w[None, :] * (V0[:, None] * s[None, :] - V2)).sum(1).astype(F32)
    B = adv_raw.size
    mean = adv_raw.astype(np.float64).mean()
    std = adv_raw.astype(np.float64).std(ddof=1)
    adv = ((adv_raw - F32(mean)) / (F32(std) + F32(1e-8))).astype(F32)
    lo, hi = F32(1 - clip), F32(1 + clip)
    rc = np.clip(ratio, lo, hi)
    s1, s2 = ratio * adv, rc * adv
    loss = float(np.minimum(s1, s2).astype(np.float64).mean())
    gclip = ((ratio >= lo) & (ratio <= hi)).astype(F32)
    g = np.where(s1 < s2, adv, np.where(s1 > s2, gclip * adv, 0.5 * adv + 0.5 * gclip * adv))
    return adv_raw, adv, loss, (g / B).astype(F32)
