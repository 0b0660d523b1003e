"""CPU ORACLE — test infrastructure only (imported by tests/ and __graft_entry__.smoke(), never
by the product path).

Restatement of the engine's in-kernel random draws, so that the sampler's actions, log-probs and
reset states can be checked against values computed from the seed alone:

  * key: Philox4x32-10 (Salmon et al., SC'11; oracle/per.py, pinned by the Random123
    known-answer vectors in tests/test_per_oracle.py) of the counter
    (env lo, env hi ^ (stream << 16), tick lo, tick hi) under key (seed lo, seed hi), where the
    tick is the env's own counter (csrc/philox.h make_rng / Rng::draw). Every lockstep step of
    env e uses tick = its counter and advances it by one (csrc/rollout.hip k_rollout,
    csrc/sample_fused.hip env_lockstep); a drawn reset outside a step (k_reset) does too.
  * action noise (stream 0): Box–Muller on four 24-bit uniforms, u1 = 1 - (x >> 8) 2^-24,
    u2 = (y >> 8) 2^-24, u3 = 1 - (z >> 8) 2^-24, u4 = (w >> 8) 2^-24;
    eps = (a cos 2 pi u2, a sin 2 pi u2, b cos 2 pi u4, b sin 2 pi u4), a = sqrt(-2 ln u1),
    b = sqrt(-2 ln u3) — evaluated here in float64 on the exact uniforms (the kernel evaluates it
    in float32 on the hardware transcendentals: Rng::normal4f_fast). The reference's noise is
    torch's CPU generator (RL/utils/act_distribution_cls.py:46, Normal.sample), which no device
    can replay: the draw is the engine's own, and this oracle pins it.
  * reset draws (streams 1..4, csrc/reset_draw.h): uniform components
    float32(lo + (hi - lo) u), u = word 2^-32, in float64 (bit-exact with the kernels), for the
    boxes of RL/env/VanderPol.py:79-82, Pendulum.py:83-86, DuctedFan.py:89-92, TwoLink.py:81-84,
    SingleTrackCar.py:121-124, QuadTracking.py:169-186 (x, v, Omega uniform in +-0.01; R the
    rotation of a N(0, 0.01^2 I) rotation vector, here in float64);
  * tanh_gauss_sample: TanhGaussDistribution.sample (act_distribution_cls.py:45-57) of
    (logits, eps) with the sample z = mean + std eps rounded to float32 as the reference's float32
    tensor holds it, everything after that in float64 (`1 + EPS` is the float32 scalar PyTorch
    uses, 1.00000095367431640625), then the sampler's clip (base.py:136-143).
"""
import numpy as np

from oracle.per import philox4x32_10

MASK = np.uint64(0xFFFFFFFF)
F32 = np.float32
ONE_PLUS_EPS = float(np.float32(1.0 + 1e-6))  # PyTorch's float32 evaluation of `1 + EPS`
LOG_SQRT_2PI = 0.5 * np.log(2.0 * np.pi)


def draw_words(seed, env, tick, stream):
    """Rng::draw(stream) of make_rng(seed, env, tick) for arrays env [n] (int) and tick [n] (uint32)."""
    env = np.asarray(env, np.uint64)
    tick = np.asarray(tick, np.uint64)
    ctr = np.stack([env & MASK, (env >> np.uint64(32)) ^ np.uint64((int(stream) << 16) & 0xFFFFFFFF),
                    tick & MASK, tick >> np.uint64(32)], -1)
    return philox4x32_10(ctr, (int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF))


def _uniforms24(q):
    v = (q >> np.uint32(8)).astype(np.float64) * 2.0 ** -24
    return 1.0 - v[:, 0], v[:, 1], 1.0 - v[:, 2], v[:, 3]


def box_muller(q):
    """Four standard normals per row of Philox words q [n, 4] (uint32), float64."""
    u1, u2, u3, u4 = _uniforms24(q)
    a, b = np.sqrt(-2.0 * np.log(u1)), np.sqrt(-2.0 * np.log(u3))
    tp = 2.0 * np.pi
    return np.stack([a * np.cos(tp * u2), a * np.sin(tp * u2), b * np.cos(tp * u4), b * np.sin(tp * u4)], -1)


def box_muller_radius(q):
    """The Box–Muller radii (a, a, b, b) of each normal: the scale of its rounding error."""
    u1, _, u3, _ = _uniforms24(q)
    a, b = np.sqrt(-2.0 * np.log(u1)), np.sqrt(-2.0 * np.log(u3))
    return np.stack([a, a, b, b], -1)


def action_normals(seed, env, tick):
    """The TanhGauss noise eps [n, 4] (float64) env `env` draws at counter `tick` (stream 0)."""
    return box_muller(draw_words(seed, env, tick, 0))


def _uni(words, lo, hi):
    u = words.astype(np.float64) * 2.3283064365386963e-10
    return (np.float64(F32(lo)) + (np.float64(F32(hi)) - np.float64(F32(lo))) * u).astype(F32)


# the reset boxes of csrc/reset_draw.h (half-widths of the symmetric boxes)
_BOX = {"DuctedFan": (6, 0.5), "TwoLink": (4, 0.5), "SingleTrackCar": (7, 0.5)}
_PENDULUM_LO = (F32(-np.pi), F32(-10.0))
_PENDULUM_HI = (F32(np.pi), F32(10.0))


def quad_rotation(rv):
    """scipy Rotation.from_rotvec(rv).as_matrix() (QuadTracking.py:177-182) in float64, rows [n, 9]."""
    th = np.linalg.norm(rv, axis=1)
    safe = np.where(th > 0, th, 1.0)
    k = rv / safe[:, None]
    c, s = np.cos(th), np.sin(th)
    K = np.zeros((rv.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 2] = -k[:, 2], k[:, 1], -k[:, 0]
    K = K - np.transpose(K, (0, 2, 1))
    R = np.eye(3)[None] + s[:, None, None] * K + (1.0 - c)[:, None, None] * np.matmul(K, K)
    return R.reshape(-1, 9)


def reset_draw(name, seed, env, tick):
    """The reset state [n, reset_dim] env `env` draws at counter `tick` (ResetDraw<Env>::draw).
    float32; bit-exact with the kernels except QuadTracking's rotation block (columns 6..14,
    float64 here, float32 quaternion arithmetic on the device)."""
    env = np.asarray(env)
    n = env.shape[0]
    if name in ("VanderPol", "Pendulum"):
        q = draw_words(seed, env, tick, 1)
        lo, hi = ((-5.0, -5.0), (5.0, 5.0)) if name == "VanderPol" else (_PENDULUM_LO, _PENDULUM_HI)
        return np.stack([_uni(q[:, 0], lo[0], hi[0]), _uni(q[:, 1], lo[1], hi[1])], -1)
    if name in _BOX:
        N, half = _BOX[name]
        out = np.empty((n, N), F32)
        for i in range(0, N, 4):
            q = draw_words(seed, env, tick, 1 + i // 4)
            for j in range(min(4, N - i)):
                out[:, i + j] = _uni(q[:, j], -F32(half), F32(half))
        return out
    if name == "QuadTracking":
        q = np.concatenate([draw_words(seed, env, tick, s) for s in (1, 2, 3)], -1)
        out = np.empty((n, 18), F32)
        for i in range(6):
            out[:, i] = _uni(q[:, i], F32(-0.01), F32(0.01))
        for i in range(3):
            out[:, 15 + i] = _uni(q[:, 6 + i], F32(-0.01), F32(0.01))
        nz = box_muller(draw_words(seed, env, tick, 4))[:, :3]
        out[:, 6:15] = quad_rotation(nz * np.float64(F32(0.01))).astype(F32)
        return out
    raise ValueError(name)


def tanh_gauss_sample(logits, eps, low, high, log_std_lo=-20.0, log_std_hi=1.0, noise=0.0):
    """TanhGaussDistribution.sample (act_distribution_cls.py:45-57) of StochaPolicy's raw head
    [mean | log_std] (mlp.py:132-136: std = exp(clamp(log_std, lo, hi))) with the noise eps, plus
    the sampler's exploration noise and clip (base.py:136-143).
    logits [n, 2A] float32, eps [n, >= A] float64 -> (action float64 [n, A], logp float64 [n]).
    z = mean + std eps is rounded to float32 (the reference's float32 sample tensor); the rest is
    float64, so the result is the exact value of the reference's formula on that sample."""
    lg = np.asarray(logits, F32)
    A = lg.shape[1] // 2
    mu = lg[:, :A].astype(np.float64)
    c = np.clip(lg[:, A:], F32(log_std_lo), F32(log_std_hi)).astype(np.float64)
    sd = np.exp(c).astype(F32).astype(np.float64)
    e = np.asarray(eps, np.float64)[:, :A]
    z = (mu + (sd * e).astype(F32)).astype(F32).astype(np.float64)
    th = np.tanh(z)
    lg_n = (-((z - mu) ** 2) / (2.0 * sd * sd) - c - LOG_SQRT_2PI).sum(1)
    # ONE_PLUS_EPS - tanh^2 without cancellation: (ONE_PLUS_EPS - 1) + 4 t / (1 + t)^2, t = exp(-2|z|)
    t = np.exp(-2.0 * np.abs(z))
    lj = np.log((ONE_PLUS_EPS - 1.0) + 4.0 * t / (1.0 + t) ** 2).sum(1)
    lo, hi = np.asarray(low, np.float64), np.asarray(high, np.float64)
    half = (hi - lo) / 2.0
    act = half * th + (hi + lo) / 2.0 + noise
    act = np.clip(act, lo, hi)
    return act, lg_n - lj - np.log(half).sum()
