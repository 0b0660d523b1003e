"""CPU ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package).

NumPy restatement of the six RL/env step functions of the reference, vectorised over a batch
of envs but with the exact per-element dtype flow the reference has under NumPy 2 (NEP 50):
Python-float constants are weak (a float32 op with the constant rounded to float32), float32
arrays meeting float64 arrays promote, and `f32 += f64` rounds once. Each function cites the
reference lines it restates. Pinned against fixtures generated from the reference's own env
methods (tools/gen_golden.py -> tests/golden/env_*.npz).
"""
from __future__ import annotations

import numpy as np

from oracle.libm import powf2

F32 = np.float32
F64 = np.float64
MAX_STEP = 1000  # every env: truncated = current_step >= 1000

ENV_IDS = {
    "VanderPol": 0,
    "Pendulum": 1,
    "DuctedFan": 2,
    "TwoLink": 3,
    "SingleTrackCar": 4,
    "QuadTracking": 5,
}


def _box(lo, hi):
    return np.asarray(lo, dtype=F64).astype(F32), np.asarray(hi, dtype=F64).astype(F32)


def _regulation_reward(s, u, Q, R):
    """-(sum(Q*obs^2) + sum(R*u^2)) + 1[all |obs| <= 0.01]  (e.g. VanderPol.py:108-115)."""
    obs_cost = (Q * s ** 2).sum(axis=1)
    ctl_cost = (R * u ** 2).sum(axis=1)
    r = -(obs_cost + ctl_cost)
    near = np.all(np.abs(s) <= 0.01, axis=1)
    return np.where(near, r + F32(1), r).astype(F32)


class VanderPol:
    """RL/env/VanderPol.py:23-129."""
    obs_dim, act_dim, state_dim, K = 2, 1, 2, 5
    obs_low, obs_high = _box([-10.0, -10.0], [10.0, 10.0])
    act_low, act_high = _box([-5.0], [5.0])
    Q = np.array([2.0, 1.0], dtype=F32)
    R = np.array([0.1], dtype=F32)

    @classmethod
    def reset_draw(cls, rng, n):  # :79-82
        return rng.uniform(-5.0 * np.ones(2, F32), 5.0 * np.ones(2, F32), size=(n, 2)).astype(F32)

    @classmethod
    def step(cls, s, u):
        s = s.copy()
        for _ in range(cls.K):  # :103-105
            x, xd = s[:, 0], s[:, 1]
            acc = 1.0 * (1 - powf2(x)) * xd - x + u[:, 0]  # scalar x**2 -> glibc powf
            s += np.stack([xd, acc], axis=1) * 0.01
        return s, s.copy(), _regulation_reward(s, u, cls.Q, cls.R)


class Pendulum:
    """RL/env/Pendulum.py:22-137."""
    obs_dim, act_dim, state_dim, K = 2, 1, 2, 5
    obs_low, obs_high = _box([-np.pi, -10.0], [np.pi, 10.0])
    act_low, act_high = _box([-5], [5])
    Q = np.array([2.0, 1.0], dtype=F32)
    R = np.array([0.1], dtype=F32)

    @classmethod
    def reset_draw(cls, rng, n):  # :83-86
        return rng.uniform(cls.obs_low, cls.obs_high, size=(n, 2)).astype(F32)

    @classmethod
    def step(cls, s, u):
        s = s.copy()
        m, g, L, b = 0.15, 9.81, 0.5, 0.1
        for _ in range(cls.K):  # :110-112, dynamics :102
            th, thd = s[:, 0], s[:, 1]
            acc = (m * g * L * np.sin(th) - b * thd + u[:, 0]) / (m * L ** 2)
            s += np.stack([thd, acc], axis=1) * 0.01
        return s, s.copy(), _regulation_reward(s, u, cls.Q, cls.R)


class DuctedFan:
    """RL/env/DuctedFan.py:24-147."""
    obs_dim, act_dim, state_dim, K = 6, 2, 6, 5
    obs_low, obs_high = _box([-5.0, -5.0, -np.pi / 2, -5.0, -5.0, -5.0], [5.0, 5.0, np.pi / 2, 5.0, 5.0, 5.0])
    act_low, act_high = _box([-5.0, -5.0], [5.0, 5.0])
    Q = np.array([2.0, 2.0, 2.0, 1.0, 1.0, 1.0], dtype=F32)
    R = np.array([0.1, 0.1], dtype=F32)

    @classmethod
    def reset_draw(cls, rng, n):  # :89-92
        return rng.uniform(-0.5 * np.ones(6, F32), 0.5 * np.ones(6, F32), size=(n, 6)).astype(F32)

    @classmethod
    def step(cls, s, u):
        s = s.copy()
        m, g, r, d, J = 8.5, 9.81, 0.26, 0.95, 0.048
        u1, u2 = u[:, 0], u[:, 1]
        for _ in range(cls.K):  # :107-109
            th, vx, vy, om = s[:, 2], s[:, 3], s[:, 4], s[:, 5]
            ax = (-m * g * np.sin(th) - d * vx + u1 * np.cos(th) - u2 * np.sin(th)) / m
            ay = (m * g * (np.cos(th) - 1) - d * vy + u1 * np.sin(th) + u2 * np.cos(th)) / m
            aw = (r * u1) / J
            s += np.stack([vx, vy, om, ax, ay, aw], axis=1) * 0.01
        return s, s.copy(), _regulation_reward(s, u, cls.Q, cls.R)


class TwoLink:
    """RL/env/TwoLink.py:22-177 — float64 M, C; float32 G; LAPACK solve."""
    obs_dim, act_dim, state_dim, K = 4, 2, 4, 5
    obs_low, obs_high = _box([-np.pi / 2, -np.pi / 2, -20.0, -20.0], [np.pi / 2, np.pi / 2, 20.0, 20.0])
    act_low, act_high = _box([-20.0, -20.0], [20.0, 20.0])
    Q = np.array([2.0, 2.0, 1.0, 1.0], dtype=F32)
    R = np.array([0.1, 0.1], dtype=F32)

    @classmethod
    def reset_draw(cls, rng, n):
        return rng.uniform(-0.5 * np.ones(4, F32), 0.5 * np.ones(4, F32), size=(n, 4)).astype(F32)

    @staticmethod
    def deriv(s, u):
        l1 = l2 = m1 = m2 = 1.0
        lc1 = lc2 = 0.5
        I1 = I2 = (1 / 12) * 1.0 * 1.0 ** 2
        g = 9.81
        q1, q2, dq1, dq2 = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
        n = s.shape[0]
        c2 = np.cos(q2)  # mass matrix :100-107
        M11 = I1 + I2 + m1 * lc1 ** 2 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * c2)
        M12 = I2 + m2 * (lc2 ** 2 + l1 * lc2 * c2)
        M = np.empty((n, 2, 2), dtype=F64)
        M[:, 0, 0], M[:, 0, 1], M[:, 1, 0], M[:, 1, 1] = M11, M12, M12, I2 + m2 * lc2 ** 2
        s2 = np.sin(q2)  # coriolis :109-119
        h = -m2 * l1 * lc2 * s2
        C = np.zeros((n, 2, 2), dtype=F64)
        C[:, 0, 0], C[:, 0, 1], C[:, 1, 0] = h * dq2, h * dq2 + h * dq1, -h * dq1
        G1 = -(m1 * lc1 + m2 * l1) * g * np.sin(q1) - m2 * lc2 * g * np.sin(q1 + q2)  # :121-129
        G2 = -m2 * lc2 * g * np.sin(q1 + q2)
        G = np.stack([G1, G2], axis=1)
        dq = s[:, 2:]
        rhs = u - np.einsum("nij,nj->ni", C, dq.astype(F64)) - G
        ddq = np.linalg.solve(M, rhs[..., None])[..., 0]
        return np.concatenate([dq, ddq], axis=1)

    @classmethod
    def step(cls, s, u):
        s = s.copy()
        for _ in range(cls.K):
            s += cls.deriv(s, u) * 0.01
        return s, s.copy(), _regulation_reward(s, u, cls.Q, cls.R)


class SingleTrackCar:
    """RL/env/SingleTrackCar.py:41-320 — f(x) + g(x) u in float64 containers."""
    obs_dim, act_dim, state_dim, K = 7, 2, 7, 5
    obs_low, obs_high = _box([-1.0, -1.0, -1.066, -1.0, -np.pi / 2, -np.pi / 2, -np.pi / 3],
                             [1.0, 1.0, 1.066, 1.0, np.pi / 2, np.pi / 2, np.pi / 3])
    act_low, act_high = _box([-5.0, -5.0], [5.0, 5.0])
    Q = np.array([2.0, 2.0, 1.0, 1.0, 1.0, 1.0, 1.0], dtype=F32)
    R = np.array([0.1, 0.1], dtype=F32)
    lf = 0.3048 * 3.793293
    lr = 0.3048 * 4.667707
    h = 0.3048 * 2.01355
    m = 4.4482216152605 / 0.3048 * (74.91452)
    Iz = 4.4482216152605 * 0.3048 * (1321.416)
    mu = 0.1 * 1.0489
    CS = -(-21.92) / 1.0489
    g = 9.81

    @classmethod
    def reset_draw(cls, rng, n):
        return rng.uniform(-0.5 * np.ones(7, F32), 0.5 * np.ones(7, F32), size=(n, 7)).astype(F32)

    @classmethod
    def deriv(cls, x, u):
        lf, lr, h, m, Iz, mu, CS, g = cls.lf, cls.lr, cls.h, cls.m, cls.Iz, cls.mu, cls.CS, cls.g
        sxe, sye, delta, ve, pe, ped, beta = (x[:, i] for i in range(7))
        n = x.shape[0]
        v = ve + 1.0
        psid = ped + 0.0
        f = np.zeros((n, 7), dtype=F64)
        G = np.zeros((n, 7, 2), dtype=F64)
        f[:, 0] = v * np.cos(pe + beta) - 1.0 + 0.0 * sye  # :165-166
        f[:, 1] = v * np.sin(pe + beta) - 0.0 * sxe
        f[:, 3] = -0.0
        dyn = ~(np.abs(v) < 0.1)
        with np.errstate(all="ignore"):
            # dynamic model :178-196, :243-256
            fd5 = (-(mu * m / (v * Iz * (lr + lf))) * (lf ** 2 * CS * g * lr + lr ** 2 * CS * g * lf) * psid
                   + (mu * m / (Iz * (lr + lf))) * (lr * CS * g * lf - lf * CS * g * lr) * beta
                   + (mu * m / (Iz * (lr + lf))) * (lf * CS * g * lr) * delta)
            fd6 = (((mu / (powf2(v) * (lr + lf))) * (CS * g * lf * lr - CS * g * lr * lf) - 1) * psid
                   - (mu / (v * (lr + lf))) * (CS * g * lf + CS * g * lr) * beta
                   + mu / (v * (lr + lf)) * (CS * g * lr) * delta)
            gd5 = (-(mu * m / (v * Iz * (lr + lf))) * (-(lf ** 2) * CS * h + lr ** 2 * CS * h) * psid
                   + (mu * m / (Iz * (lr + lf))) * (lr * CS * h + lf * CS * h) * beta
                   - (mu * m / (Iz * (lr + lf))) * (lf * CS * h) * delta)
            gd6 = ((mu / (powf2(v) * (lr + lf))) * (CS * h * lr + CS * h * lf) * psid
                   - (mu / (v * (lr + lf))) * (CS * h - CS * h) * beta
                   - mu / (v * (lr + lf)) * CS * h * delta)
            # kinematic model :199-204, :259-277
            lwb = lf + lr
            fk4 = v * np.cos(beta) / lwb * np.tan(delta) - 0.0
            bdot = 1 / (1 + powf2(np.tan(delta) * lr / lwb)) * lr / (lwb * powf2(np.cos(delta)))
            gk51 = 1 / lwb * (np.cos(beta) * np.tan(delta))
            gk50 = 1 / lwb * (-v * np.sin(beta) * np.tan(delta) * bdot + v * np.cos(beta) / powf2(np.cos(delta)))
        f[:, 4] = np.where(dyn, ped, fk4)
        f[:, 5] = np.where(dyn, fd5, 0.0)
        f[:, 6] = np.where(dyn, fd6, 0.0)
        G[:, 2, 0] = np.where(dyn, 1.0, 0.0)
        G[:, 3, 1] = np.where(dyn, 1.0, 0.0)
        G[:, 5, 1] = np.where(dyn, gd5, gk51)
        G[:, 5, 0] = np.where(dyn, 0.0, gk50)
        G[:, 6, 1] = np.where(dyn, gd6, 0.0)
        G[:, 6, 0] = np.where(dyn, 0.0, bdot)
        return f + np.einsum("nij,nj->ni", G, u.astype(F64))

    @classmethod
    def step(cls, s, u):
        s = s.copy()
        for _ in range(cls.K):
            s += cls.deriv(s, u) * 0.01
        return s, s.copy(), _regulation_reward(s, u, cls.Q, cls.R)


# ------------------------------------------------------------------------------ QuadTracking
def _rownorm(v):
    """np.linalg.norm per row (BLAS ddot: sqrt(fma(z,z,fma(y,y,x*x))), bit-exact to the
    reference's per-env call at QuadTracking.py:131,137)."""
    return np.array([np.linalg.norm(r) for r in v], dtype=F64)


QUAD_ROWS = MAX_STEP + 1


def quad_time_table(rows=QUAD_ROWS):
    """current_time accumulation (QuadTracking.py:229) and the analytic trajectory (:29-36)."""
    t = np.zeros(rows, F64)
    for k in range(1, rows):
        t[k] = t[k - 1] + 0.01 * 4
    return t


class QuadTracking:
    """RL/env/QuadTracking.py:20-424. state = [x(3) v(3) R(9 row-major) W(3)] f32,
    xstate = Rd_last (9, float64), steps since reset index the time table."""
    obs_dim, act_dim, state_dim, xstate_dim, K = 12, 4, 18, 9, 4
    obs_low, obs_high = _box(-np.full(12, 10.0), np.full(12, 10.0))
    m = 4.34
    J = np.diag([0.0820, 0.0845, 0.1377])
    kx, kv = 69.44, 24.304
    g = np.array([0, 0, 9.8])
    act_low = np.array([0.0 * (4.34 * g[2]), -10.0, -10.0, -10.0], dtype=F32)
    act_high = np.array([2.0 * (4.34 * g[2]), 10.0, 10.0, 10.0], dtype=F32)
    R_act = np.array([0.0001, 0.01, 0.01, 0.01], dtype=F32)
    T = quad_time_table()

    @classmethod
    def reset_draw(cls, rng, n, gauss=None):
        """QuadTracking.py:169-186: x, v, W ~ U(+-0.01) via the env RNG, rotvec ~ N(0, 0.01^2)
        via the global np.random + scipy Rotation.from_rotvec."""
        from scipy.spatial.transform import Rotation
        lo, hi = -0.01 * np.ones(3, F32), 0.01 * np.ones(3, F32)
        x = rng.uniform(lo, hi, size=(n, 3)).astype(F32)
        v = rng.uniform(lo, hi, size=(n, 3)).astype(F32)
        rv = (gauss(n) if gauss is not None else np.random.randn(n, 3)) * 0.01
        R = Rotation.from_rotvec(rv).as_matrix().astype(F32).reshape(n, 9)
        W = rng.uniform(lo, hi, size=(n, 3)).astype(F32)
        return np.concatenate([x, v, R, W], axis=1)

    @classmethod
    def traj(cls, t):
        t = np.asarray(t, F64)
        xd = np.stack([0.4 * t, 0.4 * np.sin(t), 0.6 * np.cos(t)], -1)
        b1 = np.stack([np.cos(t), np.sin(t), np.zeros_like(t)], -1)
        vd = np.stack([np.full_like(t, 0.4), 0.4 * np.cos(t), -0.6 * np.sin(t)], -1).astype(F32)
        ad = np.stack([np.zeros_like(t), -0.4 * np.sin(t), -0.6 * np.cos(t)], -1).astype(F32)
        return xd, vd, ad, b1

    @classmethod
    def desired(cls, x, v, kidx, Rd_last):
        """_get_desired_states (:122-149) at t = T[kidx]; Rd_last None -> Omega_d = 0."""
        t = cls.T[kidx]
        xd, vd, ad, b1 = cls.traj(t)
        ex = (x - xd).astype(F32)
        ev = (v - vd).astype(F32)
        fd = -(-cls.kx * ex - cls.kv * ev - cls.m * cls.g + cls.m * ad)
        b3 = fd / _rownorm(fd)[:, None]
        c = np.cross(b3, b1)
        b2 = c / _rownorm(c)[:, None]
        b1n = np.cross(b2, b3)
        Rd = np.stack([b1n, b2, b3], axis=2)  # columns
        if Rd_last is None:
            Od = np.zeros((x.shape[0], 3), F64)
        else:
            dt = t - cls.T[kidx - 1]
            dt = np.where(dt < 1e-6, 1e-6, dt)
            Rdot = ((Rd - Rd_last) / dt[:, None, None]).astype(F32)
            M = np.matmul(np.transpose(Rd, (0, 2, 1)), Rdot.astype(F64))
            Od = np.stack([M[:, 2, 1], M[:, 0, 2], M[:, 1, 0]], 1).astype(F32)
        return ex, ev, Rd, Od

    @classmethod
    def errors(cls, R, W, ex, ev, Rd, Od):
        """cal_eR / cal_eOmega (:328-341)."""
        R64 = R.astype(F64)
        RdT = np.transpose(Rd, (0, 2, 1))
        Dm = np.matmul(RdT, R64) - np.matmul(np.transpose(R64, (0, 2, 1)), Rd)
        eR = np.stack([Dm[:, 2, 1], Dm[:, 0, 2], Dm[:, 1, 0]], 1).astype(F32) * 0.5
        P = np.matmul(np.transpose(R64, (0, 2, 1)), Rd)
        eW = (W - np.einsum("nij,nj->ni", P, Od.astype(F64))).astype(F32)
        return np.concatenate([ex, ev, eR.astype(F32), eW], axis=1).astype(F32)

    @classmethod
    def reset_from(cls, rs, kidx=None):
        n = rs.shape[0]
        x, v, R, W = rs[:, 0:3], rs[:, 3:6], rs[:, 6:15].reshape(n, 3, 3), rs[:, 15:18]
        k0 = np.zeros(n, np.int64)
        ex, ev, Rd, Od = cls.desired(x, v, k0, None)
        obs = cls.errors(R, W, ex, ev, Rd, Od)
        return rs.astype(F32).copy(), Rd.reshape(n, 9), obs

    @staticmethod
    def polar(R, f64=False):
        """NormalizeOrientMatrix (QuadTracking.py:308-315). f64=True: the same factorisation
        from a float64 SVD of the float32 input (the kernel's arithmetic: an f64 polar factor
        rounded once); used by the tests to separate the reference's float32-SVD rounding from
        kernel error (tests/golden/quad_polar64.npz pins this variant against the reference run
        with the same substitution)."""
        U, _, Vh = np.linalg.svd(R.astype(F64) if f64 else R)
        out = np.matmul(U, Vh)
        neg = np.linalg.det(out) < 0
        if np.any(neg):
            U2 = U[neg].copy()
            U2[:, :, -1] *= -1
            out[neg] = np.matmul(U2, Vh[neg])
        return out.astype(F32)

    @classmethod
    def step(cls, s, u, xs, k, polar64=False):
        """env.step (:205-285) for a batch; k = steps since reset before the step."""
        n = s.shape[0]
        x = s[:, 0:3].copy()
        v = s[:, 3:6].copy()
        R = s[:, 6:15].reshape(n, 3, 3).copy()
        W = s[:, 15:18].copy()
        force = u[:, 0]
        M = u[:, 1:]
        Jinv = np.linalg.inv(cls.J)
        for _ in range(cls.K):
            dx = v
            dv = cls.g - (force[:, None] * R[:, :, 2]) / cls.m
            Wx = np.zeros((n, 3, 3), F32)
            Wx[:, 0, 1], Wx[:, 0, 2] = -W[:, 2], W[:, 1]
            Wx[:, 1, 0], Wx[:, 1, 2] = W[:, 2], -W[:, 0]
            Wx[:, 2, 0], Wx[:, 2, 1] = -W[:, 1], W[:, 0]
            dR = np.matmul(R, Wx)
            JW = np.einsum("ij,nj->ni", cls.J, W.astype(F64))
            dW = np.einsum("ij,nj->ni", Jinv, M - np.cross(W.astype(F64), JW))
            x += dx * 0.01
            v += dv * 0.01
            R += dR * 0.01
            W += dW * 0.01
            R = cls.polar(R, polar64)
        k1 = k + 1
        Rd_last = xs.reshape(n, 3, 3)
        ex, ev, Rd, Od = cls.desired(x, v, k1, Rd_last)
        obs = cls.errors(R, W, ex, ev, Rd, Od)
        rew = -((obs[:, 0:3] ** 2).sum(1) + (obs[:, 3:6] ** 2).sum(1) + (obs[:, 6:9] ** 2).sum(1)
                + (obs[:, 9:12] ** 2).sum(1) + (cls.R_act * u ** 2).sum(1))
        dist = np.max(np.abs(obs), axis=1)
        bonus = 10.0 * (1 - dist / F32(0.1))
        rew = np.where(dist <= 0.1, rew + bonus.astype(F32), rew).astype(F32)
        s2 = np.concatenate([x, v, R.reshape(n, 9), W], axis=1).astype(F32)
        return s2, Rd.reshape(n, 9).copy(), obs, rew


ENVS = {
    "VanderPol": VanderPol,
    "Pendulum": Pendulum,
    "DuctedFan": DuctedFan,
    "TwoLink": TwoLink,
    "SingleTrackCar": SingleTrackCar,
    "QuadTracking": QuadTracking,
}


def env_step(name, state, act, xstate=None, steps=None, polar64=False):
    """One env.step for a batch: returns (state', xstate', obs, reward f32, terminated, truncated).
    steps = steps since reset before the step; polar64: QuadTracking's polar factor from a
    float64 SVD (QuadTracking.polar)."""
    cls = ENVS[name]
    n = state.shape[0]
    steps = np.zeros(n, np.int64) if steps is None else np.asarray(steps, np.int64)
    if name == "QuadTracking":
        s2, xs2, obs, rew = cls.step(state, act, xstate, steps, polar64)
    else:
        s2, obs, rew = cls.step(state, act)
        xs2 = None
    term = np.any((obs < cls.obs_low) | (obs > cls.obs_high), axis=1)
    trunc = (steps + 1) >= MAX_STEP
    return s2, xs2, obs, rew, term, trunc


def env_reset_from(name, rs):
    """Initial (state, xstate, obs) from a drawn reset state."""
    if name == "QuadTracking":
        return QuadTracking.reset_from(rs)
    rs = rs.astype(F32).copy()
    return rs, None, rs.copy()
