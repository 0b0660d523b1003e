"""CPU ORACLE — test infrastructure only.

Vectorised restatement of glibc 2.35 powf(x, 2.0f) (sysdeps/ieee754/flt-32/e_powf.c, the ARM
optimized-routines algorithm), which is what `np.float32_scalar ** 2` evaluates: the reference
squares float32 SCALARS in VanderPol._dynamics (VanderPol.py:95) and SingleTrackCar._f/_g
(SingleTrackCar.py:190, 262-274). glibc's powf is not correctly rounded (~0.09% of inputs differ
from x*x), so a bit-exact oracle needs the same algorithm. Checked against libm through ctypes
in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import numpy as np

_LOG_INVC = np.array([float.fromhex(h) for h in (
    "0x1.661ec79f8f3bep+0", "0x1.571ed4aaf883dp+0", "0x1.49539f0f010bp+0", "0x1.3c995b0b80385p+0",
    "0x1.30d190c8864a5p+0", "0x1.25e227b0b8eap+0", "0x1.1bb4a4a1a343fp+0", "0x1.12358f08ae5bap+0",
    "0x1.0953f419900a7p+0", "0x1p+0", "0x1.e608cfd9a47acp-1", "0x1.ca4b31f026aap-1",
    "0x1.b2036576afce6p-1", "0x1.9c2d163a1aa2dp-1", "0x1.886e6037841edp-1", "0x1.767dcf5534862p-1")])
_LOG_C = np.array([float.fromhex(h) for h in (
    "-0x1.efec65b963019p-2", "-0x1.b0b6832d4fca4p-2", "-0x1.7418b0a1fb77bp-2", "-0x1.39de91a6dcf7bp-2",
    "-0x1.01d9bf3f2b631p-2", "-0x1.97c1d1b3b7afp-3", "-0x1.2f9e393af3c9fp-3", "-0x1.960cbbf788d5cp-4",
    "-0x1.a6f9db6475fcep-5", "0x0p+0", "0x1.338ca9f24f53dp-4", "0x1.476a9543891bap-3",
    "0x1.e840b4ac4e4d2p-3", "0x1.40645f0c6651cp-2", "0x1.88e9c2c1b9ff8p-2", "0x1.ce0a44eb17bccp-2")])
# tab[i] = asuint64(2^(i/32)) - (i << 47)
_EXP_T = np.array([
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
    0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
    0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
    0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
    0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
    0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
    0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540], dtype=np.uint64)
_A = [float.fromhex(h) for h in ("0x1.27616c9496e0bp-2", "-0x1.71969a075c67ap-2", "0x1.ec70a6ca7baddp-2",
                                  "-0x1.7154748bef6c8p-1", "0x1.71547652ab82bp0")]
_C = [float.fromhex(h) for h in ("0x1.c6af84b912394p-5", "0x1.ebfce50fac4f3p-3", "0x1.62e42ff0c52d6p-1")]
_SHIFT = float.fromhex("0x1.8p+52") / 32


def powf2(x):
    """glibc powf(x, 2) for a float32 array (normal and subnormal finite inputs)."""
    x = np.asarray(x, np.float32)
    shape = x.shape
    x = x.reshape(-1)
    ix = x.view(np.uint32) & np.uint32(0x7FFFFFFF)
    out = (x * x).astype(np.float32)  # zero / inf / nan / huge paths
    sub = (ix < 0x00800000) & (ix != 0)
    if np.any(sub):
        v = (ix[sub].view(np.float32) * np.float32(2.0 ** 23)).view(np.uint32) & np.uint32(0x7FFFFFFF)
        ix = ix.copy()
        ix[sub] = v - np.uint32(23 << 23)
    ok = (ix != 0) & (ix < 0x7F800000)
    ixo = ix[ok]
    tmp = (ixo - np.uint32(0x3F330000)).astype(np.uint32)
    i = ((tmp >> np.uint32(19)) % np.uint32(16)).astype(np.int64)
    top = tmp & np.uint32(0xFF800000)
    iz = (ixo - top).astype(np.uint32)
    k = (top.view(np.int32) >> 23).astype(np.float64)
    z = iz.view(np.float32).astype(np.float64)
    r = z * _LOG_INVC[i] - 1.0
    y0 = _LOG_C[i] + k
    r2 = r * r
    y = _A[0] * r + _A[1]
    p = _A[2] * r + _A[3]
    r4 = r2 * r2
    q = _A[4] * r + y0
    q = p * r2 + q
    y = y * r4 + q
    ylogx = 2.0 * y
    big = ((ylogx.view(np.uint64) >> np.uint64(47)) & np.uint64(0xFFFF)) >= (np.float64(126.0).view(np.uint64) >> np.uint64(47))
    kd = ylogx + _SHIFT
    ki = kd.view(np.uint64)
    kd = kd - _SHIFT
    rr = ylogx - kd
    t = _EXP_T[(ki % np.uint64(32)).astype(np.int64)] + (ki << np.uint64(47))
    s = t.view(np.float64)
    zz = _C[0] * rr + _C[1]
    rr2 = rr * rr
    yy = _C[2] * rr + 1.0
    yy = zz * rr2 + yy
    yy = yy * s
    with np.errstate(over="ignore", under="ignore"):
        res = yy.astype(np.float32)
    # e_powf.c: only |x^2| overflow (-> inf) and ylogx <= -150 (-> 0) leave the exp2 path;
    # subnormal results in between come from exp2 (double rounding included)
    res[big & (ylogx > float.fromhex("0x1.fffffffd1d571p+6"))] = np.float32(np.inf)
    res[big & (ylogx <= -150.0)] = np.float32(0.0)
    out[ok] = res
    return out.reshape(shape)
