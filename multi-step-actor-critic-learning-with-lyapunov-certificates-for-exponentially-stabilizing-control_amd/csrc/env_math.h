// env_math.h — per-env physics of the six MSACL control environments, written once as
// __host__ __device__ functions so the same source runs inside the gfx950 rollout kernel
// and in the host-side check build used by the CPU test-suite.
//
// Precision flow mirrors the reference's NumPy-2 (NEP 50) dtype semantics exactly:
//   * a Python float constant times a float32 value is a float32 op with the constant
//     rounded to float32 (weak scalar);
//   * float32 arrays combined with float64 arrays promote to float64, and an in-place
//     `f32_array += f64_array` is evaluated in float64 and rounded once.
// No FMA contraction (see #pragma below) so every op rounds where NumPy rounds.
// float32 transcendentals use the f32 OCML/libm functions (NumPy's SIMD float32 sin/cos are
// not correctly rounded either; both are within ~1.5 ulp), float64 ones the f64 functions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#pragma clang fp contract(off)

#define MH_HD __host__ __device__ __forceinline__

namespace mh {

enum EnvId : int {
  ENV_VANDERPOL = 0,
  ENV_PENDULUM = 1,
  ENV_DUCTEDFAN = 2,
  ENV_TWOLINK = 3,
  ENV_SINGLETRACKCAR = 4,
  ENV_QUADTRACKING = 5,
  ENV_COUNT = 6
};

constexpr int MAX_STEP = 1000;  // every env: truncated = current_step >= 1000

// ---------------------------------------------------------------- f32 helpers
// NumPy float32 sin/cos/tan (SIMD, not correctly rounded either): the f32 libm/OCML versions
// stay within 1-2 ulp, far inside the 1e-5 parity tolerance, at a fraction of the f64 cost.
MH_HD float sin32(float x) { return sinf(x); }
MH_HD float cos32(float x) { return cosf(x); }
MH_HD float tan32(float x) { return tanf(x); }
// sin and cos of one argument through one shared range reduction (OCML / glibc sincosf: the same
// reduction and polynomials as sinf and cosf, so the same values)
MH_HD void sincos32(float x, float* s, float* c) { sincosf(x, s, c); }
// a / b for the f32 sites whose reference division is not a bit-exact parity point: on the
// device the hardware reciprocal and one FMA residual correction (within 1 ulp, correctly rounded
// almost always; ~5 instructions instead of the IEEE division's scale / fixup sequence), on the
// host the division itself
MH_HD float div32(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float r = __builtin_amdgcn_rcpf(b);
  const float q = a * r;
  return fmaf(fmaf(-b, q, a), r, q);
#else
  return a / b;
#endif
}
// 1.0 / x in float64: on the device the hardware reciprocal refined by two Newton steps (within
// ~1 ulp), on the host the division
MH_HD double rcp64(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  double d = __builtin_amdgcn_rcp(x);
  d = d * fma(-x, d, 2.0);
  d = d * fma(-x, d, 2.0);
  return d;
#else
  return 1.0 / x;
#endif
}

// `s ** 2` on a NumPy float32 SCALAR calls the C library's powf (glibc 2.35 e_powf.c, the
// ARM optimized-routines algorithm: 16-entry log2 table + degree-5 poly, 32-entry exp2 table +
// degree-3 poly, all in double), which differs from s*s in ~0.09% of inputs. Arrays use
// s*s. The reference squares scalars in VanderPol._dynamics and SingleTrackCar._f/_g, so those
// sites use this bit-exact restatement (verified against libm on 9.3M random floats).
MH_HD double mh_asdouble(uint64_t u) {
  union { uint64_t u; double d; } c;
  c.u = u;
  return c.d;
}
MH_HD uint64_t mh_asuint64(double d) {
  union { uint64_t u; double d; } c;
  c.d = d;
  return c.u;
}
MH_HD float mh_asfloat(uint32_t u) {
  union { uint32_t u; float f; } c;
  c.u = u;
  return c.f;
}
MH_HD uint32_t mh_asuint(float f) {
  union { uint32_t u; float f; } c;
  c.f = f;
  return c.u;
}
// glibc's double-precision result before its final rounding to float.
MH_HD double powf2_core(float x) {
  constexpr double LOG_INVC[16] = {
      0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
      0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
      0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
      0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
  constexpr double LOG_C[16] = {
      -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
      -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3,  -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
      -0x1.a6f9db6475fcep-5, 0x0p+0,                0x1.338ca9f24f53dp-4,  0x1.476a9543891bap-3,
      0x1.e840b4ac4e4d2p-3,  0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2,  0x1.ce0a44eb17bccp-2};
  constexpr uint64_t EXP_T[32] = {
      0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
      0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
      0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
      0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
      0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
      0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
      0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
      0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
  constexpr double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                   A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp0;
  constexpr double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
  uint32_t ix = mh_asuint(x) & 0x7fffffffu;  // y = 2 is even: sign drops
  if (ix == 0u) return 0.0;
  if (ix >= 0x7f800000u) return (double)(x * x);
  if (ix < 0x00800000u) {  // subnormal: normalise
    ix = mh_asuint(mh_asfloat(ix) * 0x1p23f) & 0x7fffffffu;
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16u);
  const uint32_t top = tmp & 0xff800000u;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double z = (double)mh_asfloat(iz);
  const double r = z * LOG_INVC[i] - 1.0;
  const double y0 = LOG_C[i] + (double)k;
  const double r2 = r * r;
  double y = A0 * r + A1;
  const double p = A2 * r + A3;
  const double r4 = r2 * r2;
  double q = A4 * r + y0;
  q = p * r2 + q;
  y = y * r4 + q;
  const double ylogx = 2.0 * y;
  if (((mh_asuint64(ylogx) >> 47) & 0xffffu) >= (mh_asuint64(126.0) >> 47)) {  // |2 log2 x| >= 126
    if (ylogx > 0x1.fffffffd1d571p+6) return (double)INFINITY;  // __math_oflowf
    if (ylogx <= -150.0) return 0.0;                              // __math_uflowf
  }
  const double SHIFT = 0x1.8p+52 / 32;
  double kd = ylogx + SHIFT;
  const uint64_t ki = mh_asuint64(kd);
  kd -= SHIFT;
  const double rr = ylogx - kd;
  uint64_t t = EXP_T[ki % 32];
  t += ki << (52 - 5);
  const double s = mh_asdouble(t);
  const double zz = C0 * rr + C1;
  const double rr2 = rr * rr;
  double yy = C2 * rr + 1.0;
  yy = zz * rr2 + yy;
  yy = yy * s;
  return yy;
}

// powf(x, 2) bit-exactly, cheaply: glibc's double result differs from the exact square x*x
// (exact in double) by at most POWF2_MAX_ERR float-ulps over ALL 2^32 inputs (exhaustive scan,
// tools/powf2_exhaustive.cpp), so whenever the exact square lies farther than that from a
// float rounding midpoint, glibc returns the correctly rounded square. Only the rare
// near-midpoint inputs (and zero / subnormal / overflowing squares, powers of two) take the
// table path. The exhaustive scan also checks this function against libm powf for every input.
constexpr double POWF2_MAX_ERR = 0x1p-8;  // guard > measured maximum 1.69e-3 ulp (tools/powf2_exhaustive.cpp)
MH_HD float powf2(float x) {
  const double xd = (double)x;
  const double p = xd * xd;  // exact: 24 x 24 significant bits
  const float r = (float)p;
  const uint32_t rb = mh_asuint(r);
  const uint32_t ex = (rb >> 23) & 0xffu, man = rb & 0x7fffffu;
  if (ex > 23u && ex < 0xfeu && man != 0u) {
    const double ulp = mh_asdouble((uint64_t)(ex - 23u - 127u + 1023u) << 52);
    const double d = fabs(p - (double)r);  // exact, <= ulp / 2
    if (0.5 * ulp - d > POWF2_MAX_ERR * ulp) return r;
  }
  return (float)powf2_core(x);
}

// NumPy float32 add.reduce order (pairwise_sum: <8 sequential from -0.0, else 8 lanes).
template <int N>
MH_HD float np_sum(const float* a) {
  if constexpr (N < 8) {
    float r = -0.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) r = r + a[i];
    return r;
  } else {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
#pragma unroll
    for (; i < N - (N % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
    }
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (; i < N; ++i) res = res + a[i];
    return res;
  }
}

// f32 state updated by a float64 derivative: `obs += deriv * dt` with deriv float64.
MH_HD float upd64(float s, double d, double dt) { return (float)((double)s + d * dt); }

// Shared quadratic reward of the five regulation envs (e.g. VanderPol.py:108-115):
// reward = -(sum(Q*obs^2) + sum(R*u^2)) + 1[all |obs| <= 0.01]
template <int D, int A>
MH_HD float quad_reward(const float* s, const float* Q, const float* u, const float* R) {
  float a[D], b[A];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    float x = s[i];
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(x));  // one scalar per square: no v_pk_mul_f32 pairing (tests/test_build_isa.py)
#endif
    a[i] = Q[i] * (x * x);
  }
#pragma unroll
  for (int i = 0; i < A; ++i) {
    float x = u[i];
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(x));
#endif
    b[i] = R[i] * (x * x);
  }
  float cost = np_sum<D>(a) + np_sum<A>(b);
  float r = -cost;
  bool near = true;
#pragma unroll
  for (int i = 0; i < D; ++i) near = near && (fabsf(s[i]) <= 0.01f);
  if (near) r = r + 1.0f;
  return r;
}

// ---------------------------------------------------------------- VanderPol
// RL/env/VanderPol.py:23-129. x'' = mu (1 - x^2) x' - x + u, mu = 1, K = 5, dt = 0.01.
struct VanderPol {
  static constexpr int D = 2, A = 1, S = 2, XS = 0, RS = 2, K = 5;
  static constexpr int ROWN = 0;  // no per-step table row
  MH_HD static float obs_lo(int i) { (void)i; return -10.0f; }
  MH_HD static float obs_hi(int i) { (void)i; return 10.0f; }
  MH_HD static float act_lo(int i) { (void)i; return -5.0f; }
  MH_HD static float act_hi(int i) { (void)i; return 5.0f; }
  MH_HD static float reset_noise() { return 5.0f; }
  MH_HD static void step(float* s, double*, int, const float* u, const double*, float* obs, float* rew) {
    for (int k = 0; k < K; ++k) {
      float x = s[0], xd = s[1];
      float acc = ((1.0f * (1.0f - powf2(x))) * xd - x) + u[0];  // VanderPol.py:95 (scalar x**2)
      s[0] = s[0] + xd * 0.01f;
      s[1] = s[1] + acc * 0.01f;
    }
    const float Q[2] = {2.0f, 1.0f}, R[1] = {0.1f};
    *rew = quad_reward<2, 1>(s, Q, u, R);
    obs[0] = s[0]; obs[1] = s[1];
  }
  MH_HD static void reset_from(const float* rs, float* s, double*, const double*, float* obs) {
    s[0] = obs[0] = rs[0];
    s[1] = obs[1] = rs[1];
  }
};

// ---------------------------------------------------------------- Pendulum
// RL/env/Pendulum.py:22-137. theta'' = (m g L sin th - b th' + u) / (m L^2).
struct Pendulum {
  static constexpr int D = 2, A = 1, S = 2, XS = 0, RS = 2, K = 5;
  static constexpr int ROWN = 0;  // no per-step table row
  MH_HD static float obs_lo(int i) { return i == 0 ? -3.14159274101257324f : -10.0f; }
  MH_HD static float obs_hi(int i) { return i == 0 ? 3.14159274101257324f : 10.0f; }
  MH_HD static float act_lo(int i) { (void)i; return -5.0f; }
  MH_HD static float act_hi(int i) { (void)i; return 5.0f; }
  MH_HD static void step(float* s, double*, int, const float* u, const double*, float* obs, float* rew) {
    const float mgL = (float)((0.15 * 9.81) * 0.5);   // Pendulum.py:102 python-float prefix
    const float mL2 = (float)(0.15 * (0.5 * 0.5));
    const float b = 0.1f;
    for (int k = 0; k < K; ++k) {
      float th = s[0], thd = s[1];
      float acc = ((mgL * sin32(th) - b * thd) + u[0]) / mL2;
      s[0] = s[0] + thd * 0.01f;
      s[1] = s[1] + acc * 0.01f;
    }
    const float Q[2] = {2.0f, 1.0f}, R[1] = {0.1f};
    *rew = quad_reward<2, 1>(s, Q, u, R);
    obs[0] = s[0]; obs[1] = s[1];
  }
  MH_HD static void reset_from(const float* rs, float* s, double*, const double*, float* obs) {
    s[0] = obs[0] = rs[0];
    s[1] = obs[1] = rs[1];
  }
};

// ---------------------------------------------------------------- DuctedFan
// RL/env/DuctedFan.py:24-147, planar ducted fan, m=8.5 g=9.81 r=0.26 d=0.95 J=0.048.
struct DuctedFan {
  static constexpr int D = 6, A = 2, S = 6, XS = 0, RS = 6, K = 5;
  static constexpr int ROWN = 0;  // no per-step table row
  MH_HD static float obs_lo(int i) { return i == 2 ? -1.57079637050628662f : -5.0f; }
  MH_HD static float obs_hi(int i) { return i == 2 ? 1.57079637050628662f : 5.0f; }
  MH_HD static float act_lo(int i) { (void)i; return -5.0f; }
  MH_HD static float act_hi(int i) { (void)i; return 5.0f; }
  MH_HD static void step(float* s, double*, int, const float* u, const double*, float* obs, float* rew) {
    const float nmg = (float)(-8.5 * 9.81), mg = (float)(8.5 * 9.81);
    const float d = 0.95f, m = 8.5f, r = 0.26f, J = 0.048f;
    for (int k = 0; k < K; ++k) {
      float th = s[2], vx = s[3], vy = s[4], om = s[5];
      float st = sin32(th), ct = cos32(th);
      float ax = (((nmg * st - d * vx) + u[0] * ct) - u[1] * st) / m;            // DuctedFan.py:107
      float ay = (((mg * (ct - 1.0f) - d * vy) + u[0] * st) + u[1] * ct) / m;    // DuctedFan.py:108
      float aw = (r * u[0]) / J;                                                  // DuctedFan.py:109
      s[0] = s[0] + vx * 0.01f;
      s[1] = s[1] + vy * 0.01f;
      s[2] = s[2] + om * 0.01f;
      s[3] = s[3] + ax * 0.01f;
      s[4] = s[4] + ay * 0.01f;
      s[5] = s[5] + aw * 0.01f;
    }
    const float Q[6] = {2.0f, 2.0f, 2.0f, 1.0f, 1.0f, 1.0f}, R[2] = {0.1f, 0.1f};
    *rew = quad_reward<6, 2>(s, Q, u, R);
#pragma unroll
    for (int i = 0; i < 6; ++i) obs[i] = s[i];
  }
  MH_HD static void reset_from(const float* rs, float* s, double*, const double*, float* obs) {
#pragma unroll
    for (int i = 0; i < 6; ++i) s[i] = obs[i] = rs[i];
  }
};

// ---------------------------------------------------------------- TwoLink
// RL/env/TwoLink.py:22-177. M(q) q'' = u - C(q,q') q' - G(q); derivative in float64
// (M and C are float64 arrays, G float32), LU solve with partial pivoting (LAPACK getrf/getrs).
struct TwoLink {
  static constexpr int D = 4, A = 2, S = 4, XS = 0, RS = 4, K = 5;
  static constexpr int ROWN = 0;  // no per-step table row
  MH_HD static float obs_lo(int i) { return i < 2 ? -1.57079637050628662f : -20.0f; }
  MH_HD static float obs_hi(int i) { return i < 2 ? 1.57079637050628662f : 20.0f; }
  MH_HD static float act_lo(int i) { (void)i; return -20.0f; }
  MH_HD static float act_hi(int i) { (void)i; return 20.0f; }
  MH_HD static void deriv(const float* s, const float* u, double* out) {
    const double I1 = (1.0 / 12.0) * 1.0 * (1.0 * 1.0);
    const double I2 = I1;
    const float q1 = s[0], q2 = s[1], dq1 = s[2], dq2 = s[3];
    // mass matrix (TwoLink.py:100-107)
    float s2, c2;
    sincos32(q2, &s2, &c2);
    float in11 = (float)(1.0 * 1.0 + 0.5 * 0.5) + ((float)((2.0 * 1.0) * 0.5) * c2);
    float M11f = (float)((I1 + I2) + 1.0 * (0.5 * 0.5)) + (1.0f * in11);
    float in12 = (float)(0.5 * 0.5) + ((float)(1.0 * 0.5) * c2);
    float M12f = (float)I2 + (1.0f * in12);
    double M11 = M11f, M12 = M12f, M21 = M12f, M22 = I2 + 1.0 * (0.5 * 0.5);
    // coriolis (TwoLink.py:109-119)
    float h = (float)((-1.0 * 1.0) * 0.5) * s2;
    float C11 = h * dq2, C12 = h * dq2 + h * dq1, C21 = (-h) * dq1;
    // gravity (TwoLink.py:121-129)
    float g1a = (float)((-(1.0 * 0.5 + 1.0 * 1.0)) * 9.81) * sin32(q1);
    float sq12 = sin32(q1 + q2);
    float g1b = (float)((1.0 * 0.5) * 9.81) * sq12;
    float G1 = g1a - g1b;
    float G2 = (float)((-1.0 * 0.5) * 9.81) * sq12;
    // rhs = (u - C @ dq) - G   (float64)
    double Cq1 = (double)C11 * (double)dq1 + (double)C12 * (double)dq2;
    double Cq2 = (double)C21 * (double)dq1 + 0.0 * (double)dq2;
    double b1 = ((double)u[0] - Cq1) - (double)G1;
    double b2 = ((double)u[1] - Cq2) - (double)G2;
    // LU of the 2 x 2 mass matrix (getrf), then forward/back substitution. getrf pivots on the
    // larger |entry| of the first column, and for this arm that is always M11: M11 = 5/3 + c2 and
    // M21 = M12 = 1/3 + c2 / 2 give M11 - |M21| >= 1/2 for every c2 in [-1, 1] (a margin no f32
    // rounding of the entries can close), so the row swap never happens and is not coded (its
    // compare and six f64 selects were ~7 % of the step's VALU at 4 M envs).
    const double a11 = M11, a12 = M12, a21 = M21, a22 = M22;
    const double i11 = rcp64(a11);
    double l21 = a21 * i11;
    double u22 = a22 - l21 * a12;
    double y2 = b2 - l21 * b1;
    double x2 = y2 * rcp64(u22);
    double x1 = (b1 - a12 * x2) * i11;
    out[0] = dq1; out[1] = dq2; out[2] = x1; out[3] = x2;
  }
  MH_HD static void step(float* s, double*, int, const float* u, const double*, float* obs, float* rew) {
    for (int k = 0; k < K; ++k) {
      double d[4];
      deriv(s, u, d);
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] = upd64(s[i], d[i], 0.01);
    }
    const float Q[4] = {2.0f, 2.0f, 1.0f, 1.0f}, R[2] = {0.1f, 0.1f};
    *rew = quad_reward<4, 2>(s, Q, u, R);
#pragma unroll
    for (int i = 0; i < 4; ++i) obs[i] = s[i];
  }
  MH_HD static void reset_from(const float* rs, float* s, double*, const double*, float* obs) {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = obs[i] = rs[i];
  }
};

// ---------------------------------------------------------------- SingleTrackCar
// RL/env/SingleTrackCar.py:41-320. x' = f(x) + g(x) u in float64 containers whose entries are
// float32 expressions; dynamic model when |v| >= 0.1 (v = ve + v_ref), kinematic otherwise.
struct CarConst {
  // Python-float constant folds, evaluated in the reference's left-to-right order.
  static constexpr double lf = 0.3048 * 3.793293;
  static constexpr double lr = 0.3048 * 4.667707;
  static constexpr double h = 0.3048 * 2.01355;
  static constexpr double m = 4.4482216152605 / 0.3048 * (74.91452);
  static constexpr double Iz = 4.4482216152605 * 0.3048 * (1321.416);
  static constexpr double mu = 0.1 * 1.0489;
  static constexpr double CS = 21.92 / 1.0489;  // -tire_p_ky1 / tire_p_dy1
  static constexpr double g = 9.81;
  static constexpr double lsum = lr + lf;
  static constexpr double P1 = mu * m;
  static constexpr double Q2 = mu * m / (Iz * (lr + lf));
  static constexpr double K1 = lf * lf * CS * g * lr + lr * lr * CS * g * lf;
  static constexpr double K2 = lr * CS * g * lf - lf * CS * g * lr;
  static constexpr double K3 = lf * CS * g * lr;
  static constexpr double K4 = CS * g * lf * lr - CS * g * lr * lf;
  static constexpr double K5 = CS * g * lf + CS * g * lr;
  static constexpr double K6 = CS * g * lr;
  static constexpr double K7 = -(lf * lf) * CS * h + lr * lr * CS * h;
  static constexpr double K8 = lr * CS * h + lf * CS * h;
  static constexpr double K9 = lf * CS * h;
  static constexpr double K10 = CS * h * lr + CS * h * lf;
  static constexpr double K11 = CS * h - CS * h;
  static constexpr double lwb = lf + lr;
  static constexpr double ilwb = 1.0 / (lf + lr);
};

struct SingleTrackCar {
  static constexpr int D = 7, A = 2, S = 7, XS = 0, RS = 7, K = 5;
  static constexpr int ROWN = 0;  // no per-step table row
  MH_HD static float obs_lo(int i) {
    const float lo[7] = {-1.0f, -1.0f, -1.06599998474121094f, -1.0f, -1.57079637050628662f,
                         -1.57079637050628662f, -1.04719758033752441f};
    return lo[i];
  }
  MH_HD static float obs_hi(int i) { return -obs_lo(i); }
  MH_HD static float act_lo(int i) { (void)i; return -5.0f; }
  MH_HD static float act_hi(int i) { (void)i; return 5.0f; }
  MH_HD static void deriv(const float* x, const float* u, double* out) {
    using C = CarConst;
    const float sxe = x[0], sye = x[1], delta = x[2], ve = x[3], pe = x[4], ped = x[5], beta = x[6];
    float v = ve + 1.0f;        // v_ref = 1.0
    float psid = ped + 0.0f;    // omega_ref = 0.0
    double f[7], g5[2] = {0.0, 0.0}, g6[2] = {0.0, 0.0}, g2 = 0.0, g3 = 0.0;
    float pb = pe + beta;
    float spb, cpb;
    sincos32(pb, &spb, &cpb);
    f[0] = (double)(((v * cpb) - 1.0f) + (0.0f * sye));   // SingleTrackCar.py:165
    f[1] = (double)((v * spb) - (0.0f * sxe));            // SingleTrackCar.py:166
    f[3] = -0.0;                                               // -a_ref
    f[2] = 0.0;
    const float lsum = (float)C::lsum;
    if (!(fabsf(v) < 0.1f)) {
      // dynamic model (SingleTrackCar.py:178-196, 243-256)
      float X = div32((float)C::P1, (v * (float)C::Iz) * lsum);
      float t1 = ((-X) * (float)C::K1) * psid;
      float t2 = (float)(C::Q2 * C::K2) * beta;
      float t3 = (float)(C::Q2 * C::K3) * delta;
      f[4] = (double)ped;
      f[5] = (double)((t1 + t2) + t3);
      float Y1 = div32((float)C::mu, powf2(v) * lsum);
      float Y2 = div32((float)C::mu, v * lsum);
      float b1 = ((Y1 * (float)C::K4) - 1.0f) * psid;
      float b2 = (Y2 * (float)C::K5) * beta;
      float b3 = (Y2 * (float)C::K6) * delta;
      f[6] = (double)((b1 - b2) + b3);
      g2 = 1.0;  // g[DELTA, VDELTA]
      g3 = 1.0;  // g[VE, ALONG]
      float gt1 = ((-X) * (float)C::K7) * psid;
      float gt2 = (float)(C::Q2 * C::K8) * beta;
      float gt3 = (float)(C::Q2 * C::K9) * delta;
      g5[1] = (double)((gt1 + gt2) - gt3);
      float hb1 = (Y1 * (float)C::K10) * psid;
      float hb2 = (Y2 * (float)C::K11) * beta;
      float hb3 = ((Y2 * (float)C::CS) * (float)C::h) * delta;
      g6[1] = (double)((hb1 - hb2) - hb3);
    } else {
      // kinematic model (SingleTrackCar.py:199-204, 259-277)
      // (a lane in this branch makes its whole wave run it: every division here is div32, sin /
      // cos of each angle share one range reduction, and tan(delta) is their quotient, within
      // ~2 ulp of tanf like the other f32 transcendental sites)
      const float lwb = (float)C::lwb, lr = (float)C::lr, ilwb = (float)C::ilwb;
      float sd, cd, cb, sb;
      sincos32(delta, &sd, &cd);
      sincos32(beta, &sb, &cb);
      const float td = div32(sd, cd);
      f[4] = (double)((div32(v * cb, lwb) * td) - 0.0f);
      f[5] = 0.0;
      f[6] = 0.0;
      float tt = div32(td * lr, lwb);
      const float cd2 = powf2(cd);
      float bdot = div32(div32(1.0f, 1.0f + powf2(tt)) * lr, lwb * cd2);
      g5[1] = (double)(ilwb * (cb * td));
      float inner = ((((-v) * sb) * td) * bdot) + div32(v * cb, cd2);
      g5[0] = (double)(ilwb * inner);
      g6[0] = (double)bdot;
    }
    // f + g @ u   (float64)
    const double u0 = (double)u[0], u1 = (double)u[1];
    out[0] = f[0] + (0.0 * u0 + 0.0 * u1);
    out[1] = f[1] + (0.0 * u0 + 0.0 * u1);
    out[2] = f[2] + (g2 * u0 + 0.0 * u1);
    out[3] = f[3] + (0.0 * u0 + g3 * u1);
    out[4] = f[4] + (0.0 * u0 + 0.0 * u1);
    out[5] = f[5] + (g5[0] * u0 + g5[1] * u1);
    out[6] = f[6] + (g6[0] * u0 + g6[1] * u1);
  }
  MH_HD static void step(float* s, double*, int, const float* u, const double*, float* obs, float* rew) {
    for (int k = 0; k < K; ++k) {
      double d[7];
      deriv(s, u, d);
#pragma unroll
      for (int i = 0; i < 7; ++i) s[i] = upd64(s[i], d[i], 0.01);
    }
    const float Q[7] = {2.0f, 2.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f}, R[2] = {0.1f, 0.1f};
    *rew = quad_reward<7, 2>(s, Q, u, R);
#pragma unroll
    for (int i = 0; i < 7; ++i) obs[i] = s[i];
  }
  MH_HD static void reset_from(const float* rs, float* s, double*, const double*, float* obs) {
#pragma unroll
    for (int i = 0; i < 7; ++i) s[i] = obs[i] = rs[i];
  }
};

// ---------------------------------------------------------------- QuadTracking
// RL/env/QuadTracking.py:20-424. Persistent f32 state x[3] v[3] R[9] (row-major) W[3];
// float64 Rd_last[9]; desired trajectory rows are a host table indexed by steps-since-reset.
constexpr int QT_ROW = 16;  // T, DT, XD[3], B1[3], VD[3] (f32 values), AD[3] (f32 values), pad, 1/DT

struct QuadConst {
  static constexpr double m = 4.34;
  static constexpr double g3 = 9.8;
  static constexpr double J0 = 0.0820, J1 = 0.0845, J2 = 0.1377;
  static constexpr double kx = 69.44, kv = 24.304;
  static constexpr double mg = 4.34 * 9.8;  // model.m * g[2]
};

// max |X^T X - I| of a 3x3 (row-major)
template <typename T>
MH_HD T orth_err3(const T* X, T* G) {
  T e = T(0);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) {
      T acc = X[0 * 3 + i] * X[0 * 3 + j];
      acc = fma(X[1 * 3 + i], X[1 * 3 + j], acc);
      acc = fma(X[2 * 3 + i], X[2 * 3 + j], acc);
      G[i * 3 + j] = G[j * 3 + i] = acc;
      T d = acc - (i == j ? T(1) : T(0));
      e = fmax(e, fabs(d));
    }
  return e;
}

// Newton-Schulz step X <- X (3I - G)/2 = X + X (I - G)/2 with G = X^T X formed in float64.
MH_HD void ns_step3(double* X, const double* G) {
  double M[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) M[i] = (((i % 4) == 0 ? 1.0 : 0.0) - G[i]) * 0.5;
  double Y[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double acc = X[i * 3 + 0] * M[0 * 3 + j];
      acc = fma(X[i * 3 + 1], M[1 * 3 + j], acc);
      acc = fma(X[i * 3 + 2], M[2 * 3 + j], acc);
      Y[i * 3 + j] = X[i * 3 + j] + acc;
    }
#pragma unroll
  for (int i = 0; i < 9; ++i) X[i] = Y[i];
}

// Same step with the correction X (I - G)/2 formed in float32 and added in float64: once
// |I - G| < 1e-6 its rounding error (~6e-8 |I - G|) is ~1e-13, far below the result ulp.
MH_HD void ns_step3_mixed(double* X, const double* G) {
  float Mf[9], Xf[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    Mf[i] = (float)(((i % 4) == 0 ? 1.0 : 0.0) - G[i]) * 0.5f;
    Xf[i] = (float)X[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float acc = Xf[i * 3 + 0] * Mf[0 * 3 + j];
      acc = fmaf(Xf[i * 3 + 1], Mf[1 * 3 + j], acc);
      acc = fmaf(Xf[i * 3 + 2], Mf[2 * 3 + j], acc);
      X[i * 3 + j] += (double)acc;
    }
}

// Third-order Newton-Schulz step X <- X (15I - 10G + 3G^2)/8 = X (I - E/2 + 3E^2/8), E = G - I
// (the binomial series of G^{-1/2} to second order): max|X^T X - I| goes e -> ~(5/8) e^3, so a
// rotation perturbed by one Euler substep (e ~ 1e-4 .. 1e-2) is at ~1e-7 after ONE step where
// the quadratic iteration needs two or three. G is symmetric; E^2 uses its 6 unique entries.
MH_HD void ns3_step3(double* X, const double* G) {
  const double E00 = G[0] - 1.0, E11 = G[4] - 1.0, E22 = G[8] - 1.0;
  const double E01 = G[1], E02 = G[2], E12 = G[5];
  const double Q00 = fma(E02, E02, fma(E01, E01, E00 * E00));
  const double Q11 = fma(E12, E12, fma(E11, E11, E01 * E01));
  const double Q22 = fma(E22, E22, fma(E12, E12, E02 * E02));
  const double Q01 = fma(E02, E12, fma(E01, E11, E00 * E01));
  const double Q02 = fma(E02, E22, fma(E01, E12, E00 * E02));
  const double Q12 = fma(E12, E22, fma(E11, E12, E01 * E02));
  const double M[9] = {fma(0.375, Q00, -0.5 * E00), fma(0.375, Q01, -0.5 * E01), fma(0.375, Q02, -0.5 * E02),
                       fma(0.375, Q01, -0.5 * E01), fma(0.375, Q11, -0.5 * E11), fma(0.375, Q12, -0.5 * E12),
                       fma(0.375, Q02, -0.5 * E02), fma(0.375, Q12, -0.5 * E12), fma(0.375, Q22, -0.5 * E22)};
  double Y[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double acc = X[i * 3 + 0] * M[0 * 3 + j];
      acc = fma(X[i * 3 + 1], M[1 * 3 + j], acc);
      acc = fma(X[i * 3 + 2], M[2 * 3 + j], acc);
      Y[i * 3 + j] = X[i * 3 + j] + acc;
    }
#pragma unroll
  for (int i = 0; i < 9; ++i) X[i] = Y[i];
}

// Orthogonal polar factor of a float32 3x3, with the det<0 column flip of
// NormalizeOrientMatrix (QuadTracking.py:308-315; U @ Vh of a float32 SVD).
// The integrator keeps R within ~(0.01|W|)^2 of SO(3), where Newton-Schulz converges
// quadratically without a division (2-3 steps to max|X^T X - I| < 1e-12, i.e. the
// float64-exact polar factor before the final rounding). Inputs farther than 0.25 from
// orthogonal take the float64 Newton iteration X <- (X + X^-T)/2.
MH_HD void polar3_general(const float* Rin, float* Rout);
struct F9 {
  float v[9];
};
// Out-of-line entry to the general routine, by value: the rare path's registers and code stay
// out of the rollout kernel's allocation (a call only where a lane needs it).
static __host__ __device__ __noinline__ F9 polar3_general_call(F9 in) {
  F9 out;
  polar3_general(in.v, out.v);
  return out;
}

// Fast path for what the integrator produces every substep: a proper rotation perturbed by one
// Euler step (max|X^T X - I| = e < 0.25, det > 0). One or two third-order steps bring e to
// < 1e-6 (e -> ~(5/8) e^3), then, when e is still >= 1e-12, one quadratic step with its f32
// correction finishes (error < 1e-12 before the final rounding): straight-line code without the
// general routine's iteration control, determinant and rare-branch code, converging to the same
// float64 polar factor (the final float32 rounding differs in ~3 of 1e6 elements, by 1 ulp).
MH_HD void polar3(const float* Rin, float* Rout) {
  double X[9], G[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) X[i] = (double)Rin[i];
  double e = orth_err3<double>(X, G);
  // sign of det: |det| is within a few % of 1 here, so float32 decides it exactly
  const float det = Rin[0] * (Rin[4] * Rin[8] - Rin[5] * Rin[7]) - Rin[1] * (Rin[3] * Rin[8] - Rin[5] * Rin[6]) +
                    Rin[2] * (Rin[3] * Rin[7] - Rin[4] * Rin[6]);
  if (__builtin_expect(e < 0.25 && det > 0.5f, 1)) {
    if (e >= 1e-7) {
      ns3_step3(X, G);
      e = orth_err3<double>(X, G);
    }
    if (e >= 1e-6) {  // e0 in [~0.01, 0.25): a second third-order step (0.25 -> 0.01 -> 6e-7)
      ns3_step3(X, G);
      e = orth_err3<double>(X, G);
    }
    if (__builtin_expect(e < 1e-6, 1)) {
      if (e >= 1e-12) ns_step3_mixed(X, G);  // e -> 0.75 e^2 + ~3e-14
#pragma unroll
      for (int i = 0; i < 9; ++i) Rout[i] = (float)X[i];
      return;
    }
  }
  F9 in;
#pragma unroll
  for (int i = 0; i < 9; ++i) in.v[i] = Rin[i];
  const F9 out = polar3_general_call(in);
#pragma unroll
  for (int i = 0; i < 9; ++i) Rout[i] = out.v[i];
}

// General polar factor: any conditioning, det < 0 flip.
MH_HD void polar3_general(const float* Rin, float* Rout) {
  double X[9], G[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) X[i] = (double)Rin[i];
  double e = orth_err3<double>(X, G);
  const bool near = e < 0.25;
  if (near) {
    for (int it = 0; it < 8 && e >= 1e-12; ++it) {
      if (e < 1e-7) {  // quadratic step, f32 correction: e -> 0.75 e^2 + ~3e-14 < 1e-13, done
        ns_step3_mixed(X, G);
        break;
      }
      if (e < 1e-6)
        ns_step3_mixed(X, G);
      else if (e < 0.05)
        ns3_step3(X, G);
      else
        ns_step3(X, G);
      e = orth_err3<double>(X, G);
    }
  }
  double X0[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) X0[i] = (double)Rin[i];
  double det0 = X0[0] * (X0[4] * X0[8] - X0[5] * X0[7]) - X0[1] * (X0[3] * X0[8] - X0[5] * X0[6]) +
                X0[2] * (X0[3] * X0[7] - X0[4] * X0[6]);
  for (int it = 0; it < 60 && !near; ++it) {
    double C[9];
    C[0] = X[4] * X[8] - X[5] * X[7];
    C[1] = X[5] * X[6] - X[3] * X[8];
    C[2] = X[3] * X[7] - X[4] * X[6];
    C[3] = X[2] * X[7] - X[1] * X[8];
    C[4] = X[0] * X[8] - X[2] * X[6];
    C[5] = X[1] * X[6] - X[0] * X[7];
    C[6] = X[1] * X[5] - X[2] * X[4];
    C[7] = X[2] * X[3] - X[0] * X[5];
    C[8] = X[0] * X[4] - X[1] * X[3];
    double det = X[0] * C[0] + X[1] * C[1] + X[2] * C[2];
    double idet = 1.0 / det;
    double diff = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      double xn = 0.5 * (X[i] + C[i] * idet);
      diff = fmax(diff, fabs(xn - X[i]));
      X[i] = xn;
    }
    if (diff <= 4e-16) break;
  }
  if (det0 < 0.0) {
    // R = U diag(1,1,-1) Vh = X (I - 2 v3 v3^T), v3 = eigenvector of H = X^T A (smallest eig).
    double H[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double acc = 0.0;
        for (int k = 0; k < 3; ++k) acc += X[k * 3 + i] * (double)Rin[k * 3 + j];
        H[i * 3 + j] = acc;
      }
    for (int i = 0; i < 3; ++i)
      for (int j = i + 1; j < 3; ++j) {
        double a = 0.5 * (H[i * 3 + j] + H[j * 3 + i]);
        H[i * 3 + j] = H[j * 3 + i] = a;
      }
    double V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 30; ++sweep) {
      double off = fabs(H[1]) + fabs(H[2]) + fabs(H[5]);
      if (off < 1e-300) break;
      for (int p = 0; p < 2; ++p)
        for (int q = p + 1; q < 3; ++q) {
          double apq = H[p * 3 + q];
          if (fabs(apq) < 1e-300) continue;
          double app = H[p * 3 + p], aqq = H[q * 3 + q];
          double theta = 0.5 * (aqq - app) / apq;
          double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
          for (int k = 0; k < 3; ++k) {  // H <- J^T H J
            double hkp = H[k * 3 + p], hkq = H[k * 3 + q];
            H[k * 3 + p] = c * hkp - s * hkq;
            H[k * 3 + q] = s * hkp + c * hkq;
          }
          for (int k = 0; k < 3; ++k) {
            double hpk = H[p * 3 + k], hqk = H[q * 3 + k];
            H[p * 3 + k] = c * hpk - s * hqk;
            H[q * 3 + k] = s * hpk + c * hqk;
          }
          for (int k = 0; k < 3; ++k) {
            double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
            V[k * 3 + p] = c * vkp - s * vkq;
            V[k * 3 + q] = s * vkp + c * vkq;
          }
        }
    }
    int mi = 0;
    for (int i = 1; i < 3; ++i)
      if (H[i * 3 + i] < H[mi * 3 + mi]) mi = i;
    double v3[3] = {V[0 * 3 + mi], V[1 * 3 + mi], V[2 * 3 + mi]};
    double Y[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double acc = 0.0;
        for (int k = 0; k < 3; ++k) {
          double hk = (k == j ? 1.0 : 0.0) - 2.0 * v3[k] * v3[j];
          acc += X[i * 3 + k] * hk;
        }
        Y[i * 3 + j] = acc;
      }
    for (int i = 0; i < 9; ++i) X[i] = Y[i];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) Rout[i] = (float)X[i];
}

MH_HD void cross64(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
// np.linalg.norm of a 3-vector = sqrt(ddot) and OpenBLAS's ddot accumulates with FMA
MH_HD double norm3(const double* a) { return sqrt(fma(a[2], a[2], fma(a[1], a[1], a[0] * a[0]))); }
// 1 / norm3(a): on the device the hardware reciprocal square root refined by two Newton steps
// (error ~1 ulp, no division / square-root expansion in the dependent chain); on the host the
// division of the square root
MH_HD double rnorm3(const double* a) {
  const double ss = fma(a[2], a[2], fma(a[1], a[1], a[0] * a[0]));
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rsq(ss);
  r = r * fma(-0.5 * ss * r, r, 1.5);
  r = r * fma(-0.5 * ss * r, r, 1.5);
  return r;
#else
  return 1.0 / sqrt(ss);
#endif
}

// Polar factor of the integrator's substep matrix X = fl32(R + dt R hat(W)), R = fl32(P), from
// the previous substep's float64 polar factor P (orthogonal to ~1e-14) instead of iterating on X:
// with M = I + h hat(w), M = C H exactly (C = polar(M) = (I + h hat(w)) / s + h^2 w w^T / (s (s+1)),
// H = s I + (1 - s) w w^T / |w|^2, s = sqrt(1 + h^2 |w|^2)), Y = P C is orthogonal and
// Z = Y^T X = H + D with D = O(1e-7) (the float32 roundings of R and X); polar(X) = Y polar(Z)
// and polar(H + D) = I + hat(k) + O(|D|^2), where hat(k) H + H hat(k) = D - D^T, i.e.
// k = (tr H I - H)^-1 vee(Z - Z^T) = sigma / (s+1) - w (w . sigma) h^2 / (2 s (s+1)^2).
// The result is within ~1e-14 of the float64 polar factor of X (numpy check against an SVD on
// 180,000 elements: max 5.9e-15, identical float32 roundings), at ~150 float64 operations per
// substep instead of two or three Newton-Schulz iterations on X. P is updated in place.
MH_HD void polar_step_incremental(double* P, const float* X, const float* W, float* Rout) {
  const double h = (double)0.01f;  // the float32 dt of R += dR * dt
  const double wx = W[0], wy = W[1], wz = W[2];
  const double q = h * h * fma(wz, wz, fma(wy, wy, wx * wx));
#if defined(__HIP_DEVICE_COMPILE__)
  // hardware reciprocal square root / reciprocal, each refined by two Newton steps
  const double x1 = 1.0 + q;
  double t = __builtin_amdgcn_rsq(x1);
  t = t * fma(-0.5 * x1 * t, t, 1.5);
  t = t * fma(-0.5 * x1 * t, t, 1.5);
  const double sq = x1 * t;
  const double y1 = sq + 1.0;
  double d = __builtin_amdgcn_rcp(y1);
  d = d * fma(-y1, d, 2.0);
  d = d * fma(-y1, d, 2.0);
#else
  const double sq = sqrt(1.0 + q);
  const double t = 1.0 / sq, d = 1.0 / (sq + 1.0);
#endif
  const double u = h * h * t * d, th = t * h;
  const double C[9] = {fma(u * wx, wx, t),       fma(u * wx, wy, -th * wz), fma(u * wx, wz, th * wy),
                       fma(u * wy, wx, th * wz), fma(u * wy, wy, t),       fma(u * wy, wz, -th * wx),
                       fma(u * wz, wx, -th * wy), fma(u * wz, wy, th * wx), fma(u * wz, wz, t)};
  double Y[9], Xd[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      Y[i * 3 + j] = fma(P[i * 3 + 2], C[2 * 3 + j], fma(P[i * 3 + 1], C[1 * 3 + j], P[i * 3 + 0] * C[0 * 3 + j]));
  for (int i = 0; i < 9; ++i) Xd[i] = (double)X[i];
  // sigma = vee(Z - Z^T), Z = Y^T X: (Z21 - Z12, Z02 - Z20, Z10 - Z01), each one FMA chain
  double sg[3];
  const int a0[3] = {2, 0, 1}, a1[3] = {1, 2, 0};
  for (int c = 0; c < 3; ++c) {
    const int i = a0[c], j = a1[c];
    double acc = Y[0 * 3 + i] * Xd[0 * 3 + j];
    acc = fma(-Y[0 * 3 + j], Xd[0 * 3 + i], acc);
    for (int k = 1; k < 3; ++k) {
      acc = fma(Y[k * 3 + i], Xd[k * 3 + j], acc);
      acc = fma(-Y[k * 3 + j], Xd[k * 3 + i], acc);
    }
    sg[c] = acc;
  }
  const double wsg = fma(wz, sg[2], fma(wy, sg[1], wx * sg[0]));
  const double f2 = 0.5 * u * d * wsg;  // h^2 (w . sigma) / (2 s (s+1)^2)
  const double k0 = fma(sg[0], d, -f2 * wx), k1 = fma(sg[1], d, -f2 * wy), k2 = fma(sg[2], d, -f2 * wz);
  // P <- Y (I + hat(k)): row i is y_i + y_i x k
  for (int i = 0; i < 3; ++i) {
    const double y0 = Y[i * 3 + 0], y1 = Y[i * 3 + 1], y2 = Y[i * 3 + 2];
    P[i * 3 + 0] = y0 + fma(y1, k2, -y2 * k1);
    P[i * 3 + 1] = y1 + fma(y2, k0, -y0 * k2);
    P[i * 3 + 2] = y2 + fma(y0, k1, -y1 * k0);
  }
  for (int i = 0; i < 9; ++i) Rout[i] = (float)P[i];
}

// float64 polar factor of a step's starting R (a float32-rounded rotation): one third-order
// Newton-Schulz step (error ~ (5/8) e^3). False when R is not within 1e-6 of orthogonal or not a
// proper rotation: the substeps then take polar3.
MH_HD bool polar_start(const float* R, double* P) {
  double G[9];
  for (int i = 0; i < 9; ++i) P[i] = (double)R[i];
  const double e = orth_err3<double>(P, G);
  const float det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                    R[2] * (R[3] * R[7] - R[4] * R[6]);
  if (!(e < 1e-6 && det > 0.5f)) return false;
  ns3_step3(P, G);
  return true;
}

struct QuadSub {
  float s[18];
};
// QuadTracking::substeps<false> by value, out of line (the general polar routine's registers stay
// out of the caller's allocation). File-static, like polar3_general_call: every translation unit
// keeps its own copy compiled with its own flags (an inline-linkage member would be merged by the
// linker across units built with different options).
static __host__ __device__ __noinline__ QuadSub quad_substeps_general_call(QuadSub q, bool inc, float f, float m0,
                                                                           float m1, float m2);

struct QuadTracking {
  // state floats: x[0:3] v[3:6] R[6:15] W[15:18]; xstate doubles: Rd_last[9]
  static constexpr int D = 12, A = 4, S = 18, XS = 9, RS = 18, K = 4;
  static constexpr int ROWN = QT_ROW;  // desired-trajectory row of the step (load_row)
  MH_HD static float obs_lo(int i) { (void)i; return -10.0f; }
  MH_HD static float obs_hi(int i) { (void)i; return 10.0f; }
  MH_HD static float act_lo(int i) { return i == 0 ? 0.0f : -10.0f; }
  MH_HD static float act_hi(int i) { return i == 0 ? (float)(2.0 * QuadConst::mg) : 10.0f; }

  // _get_desired_states (QuadTracking.py:122-149) + error observation (QuadTracking.py:241-246).
  MH_HD static void desired_and_obs(const float* s, const double* row, bool have_last,
                                    const double* Rdl, double* Rd, float* obs) {
    using Q = QuadConst;
    const float* x = s;
    const float* v = s + 3;
    const float* R = s + 6;
    const float* W = s + 15;
    const double* xd = row + 2;
    const double* b1 = row + 5;
    float vd[3] = {(float)row[8], (float)row[9], (float)row[10]};
    float ad[3] = {(float)row[11], (float)row[12], (float)row[13]};
    float ex[3], ev[3];
    double fd[3];
    const float nkx = (float)(-Q::kx), kv = (float)Q::kv, mf = (float)Q::m;
    const double mg[3] = {Q::m * 0.0, Q::m * 0.0, Q::m * Q::g3};
    for (int i = 0; i < 3; ++i) {
      ex[i] = (float)((double)x[i] - xd[i]);       // cal_ex
      ev[i] = v[i] - vd[i];                         // cal_ev (f32 - f32)
      float t = nkx * ex[i] - kv * ev[i];           // f32
      double u = (double)t - mg[i];                 // f32 - f64 -> f64
      double w = u + (double)(mf * ad[i]);          // + f32
      fd[i] = -w;
    }
    // 1 / ||v|| as one reciprocal square root (the product fd / ||fd|| then stays within ~2 ulp
    // of numpy's f64 division, far below the float32 outputs' resolution)
    const double infd = rnorm3(fd);
    double b3[3] = {fd[0] * infd, fd[1] * infd, fd[2] * infd};
    double c[3];
    cross64(b3, b1, c);
    const double inc = rnorm3(c);
    double b2[3] = {c[0] * inc, c[1] * inc, c[2] * inc};
    double b1n[3];
    cross64(b2, b3, b1n);
    for (int i = 0; i < 3; ++i) {
      Rd[i * 3 + 0] = b1n[i];
      Rd[i * 3 + 1] = b2[i];
      Rd[i * 3 + 2] = b3[i];
    }
    float Od[3] = {0.0f, 0.0f, 0.0f};
    double Odd[3] = {0.0, 0.0, 0.0};
    if (have_last) {
      const double idt = row[15];  // 1.0 / row[1], tabulated (quad_fill_table)
      float Rdot[9];
      for (int i = 0; i < 9; ++i) Rdot[i] = (float)((Rd[i] - Rdl[i]) * idt);   // RDerive
      // getOmega: So3ToVec(Rd^T @ Rdot) -> f32
      double M21 = 0.0, M02 = 0.0, M10 = 0.0;
      for (int k = 0; k < 3; ++k) {
        M21 += Rd[k * 3 + 2] * (double)Rdot[k * 3 + 1];
        M02 += Rd[k * 3 + 0] * (double)Rdot[k * 3 + 2];
        M10 += Rd[k * 3 + 1] * (double)Rdot[k * 3 + 0];
      }
      Od[0] = (float)M21; Od[1] = (float)M02; Od[2] = (float)M10;
      Odd[0] = Od[0]; Odd[1] = Od[1]; Odd[2] = Od[2];
    }
    // e_R = So3ToVec(Rd^T R - R^T Rd) * 0.5 ; P = R^T Rd
    double A_[9], P[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        double a = 0.0, p = 0.0;
        for (int k = 0; k < 3; ++k) {
          a += Rd[k * 3 + i] * (double)R[k * 3 + j];
          p += (double)R[k * 3 + i] * Rd[k * 3 + j];
        }
        A_[i * 3 + j] = a;
        P[i * 3 + j] = p;
      }
    float eR0 = (float)(A_[7] - P[7]);  // [2,1]
    float eR1 = (float)(A_[2] - P[2]);  // [0,2]
    float eR2 = (float)(A_[3] - P[3]);  // [1,0]
    // e_W = W - (R^T Rd) @ Omega_d
    for (int i = 0; i < 3; ++i) {
      double q = (P[i * 3 + 0] * Odd[0] + P[i * 3 + 1] * Odd[1]) + P[i * 3 + 2] * Odd[2];
      obs[9 + i] = (float)((double)W[i] - q);
    }
    for (int i = 0; i < 3; ++i) {
      obs[i] = ex[i];
      obs[3 + i] = ev[i];
    }
    obs[6] = eR0 * 0.5f;
    obs[7] = eR1 * 0.5f;
    obs[8] = eR2 * 0.5f;
  }

  // The desired-trajectory row of a step from k (steps since reset): the rollout kernel issues
  // it as soon as the step counter arrives, so its latency hides behind the action sampling and
  // the substeps instead of stalling desired_and_obs.
  MH_HD static void load_row(const double* tab, int k, double* rowv) {
    const double* rp = tab + (size_t)(k + 1) * QT_ROW;
    for (int i = 2; i < QT_ROW; ++i) rowv[i] = rp[i];
  }

  // One env.step (QuadTracking.py:205-285); k = steps since reset before this step.
  MH_HD static void step(float* s, double* xs, int k, const float* a, const double* tab,
                         float* obs, float* rew) {
    double rowv[QT_ROW];
    load_row(tab, k, rowv);
    step_row(s, xs, rowv, a, obs, rew);
  }

  // The K Euler substeps of env.step (QuadTracking.py:205-227) with NormalizeOrientMatrix after
  // each: FAST = every substep through the incremental polar factor P (the step's starting R is a
  // rounded rotation, `inc`), else polar3 wherever a lane's starting R is not (externally set
  // states). Both forms do the same arithmetic for a lane with inc; the split only keeps the
  // general routine (a call) and its registers out of the code every sampled lockstep runs.
  template <bool FAST>
  MH_HD static void substeps(float* s, double* P, bool inc, float f, const float* M) {
    using Q = QuadConst;
    const float mf = (float)Q::m;
    for (int it = 0; it < K; ++it) {
      float* x = s;
      float* v = s + 3;
      float* R = s + 6;
      float* W = s + 15;
      double dv[3];
      for (int i = 0; i < 3; ++i) dv[i] = (i == 2 ? Q::g3 : 0.0) - (double)((f * R[i * 3 + 2]) / mf);
      // dR = R @ hat(W)   (float32)
      float Hh[9] = {0.0f, -W[2], W[1], W[2], 0.0f, -W[0], -W[1], W[0], 0.0f};
      float dR[9];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
          dR[i * 3 + j] = (R[i * 3 + 0] * Hh[0 * 3 + j] + R[i * 3 + 1] * Hh[1 * 3 + j]) + R[i * 3 + 2] * Hh[2 * 3 + j];
      // dW = J^-1 (M - W x (J W))   (float64)
      double Wd[3] = {(double)W[0], (double)W[1], (double)W[2]};
      double JW[3] = {Q::J0 * Wd[0], Q::J1 * Wd[1], Q::J2 * Wd[2]};
      double cr[3];
      cross64(Wd, JW, cr);
      double dW[3] = {(1.0 / Q::J0) * ((double)M[0] - cr[0]), (1.0 / Q::J1) * ((double)M[1] - cr[1]),
                      (1.0 / Q::J2) * ((double)M[2] - cr[2])};
      const float Wf[3] = {W[0], W[1], W[2]};  // the W of dR (before its own update)
      for (int i = 0; i < 3; ++i) x[i] = x[i] + v[i] * 0.01f;
      for (int i = 0; i < 3; ++i) v[i] = upd64(v[i], dv[i], 0.01);
      for (int i = 0; i < 9; ++i) R[i] = R[i] + dR[i] * 0.01f;
      for (int i = 0; i < 3; ++i) W[i] = upd64(W[i], dW[i], 0.01);
      float Rn[9];
      if (FAST || __builtin_expect(inc, 1))
        polar_step_incremental(P, R, Wf, Rn);
      else
        polar3(R, Rn);
      for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    }
  }

  // env.step on a preloaded row (load_row)
  MH_HD static void step_row(float* s, double* xs, const double* rowv, const float* a, float* obs, float* rew) {
    const float f = a[0];
    const float* M = a + 1;
    // NormalizeOrientMatrix of every substep through the incremental polar factor (one
    // float64 polar factor P carried across the substeps); polar3 when the starting R is not
    // a rounded rotation (externally set states)
    double P[9];
#ifndef MH_QUAD_POLAR_NS
    const bool inc = polar_start(s + 6, P);  // float64 polar factor of the step's starting R
#if defined(__HIP_DEVICE_COMPILE__)
    const bool fast = __all(inc);  // wave-uniform: the sampled locksteps take the FAST form
#else
    const bool fast = inc;
#endif
#else
    const bool inc = false, fast = false;
#endif
    if (__builtin_expect(fast, 1)) {
      substeps<true>(s, P, true, f, M);
    } else {  // out of line: one call, in the branch no sampled lockstep takes
      QuadSub q;
      for (int i = 0; i < 18; ++i) q.s[i] = s[i];
      q = quad_substeps_general_call(q, inc, f, M[0], M[1], M[2]);
      for (int i = 0; i < 18; ++i) s[i] = q.s[i];
    }
    const double* row = rowv;
    double Rd[9];
    desired_and_obs(s, row, true, xs, Rd, obs);
    for (int i = 0; i < 9; ++i) xs[i] = Rd[i];
    // reward (QuadTracking.py:250-273), reward type 1 (linear bonus)
    float sx[3], sv[3], sr[3], sw[3], su[4];
    for (int i = 0; i < 3; ++i) {
      sx[i] = 1.0f * (obs[i] * obs[i]);
      sv[i] = 1.0f * (obs[3 + i] * obs[3 + i]);
      sr[i] = 1.0f * (obs[6 + i] * obs[6 + i]);
      sw[i] = 1.0f * (obs[9 + i] * obs[9 + i]);
    }
    const float Ract[4] = {0.0001f, 0.01f, 0.01f, 0.01f};
    for (int i = 0; i < 4; ++i) su[i] = Ract[i] * (a[i] * a[i]);
    float tot = (((np_sum<3>(sx) + np_sum<3>(sv)) + np_sum<3>(sr)) + np_sum<3>(sw)) + np_sum<4>(su);
    float r = -tot;
    float dist = 0.0f;
    for (int i = 0; i < 12; ++i) dist = fmaxf(dist, fabsf(obs[i]));
    if (dist <= 0.1f) r = r + 10.0f * (1.0f - dist / 0.1f);
    *rew = r;
  }

  // Row 0 of the desired-trajectory table (t = 0: quad_fill_table's expressions with sin 0 = 0,
  // cos 0 = 1, signed zeros kept) as constants, so a reset reads no memory; mh_env_create and
  // the host engine compare it with the filled table (quad_row0_matches).
  MH_HD static double row0(int i) {
    switch (i) {
      case 0: return 0.0;                   // t
      case 1: return 1e-6;                  // safe_time_diff(0, 0)
      case 2: return 0.4 * 0.0;             // x_d = (0.4 t, 0.4 sin t, 0.6 cos t)
      case 3: return 0.4 * 0.0;
      case 4: return 0.6 * 1.0;
      case 5: return 1.0;                   // b1_d = (cos t, sin t, 0)
      case 6: return 0.0;
      case 7: return 0.0;
      case 8: return (double)(float)0.4;    // v_d (float32 values)
      case 9: return (double)(float)(0.4 * 1.0);
      case 10: return (double)(float)(-0.6 * 0.0);
      case 11: return (double)(float)0.0;   // a_d (float32 values)
      case 12: return (double)(float)(-0.4 * 0.0);
      case 13: return (double)(float)(-0.6 * 1.0);
      case 14: return 0.0;
      default: return 1.0 / 1e-6;
    }
  }

  // reset tail (QuadTracking.py:188-202) from drawn x, v, R, W
  MH_HD static void reset_from(const float* rs, float* s, double* xs, const double* tab, float* obs) {
    (void)tab;
    for (int i = 0; i < 18; ++i) s[i] = rs[i];
    double row[QT_ROW];
    for (int i = 0; i < QT_ROW; ++i) row[i] = row0(i);
    double Rd[9];
    desired_and_obs(s, row, false, nullptr, Rd, obs);
    for (int i = 0; i < 9; ++i) xs[i] = Rd[i];
  }
};

static __host__ __device__ __noinline__ QuadSub quad_substeps_general_call(QuadSub q, bool inc, float f, float m0,
                                                                           float m1, float m2) {
  double P[9];
  if (inc) (void)polar_start(q.s + 6, P);
  const float M[3] = {m0, m1, m2};
  QuadTracking::substeps<false>(q.s, P, inc, f, M);
  return q;
}

// Row 0 of a filled table equals QuadTracking::row0 bit for bit (signed zeros included).
inline bool quad_row0_matches(const double* tab) {
  for (int i = 0; i < QT_ROW; ++i) {
    const double c = QuadTracking::row0(i);
    uint64_t a, b;
    __builtin_memcpy(&a, tab + i, 8);
    __builtin_memcpy(&b, &c, 8);
    if (a != b) return false;
  }
  return true;
}

// Host-side fill of the desired-trajectory table (QuadTracking.py:29-36, 229):
// current_time accumulates += dt * control_step in float64; row k is the time after k steps.
inline void quad_fill_table(double* tab, int rows) {
  const double inc = 0.01 * 4;
  double t = 0.0, tprev = 0.0;
  for (int k = 0; k < rows; ++k) {
    if (k > 0) {
      tprev = t;
      t = t + inc;
    }
    double* r = tab + (size_t)k * QT_ROW;
    double dt = t - tprev;
    if (dt < 1e-6) dt = 1e-6;  // safe_time_diff
    r[0] = t;
    r[1] = dt;
    r[2] = 0.4 * t;
    r[3] = 0.4 * sin(t);
    r[4] = 0.6 * cos(t);
    r[5] = cos(t);
    r[6] = sin(t);
    r[7] = 0.0;
    r[8] = (double)(float)0.4;
    r[9] = (double)(float)(0.4 * cos(t));
    r[10] = (double)(float)(-0.6 * sin(t));
    r[11] = (double)(float)0.0;
    r[12] = (double)(float)(-0.4 * sin(t));
    r[13] = (double)(float)(-0.6 * cos(t));
    r[14] = 0.0;
    r[15] = 1.0 / dt;  // reciprocal of the step for Omega_d = vee(Rd^T (Rd - Rd_last) / dt)
  }
}

}  // namespace mh
