// philox.h — counter-based Philox4x32-10 for in-kernel action noise and reset draws.
// Stateless: the counter is (env index, stream id, lockstep tick) so a hipGraph replay only
// needs the device-resident tick to advance, never a host-side RNG state.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mh {

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)M0 * c.x;
    uint64_t p1 = (uint64_t)M1 * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// uniform in [0, 1) with 32 random bits, as double
__host__ __device__ __forceinline__ double u01(uint32_t v) { return (double)v * 2.3283064365386963e-10; }

struct Rng {
  uint32_t k0, k1;
  uint32_t env_lo, env_hi, tick_lo, tick_hi;
  __host__ __device__ __forceinline__ u32x4 draw(uint32_t stream) const {
    return philox4x32_10(u32x4{env_lo, env_hi ^ (stream << 16), tick_lo, tick_hi}, k0, k1);
  }
  // 4 standard normals via Box-Muller in float32 (action noise: torch draws float32 normals too)
  __host__ __device__ __forceinline__ void normal4f(uint32_t stream, float* out) const {
    u32x4 r = draw(stream);
    // 24-bit uniforms; u1,u3 in (0, 1] so log() stays finite
    float u1 = 1.0f - (float)(r.x >> 8) * 5.9604644775390625e-08f, u2 = (float)(r.y >> 8) * 5.9604644775390625e-08f;
    float u3 = 1.0f - (float)(r.z >> 8) * 5.9604644775390625e-08f, u4 = (float)(r.w >> 8) * 5.9604644775390625e-08f;
    float a = sqrtf(-2.0f * logf(u1)), b = sqrtf(-2.0f * logf(u3));
    const float tp = 6.28318530717958648f;
    float s2, c2, s4, c4;
    sincosf(tp * u2, &s2, &c2);
    sincosf(tp * u4, &s4, &c4);
    out[0] = a * c2;
    out[1] = a * s2;
    out[2] = b * c4;
    out[3] = b * s4;
  }
  // 4 standard normals via Box-Muller on the hardware transcendentals (v_log_f32, v_sqrt_f32,
  // v_sin_f32/v_cos_f32, which take the angle in revolutions: sin(2 pi u) = v_sin_f32(u)).
  // ~1 ulp each; used for the policy's action noise, whose values are distribution-matched only
  // (torch's CPU generator cannot be replayed on the device).
  __device__ __forceinline__ void normal4f_fast(uint32_t stream, float* out) const {
    u32x4 r = draw(stream);
    const float u1 = 1.0f - (float)(r.x >> 8) * 5.9604644775390625e-08f;
    const float u2 = (float)(r.y >> 8) * 5.9604644775390625e-08f;
    const float u3 = 1.0f - (float)(r.z >> 8) * 5.9604644775390625e-08f;
    const float u4 = (float)(r.w >> 8) * 5.9604644775390625e-08f;
    const float ln2x2 = -2.0f * 0.693147180559945309f;  // -2 ln(u) = -2 ln2 log2(u)
    const float a = __builtin_amdgcn_sqrtf(ln2x2 * __builtin_amdgcn_logf(u1));
    const float b = __builtin_amdgcn_sqrtf(ln2x2 * __builtin_amdgcn_logf(u3));
    out[0] = a * __builtin_amdgcn_cosf(u2);
    out[1] = a * __builtin_amdgcn_sinf(u2);
    out[2] = b * __builtin_amdgcn_cosf(u4);
    out[3] = b * __builtin_amdgcn_sinf(u4);
  }
  // 4 standard normals via Box-Muller (float64 internally)
  __host__ __device__ __forceinline__ void normal4(uint32_t stream, double* out) const {
    u32x4 r = draw(stream);
    double u1 = 1.0 - u01(r.x), u2 = u01(r.y), u3 = 1.0 - u01(r.z), u4 = u01(r.w);
    double a = sqrt(-2.0 * log(u1)), b = sqrt(-2.0 * log(u3));
    const double tp = 6.283185307179586;
    out[0] = a * cos(tp * u2);
    out[1] = a * sin(tp * u2);
    out[2] = b * cos(tp * u4);
    out[3] = b * sin(tp * u4);
  }
};

// The argument of TanhGaussDistribution's log-Jacobian term, 1 + EPS - tanh(z)^2
// (act_distribution_cls.py:50-54), from t = exp(-2|z|) and rt = 1 / (1 + t). PyTorch evaluates
// `1 + EPS - tensor` with the Python scalar rounded to float32 (1.00000095367431640625), so the
// constant here is that value minus 1, exactly. 1 - tanh^2 = 4 t / (1 + t)^2 has no cancellation,
// whereas float32 1.000001 - th * th keeps only a few digits once |z| > 2 (the log term's error
// reached 1e-4 at |z| = 4): this form is within a few float32 ulp of the exact value everywhere
// (oracle/rng.py tanh_gauss_sample, tests/test_gpu_sampler_oracle.py).
__host__ __device__ __forceinline__ float squash_arg(float t, float rt) {
  return 9.5367431640625e-07f + (4.0f * t) * (rt * rt);
}

__host__ __device__ __forceinline__ Rng make_rng(uint64_t seed, uint64_t env, uint64_t tick) {
  return Rng{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)env, (uint32_t)(env >> 32),
             (uint32_t)tick, (uint32_t)(tick >> 32)};
}

}  // namespace mh
