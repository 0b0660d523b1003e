// gae.hip — generalized advantage estimation over the on-policy trajectory store (gfx950).
//
// Restates OnSampler._process_experiences / _finish_trajs (RL/trainer/sampler/on_sampler.py:
// 108-154) for a whole [E][H] trajectory block at once. A segment of env e ends at step t when
// done[e][t] or t == H-1; its bootstrap value is V(real_next_obs) * (1 - done) (:125-129), the
// rest of the segment bootstraps from V(obs[t+1]) (:143-148). Per step, reverse over time:
//   delta = rew + gamma * V_next - V          (float64: the reference's value slice is float64)
//   gae   = delta + (gamma * lambda) * gae    (float64, stored rounded to float32)
//   G     = rew + gamma * G                   (float32: NumPy-2 scalar promotion, weak Python float)
// The return recurrence must stay sequential per env (float32 rounding order = the reference's),
// so the parallelism is one lane per env.
//
// Layout: every array is env-major [E][H] (the reference's mb_* arrays). One wavefront owns 64
// envs and walks the horizon backwards in 32-step chunks. A chunk is staged through LDS with
// coalesced row loads (32 consecutive steps of one env = 128 contiguous bytes per half-wave); the
// per-env recurrence then reads LDS column-wise (rows padded by one dword: conflict-free) and
// adv/ret leave through the same tiles with coalesced row stores. The loads are software-
// pipelined in registers: while chunk c is computed, chunk c-1's val/rew are in flight, and so
// are its bootstrap values val2 — loaded ONLY where a segment ends (the done flags of chunk c-1
// were fetched one stage earlier), so the kernel moves the algorithmic bytes: 17 B per step
// (val, rew, done in; adv, ret out) + 4 B per segment end.
#include "rollout.h"

namespace mh {

constexpr int GAE_TC = 32;       // steps per chunk
constexpr int GAE_RPL = 32;      // rows (envs) each lane loads per chunk: 64 rows / 2 half-waves

struct GaeTile {
  float v[GAE_RPL], r[GAE_RPL], v2[GAE_RPL];
  uint32_t d[GAE_RPL];
};

__device__ __forceinline__ void gae_load_done(const uint8_t* __restrict__ done, int64_t e0, int64_t E, int H, int t0,
                                              int tn, int half, int col, uint32_t* d) {
#pragma unroll
  for (int k = 0; k < GAE_RPL; ++k) {
    const int64_t er = e0 + half + 2 * k;
    d[k] = (er < E && col < tn) ? (uint32_t)done[er * H + t0 + col] : 0u;
  }
}

// val/rew of a chunk, and val2 where the chunk's step ends a segment (done, or the horizon)
__device__ __forceinline__ void gae_load_vals(const float* __restrict__ val, const float* __restrict__ val2,
                                              const float* __restrict__ rew, int64_t e0, int64_t E, int H, int t0,
                                              int tn, int half, int col, const uint32_t* d, GaeTile& x) {
  const bool last_col = (t0 + col == H - 1);
#pragma unroll
  for (int k = 0; k < GAE_RPL; ++k) {
    const int64_t er = e0 + half + 2 * k;
    const bool ok = er < E && col < tn;
    const int64_t o = er * H + t0 + col;
    x.v[k] = ok ? val[o] : 0.0f;
    x.r[k] = ok ? rew[o] : 0.0f;
    x.v2[k] = (ok && (d[k] != 0u || last_col)) ? val2[o] : 0.0f;
  }
}

__global__ __launch_bounds__(64) void k_gae(const float* __restrict__ val, const float* __restrict__ val2,
                                            const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                            int64_t E, int H, double gamma, double lam,
                                            float* __restrict__ adv, float* __restrict__ ret) {
  __shared__ float s_a[64][GAE_TC + 1];   // val in, adv out
  __shared__ float s_b[64][GAE_TC + 1];   // rew in, ret out
  __shared__ float s_v2[64][GAE_TC + 1];  // bootstrap values at segment ends
  __shared__ uint8_t s_d[64][GAE_TC + 1];
  const int lane = threadIdx.x;
  const int half = lane >> 5, col = lane & 31;
  const int64_t e0 = (int64_t)blockIdx.x * 64;
  const int64_t e = e0 + lane;
  const float gf = (float)gamma;
  const double gl = gamma * lam;
  double gae = 0.0;
  float G = 0.0f;
  float next_v = 0.0f;

  const int c0 = (H - 1) / GAE_TC;
  GaeTile x;
  uint32_t d_cur[GAE_RPL], d_next[GAE_RPL];
  // prologue: done + values of the last chunk, done of the one before it
  gae_load_done(done, e0, E, H, c0 * GAE_TC, min(GAE_TC, H - c0 * GAE_TC), half, col, d_cur);
  gae_load_vals(val, val2, rew, e0, E, H, c0 * GAE_TC, min(GAE_TC, H - c0 * GAE_TC), half, col, d_cur, x);
  if (c0 > 0) gae_load_done(done, e0, E, H, (c0 - 1) * GAE_TC, GAE_TC, half, col, d_next);

  for (int c = c0; c >= 0; --c) {
    const int t0 = c * GAE_TC;
    const int tn = min(GAE_TC, H - t0);
    // stage chunk c (registers -> LDS)
#pragma unroll
    for (int k = 0; k < GAE_RPL; ++k) {
      const int r = half + 2 * k;
      s_a[r][col] = x.v[k];
      s_b[r][col] = x.r[k];
      s_v2[r][col] = x.v2[k];
      s_d[r][col] = (uint8_t)d_cur[k];
    }
    __syncthreads();
    // prefetch chunk c-1 (its done flags arrived last iteration) and the done flags of c-2
    if (c > 0) {
#pragma unroll
      for (int k = 0; k < GAE_RPL; ++k) d_cur[k] = d_next[k];
      gae_load_vals(val, val2, rew, e0, E, H, t0 - GAE_TC, GAE_TC, half, col, d_cur, x);
      if (c > 1) gae_load_done(done, e0, E, H, t0 - 2 * GAE_TC, GAE_TC, half, col, d_next);
    }
    // reverse recurrence of chunk c, one env per lane
    if (e < E) {
#pragma unroll
      for (int j = GAE_TC - 1; j >= 0; --j) {
        if (j < tn) {
          const int t = t0 + j;
          const float v = s_a[lane][j];
          const float rw = s_b[lane][j];
          const bool d = s_d[lane][j] != 0;
          double nv;
          if (d || t == H - 1) {  // segment end: est_last_value = V(real_next_obs) * (1 - done)
            nv = (double)s_v2[lane][j] * (d ? 0.0 : 1.0);
            gae = 0.0;
            G = 0.0f;
          } else {
            nv = (double)next_v;
          }
          const double delta = ((double)rw + gamma * nv) - (double)v;
          gae = delta + gl * gae;
          G = rw + gf * G;
          s_a[lane][j] = (float)gae;
          s_b[lane][j] = G;
          next_v = v;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GAE_RPL; ++k) {
      const int r = half + 2 * k;
      const int64_t er = e0 + r;
      if (er < E && col < tn) {
        const int64_t o = er * H + t0 + col;
        adv[o] = s_a[r][col];
        ret[o] = s_b[r][col];
      }
    }
    __syncthreads();
  }
}

hipError_t launch_gae(const float* val, const float* val2, const float* rew, const uint8_t* done, int64_t E,
                      int H, double gamma, double lam, float* adv, float* ret, hipStream_t st) {
  if (E <= 0 || H <= 0) return hipSuccess;
  const int64_t grid = (E + 63) / 64;
  k_gae<<<(unsigned)grid, 64, 0, st>>>(val, val2, rew, done, E, H, gamma, lam, adv, ret);
  return hipGetLastError();
}

}  // namespace mh
