// gae.hip — generalized advantage estimation over the on-policy trajectory store (gfx950).
//
// Restates OnSampler._process_experiences / _finish_trajs (RL/trainer/sampler/on_sampler.py:
// 108-154) for a whole [E][H] trajectory block at once. A segment of env e ends at step t when
// done[e][t] or t == H-1; its bootstrap value is V(real_next_obs) * (1 - done) (:125-129), the
// rest of the segment bootstraps from V(obs[t+1]) (:143-148). Per step, reverse over time:
//   delta = rew + gamma * V_next - V          (float64: the reference's value slice is float64)
//   gae   = delta + (gamma * lambda) * gae    (float64, stored rounded to float32)
//   G     = rew + gamma * G                   (float32: NumPy-2 scalar promotion, weak Python float)
//
// Layout: every array is env-major [E][H] (the reference's mb_* arrays). One wavefront owns 64
// envs and walks the horizon backwards in 32-step chunks; each chunk is staged through LDS with
// coalesced row loads (32 consecutive steps of one env = 128 contiguous bytes per half-wave),
// the per-env recurrence then reads LDS column-wise (rows padded by one dword: conflict-free),
// and adv/ret leave through the same tiles with coalesced row stores. HBM-bound: 17 B per step
// (val, rew, done in; adv, ret out) plus one bootstrap read per segment end.
#include "rollout.h"

namespace mh {

constexpr int GAE_TC = 32;

__global__ __launch_bounds__(64) void k_gae(const float* __restrict__ val, const float* __restrict__ val2,
                                            const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                            int64_t E, int H, double gamma, double lam,
                                            float* __restrict__ adv, float* __restrict__ ret) {
  __shared__ float s_a[64][GAE_TC + 1];   // val in, adv out
  __shared__ float s_b[64][GAE_TC + 1];   // rew in, ret out
  __shared__ uint8_t s_d[64][GAE_TC + 4];
  const int lane = threadIdx.x;
  const int64_t e0 = (int64_t)blockIdx.x * 64;
  const int64_t e = e0 + lane;
  const float gf = (float)gamma;
  const double gl = gamma * lam;
  double gae = 0.0;
  float G = 0.0f;
  float next_v = 0.0f;
  const int half = lane >> 5, col = lane & 31;
  for (int c = (H - 1) / GAE_TC; c >= 0; --c) {
    const int t0 = c * GAE_TC;
    const int tn = min(GAE_TC, H - t0);
    for (int r = half; r < 64; r += 2) {
      const int64_t er = e0 + r;
      if (er < E && col < tn) {
        const int64_t o = er * H + t0 + col;
        s_a[r][col] = val[o];
        s_b[r][col] = rew[o];
        s_d[r][col] = done[o];
      }
    }
    __syncthreads();
    if (e < E) {
      for (int j = tn - 1; j >= 0; --j) {
        const int t = t0 + j;
        const float v = s_a[lane][j];
        const float rw = s_b[lane][j];
        const bool d = s_d[lane][j] != 0;
        double nv;
        if (d || t == H - 1) {  // segment end: est_last_value = V(real_next_obs) * (1 - done)
          nv = (double)val2[e * H + t] * (d ? 0.0 : 1.0);
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
    __syncthreads();
    for (int r = half; r < 64; r += 2) {
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
