// policy_mlp.hip — the sampler's policy forward (StochaPolicy MLP, RL/apprfunc/mlp.py:111-136)
// as ONE fused f32-MFMA kernel for gfx950.
//
//   logits = W3 relu(W2 relu(W1 obs + b1) + b2) + b3     obs [E][D], logits [E][N3] (mean | log_std)
//
// Computed transposed, one wavefront per 32-env tile, entirely in registers: with
// v_mfma_f32_32x32x2_f32 a 32x32 accumulator tile holds its COLUMN on the lane and its ROWS in
// the 16 registers, so a following MFMA that sums over the tile's row index takes the
// accumulator as its B operand with no data movement (cdna_hip_programming.md §3). Hence
//   H1^T = W1 . obs^T   (8 blocks of 32 hidden rows x 32 envs, K = D, B operand loaded from obs)
//   H2^T = W2 . H1^T    (B operand = the H1^T accumulators, k order = the accumulator row map)
//   out^T = W3 . H2^T   (accumulated block by block as each H2^T block is finished)
// so the two 256-wide hidden activations never leave the register file (the PyTorch path writes
// and re-reads 2 x 64 MB of them per lockstep at 65,536 envs). The A operands (weights) are
// pre-packed once per sample() by k_policy_pack into exactly the per-lane fragment order of
// each MFMA, so every weight fetch is a 16-B-per-lane contiguous load (L2-resident, 280 KB).
// Arithmetic is float32 in, float32 accumulate (the MFMA is a k-ordered fmaf chain); the sum
// order differs from hipBLASLt's, the values agree to float32 rounding.
//
// Fixed shape: hidden sizes 256 x 256 (the default of every reference training script), ReLU
// hidden activation, identity output, D <= 16, N3 <= 32. Other shapes use the PyTorch path.
#include "rollout.h"

namespace mh {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int PM_H = 256;           // hidden width (both layers)
constexpr int PM_NB = PM_H / 32;    // 32-row blocks per hidden layer

// packed parameter layout (floats):
//   W1p [NB][K1][64]        W1[blk*32 + (l&31)][2s + (l>>5)]
//   b1p [NB][64][16]        b1[blk*32 + row(r, l)]
//   W2p [NB ob][NB ib][4 q][64][4]   W2[ob*32 + (l&31)][ib*32 + row(4q + j, l)]
//   b2p [NB][64][16]
//   W3p [NB][4 q][64][4]    W3[(l&31)][ob*32 + row(4q + j, l)]   (0 for l&31 >= N3)
//   b3  [32]
// row(r, l) = (r & 3) + 8 (r >> 2) + 4 (l >> 5): the accumulator row held in register r.
__host__ __device__ constexpr int64_t pm_off_b1(int K1) { return (int64_t)PM_NB * K1 * 64; }
__host__ __device__ constexpr int64_t pm_off_w2(int K1) { return pm_off_b1(K1) + PM_NB * 64 * 16; }
__host__ __device__ constexpr int64_t pm_off_b2(int K1) { return pm_off_w2(K1) + (int64_t)PM_NB * PM_NB * 16 * 64; }
__host__ __device__ constexpr int64_t pm_off_w3(int K1) { return pm_off_b2(K1) + PM_NB * 64 * 16; }
__host__ __device__ constexpr int64_t pm_off_b3(int K1) { return pm_off_w3(K1) + PM_NB * 16 * 64; }
__host__ __device__ constexpr int64_t pm_packed_floats(int K1) { return pm_off_b3(K1) + 32; }

__device__ __forceinline__ int pm_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// One thread per packed float.
__global__ __launch_bounds__(256) void k_policy_pack(const float* __restrict__ W1, const float* __restrict__ b1,
                                                     const float* __restrict__ W2, const float* __restrict__ b2,
                                                     const float* __restrict__ W3, const float* __restrict__ b3,
                                                     int D, int N3, int K1, float* __restrict__ P) {
  const int64_t total = pm_packed_floats(K1);
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    float v = 0.0f;
    if (q < pm_off_b1(K1)) {
      const int l = (int)(q % 64), s = (int)((q / 64) % K1), blk = (int)(q / (64 * K1));
      const int k = 2 * s + (l >> 5);
      if (k < D) v = W1[(int64_t)(blk * 32 + (l & 31)) * D + k];
    } else if (q < pm_off_w2(K1)) {
      const int64_t o = q - pm_off_b1(K1);
      const int r = (int)(o % 16), l = (int)((o / 16) % 64), blk = (int)(o / (16 * 64));
      v = b1[blk * 32 + pm_row(r, l)];
    } else if (q < pm_off_b2(K1)) {
      const int64_t o = q - pm_off_w2(K1);
      const int j = (int)(o % 4), l = (int)((o / 4) % 64), qq = (int)((o / 256) % 4), ib = (int)((o / 1024) % PM_NB),
                ob = (int)(o / (1024 * PM_NB));
      v = W2[(int64_t)(ob * 32 + (l & 31)) * PM_H + ib * 32 + pm_row(4 * qq + j, l)];
    } else if (q < pm_off_w3(K1)) {
      const int64_t o = q - pm_off_b2(K1);
      const int r = (int)(o % 16), l = (int)((o / 16) % 64), blk = (int)(o / (16 * 64));
      v = b2[blk * 32 + pm_row(r, l)];
    } else if (q < pm_off_b3(K1)) {
      const int64_t o = q - pm_off_w3(K1);
      const int j = (int)(o % 4), l = (int)((o / 4) % 64), qq = (int)((o / 256) % 4), ob = (int)(o / 1024);
      if ((l & 31) < N3) v = W3[(int64_t)(l & 31) * PM_H + ob * 32 + pm_row(4 * qq + j, l)];
    } else {
      const int o = (int)(q - pm_off_b3(K1));
      if (o < N3) v = b3[o];
    }
    P[q] = v;
  }
}

template <int K1>
#ifndef MH_POLICY_MIN_WAVES
#define MH_POLICY_MIN_WAVES 1
#endif
__global__ __launch_bounds__(256, MH_POLICY_MIN_WAVES) void k_policy_forward(const float* __restrict__ P, const float* __restrict__ obs,
                                                           int64_t E, int D, int N3, float* __restrict__ logits) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b0 = tile * 32;
  if (b0 >= E) return;
  const int64_t brow = min(b0 + (lane & 31), E - 1);  // padded tail rows read the last env
  const float* W1p = P;
  const float* b1p = P + pm_off_b1(K1);
  const f32x4* W2p = reinterpret_cast<const f32x4*>(P + pm_off_w2(K1));
  const float* b2p = P + pm_off_b2(K1);
  const f32x4* W3p = reinterpret_cast<const f32x4*>(P + pm_off_w3(K1));
  const float* b3 = P + pm_off_b3(K1);

  // ---- layer 1: H1^T blocks (32 hidden x 32 envs), bias + ReLU
  float xo[K1];
#pragma unroll
  for (int s = 0; s < K1; ++s) {
    const int k = 2 * s + (lane >> 5);
    xo[s] = k < D ? obs[brow * D + k] : 0.0f;
  }
  f32x16 h1[PM_NB];
#pragma unroll
  for (int blk = 0; blk < PM_NB; ++blk) {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < K1; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(W1p[(blk * K1 + s) * 64 + lane], xo[s], acc, 0, 0, 0);
    const f32x4* bb = reinterpret_cast<const f32x4*>(b1p + (blk * 64 + lane) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b = bb[q];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 * q + j] = fmaxf(acc[4 * q + j] + b[j], 0.0f);
    }
    h1[blk] = acc;
  }
  // ---- layers 2 and 3: each H2^T block in turn, folded into out^T right away. The W2 fragments
  // stream through a ring of PF registers loaded PF steps ahead of their MFMAs (one step = one
  // 16-B load feeding four MFMAs = 256 MFMA cycles), crossing block boundaries, so the L2
  // latency hides behind the MFMA pipe; bias/W3 fragments of a block are fetched at its start.
  constexpr int PF = 8;
  constexpr int STEPS = PM_NB * 4;  // 16-B fragments per output block
  f32x16 o3 = {};
  f32x4 ring[PF];
#pragma unroll
  for (int t = 0; t < PF; ++t) ring[t] = W2p[t * 64 + lane];
  for (int ob = 0; ob < PM_NB; ++ob) {
    const f32x4* bb = reinterpret_cast<const f32x4*>(b2p + (ob * 64 + lane) * 16);
    const f32x4* w3 = W3p + (int64_t)ob * 4 * 64 + lane;
    f32x4 bias[4], w3f[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bias[q] = bb[q];
      w3f[q] = w3[q * 64];
    }
    // fragment t of block ob is W2p[(ob * STEPS + t) * 64 + lane]; the prefetch of step t + PF runs
    // into block ob + 1 near the end (for the last block it reads the b2 region: in bounds, unused)
    const f32x4* w2 = W2p + (int64_t)ob * STEPS * 64 + lane;
    f32x16 acc = {};
#pragma unroll
    for (int t = 0; t < STEPS; ++t) {
      const f32x4 a = ring[t % PF];
      ring[t % PF] = w2[(t + PF) * 64];
      const int ib = t >> 2, q = t & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], h1[ib][4 * q + j], acc, 0, 0, 0);
      // keep the prefetch in this step: without a barrier the scheduler sinks every load next
      // to its first use and the MFMA pipe waits on L2 latency each step
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 * q + j] = fmaxf(acc[4 * q + j] + bias[q][j], 0.0f);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) o3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w3f[q][j], acc[4 * q + j], o3, 0, 0, 0);
  }
  // ---- out^T rows o = row(r, lane) for env column lane & 31: + b3, store [E][N3]
  const int64_t b = b0 + (lane & 31);
  if (b < E) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = pm_row(r, lane);
      if (o < N3) logits[b * N3 + o] = o3[r] + b3[o];
    }
  }
}

int64_t policy_packed_floats(int D) { return pm_packed_floats((D + 1) / 2); }

hipError_t launch_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                              const float* b3, int D, int N3, float* P, hipStream_t st) {
  const int K1 = (D + 1) / 2;
  const int64_t total = pm_packed_floats(K1);
  const int grid = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
  k_policy_pack<<<grid, 256, 0, st>>>(W1, b1, W2, b2, W3, b3, D, N3, K1, P);
  return hipGetLastError();
}

template <int K1>
static hipError_t launch_fwd_t(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                               hipStream_t st) {
  const int64_t tiles = (E + 31) / 32;
  k_policy_forward<K1><<<(unsigned)((tiles + 3) / 4), 256, 0, st>>>(P, obs, E, D, N3, logits);
  return hipGetLastError();
}

hipError_t launch_policy_forward(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                                 hipStream_t st) {
  if (E <= 0) return hipSuccess;
  switch ((D + 1) / 2) {
    case 1: return launch_fwd_t<1>(P, obs, E, D, N3, logits, st);
    case 2: return launch_fwd_t<2>(P, obs, E, D, N3, logits, st);
    case 3: return launch_fwd_t<3>(P, obs, E, D, N3, logits, st);
    case 4: return launch_fwd_t<4>(P, obs, E, D, N3, logits, st);
    case 5: return launch_fwd_t<5>(P, obs, E, D, N3, logits, st);
    case 6: return launch_fwd_t<6>(P, obs, E, D, N3, logits, st);
    case 7: return launch_fwd_t<7>(P, obs, E, D, N3, logits, st);
    case 8: return launch_fwd_t<8>(P, obs, E, D, N3, logits, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mh
