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
//   W1p [NB][K1][64]        W1[blk*32 + (l&31)][2s + (l>>5)]; k = D holds b1 (constant-1 input)
//   b1p [NB][64][16]        b1[blk*32 + row(r, l)]
//   W2p [NB ob][NB ib][4 q][64][4]   W2[ob*32 + (l&31)][ib*32 + row(4q + j, l)]
//   b2p [NB][64][16]
//   W3p [NB][4 q][64][4]    W3[(l&15)][ob*32 + row(4q + j, l)] for N3 <= 16 (layer 3 on the
//                           16x16x1 4-block MFMA), else W3[(l&31)][...]   (0 for rows >= N3)
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
      else if (k == D) v = b1[blk * 32 + (l & 31)];  // bias as the weight of a constant-1 input
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
      // N3 <= 16 (layer 3 on v_mfma_f32_16x16x1_4b: output row = lane & 15), else lane & 31
      const int orow = N3 <= 16 ? (l & 15) : (l & 31);
      if (orow < N3) v = W3[(int64_t)orow * PM_H + ob * 32 + pm_row(4 * qq + j, l)];
    } else {
      const int o = (int)(q - pm_off_b3(K1));
      if (o < N3) v = b3[o];
    }
    P[q] = v;
  }
}

// K1 = k-steps of layer 1 = ceil((D + 1) / 2): the observation plus a constant-1 input that
// carries the layer-1 bias inside the MFMA. Persistent: each wave walks tiles tile0,
// tile0 + nwaves, ...; W1 fragments stay in registers, the W2 ring runs on across tiles (the
// same weights for every tile) and the next tile's observations are fetched a tile ahead.
#ifndef MH_POLICY_MIN_WAVES
#define MH_POLICY_MIN_WAVES 1
#endif
template <int K1, bool L3B4>
__global__ __launch_bounds__(256, MH_POLICY_MIN_WAVES) void k_policy_forward(const float* __restrict__ P,
                                                                            const float* __restrict__ obs, int64_t E,
                                                                            int D, int N3, float* __restrict__ logits) {
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (E + 31) / 32;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const float* W1p = P;
  const f32x4* W2p = reinterpret_cast<const f32x4*>(P + pm_off_w2(K1));
  const float* b2p = P + pm_off_b2(K1);
  const f32x4* W3p = reinterpret_cast<const f32x4*>(P + pm_off_w3(K1));
  const float* b3 = P + pm_off_b3(K1);
  constexpr int PF = 8;                 // W2 prefetch distance (16-B fragments)
#ifndef MH_POLICY_NACC
#define MH_POLICY_NACC 1
#endif
  constexpr int NACC = MH_POLICY_NACC;  // accumulation chains of layer 2
  constexpr int STEPS = PM_NB * 4;      // fragments per output block
  constexpr int ALL = PM_NB * STEPS;    // fragments of W2 (the ring wraps: same W2 every tile)

  float w1f[PM_NB][K1];
#pragma unroll
  for (int blk = 0; blk < PM_NB; ++blk)
#pragma unroll
    for (int s = 0; s < K1; ++s) w1f[blk][s] = W1p[(blk * K1 + s) * 64 + lane];
  auto load_obs = [&](int64_t t, float* xo) {
    const int64_t brow = min(t * 32 + (lane & 31), E - 1);  // padded tail rows read the last env
#pragma unroll
    for (int s = 0; s < K1; ++s) {
      const int k = 2 * s + (lane >> 5);
      xo[s] = k < D ? obs[brow * D + k] : (k == D ? 1.0f : 0.0f);
    }
  };
  float xo[K1];
  load_obs(tile, xo);
  f32x4 ring[PF];
#pragma unroll
  for (int t = 0; t < PF; ++t) ring[t] = W2p[t * 64 + lane];

  for (; tile < ntiles; tile += nwaves) {
    // ---- layer 1: H1^T blocks (32 hidden x 32 envs) = ReLU(W1 [obs; 1]), bias inside the MFMA
    f32x16 h1[PM_NB];
#pragma unroll
    for (int blk = 0; blk < PM_NB; ++blk) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < K1; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1f[blk][s], xo[s], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = fmaxf(acc[r], 0.0f);
      h1[blk] = acc;
    }
    const int64_t next = tile + nwaves;
    if (next < ntiles) load_obs(next, xo);  // a whole tile of MFMAs to land
    // ---- layers 2 and 3: each H2^T block in turn, folded into out^T right away. W2 fragments
    // stream through a ring of PF registers loaded PF steps ahead of their MFMAs (one step = one
    // 16-B load feeding four MFMAs = 256 MFMA cycles); bias/W3 fragments at the block start.
    f32x16 o3 = {};
    for (int ob = 0; ob < PM_NB; ++ob) {
      const f32x4* bb = reinterpret_cast<const f32x4*>(b2p + (ob * 64 + lane) * 16);
      const f32x4* w3 = W3p + (int64_t)ob * 4 * 64 + lane;
      f32x4 bias[4], w3f[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bias[q] = bb[q];
        w3f[q] = w3[q * 64];
      }
      // NACC independent accumulation chains (k interleaved), summed at the end: one dependent
      // chain of v_mfma_f32_32x32x2_f32 does not keep the MFMA pipe full
      f32x16 accs[NACC];
#pragma unroll
      for (int c = 0; c < NACC; ++c) accs[c] = f32x16{};
#pragma unroll
      for (int t = 0; t < STEPS; ++t) {
        const f32x4 a = ring[t % PF];
        int nxt = ob * STEPS + t + PF;
        nxt = nxt >= ALL ? nxt - ALL : nxt;
        ring[t % PF] = W2p[nxt * 64 + lane];
        const int ib = t >> 2, q = t & 3;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          accs[j % NACC] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], h1[ib][4 * q + j], accs[j % NACC], 0, 0, 0);
        // keep the prefetch in this step: without a barrier the scheduler sinks every load next
        // to its first use and the MFMA pipe waits on L2 latency each step
        __builtin_amdgcn_sched_barrier(0);
      }
      f32x16 acc = accs[0];
#pragma unroll
      for (int c = 1; c < NACC; ++c) acc = acc + accs[c];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[4 * q + j] = fmaxf(acc[4 * q + j] + bias[q][j], 0.0f);
      if constexpr (L3B4) {
        // N3 <= 16: v_mfma_f32_16x16x1_4b_f32, 16 output rows instead of 32 (half the cycles).
        // Block b (lanes 16b..16b+15) takes B = acc[r] there: envs 16 (b & 1) + (l & 15), the
        // k row of half b >> 1; A = W3[l & 15][that k]. Blocks b and b + 2 hold the two k halves
        // of the same envs, in registers 4b..4b+3 and 4b+8..4b+11 of the same lane
        // (tools/mfma_probe.hip: C of block b at reg 4b + q, row 4 (l >> 4) + q, column l & 15).
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) o3 = __builtin_amdgcn_mfma_f32_16x16x1f32(w3f[q][j], acc[4 * q + j], o3, 0, 0, 0);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) o3 = __builtin_amdgcn_mfma_f32_32x32x2f32(w3f[q][j], acc[4 * q + j], o3, 0, 0, 0);
      }
    }
    if constexpr (L3B4) {
      // ---- out^T row o = 4 (lane >> 4) + q for envs (lane & 15) + 16 h: the two k halves
      // (blocks h and h + 2) added, + b3, store [E][N3]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t b = tile * 32 + (lane & 15) + 16 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int o = 4 * (lane >> 4) + q;
          if (b < E && o < N3) logits[b * N3 + o] = (o3[4 * h + q] + o3[4 * h + 8 + q]) + b3[o];
        }
      }
    } else {
      // ---- out^T rows o = row(r, lane) for env column lane & 31: + b3, store [E][N3]
      const int64_t b = tile * 32 + (lane & 31);
      if (b < E) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = pm_row(r, lane);
          if (o < N3) logits[b * N3 + o] = o3[r] + b3[o];
        }
      }
    }
  }
}

int64_t policy_packed_floats(int D) { return pm_packed_floats(D / 2 + 1); }

hipError_t launch_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                              const float* b3, int D, int N3, float* P, hipStream_t st) {
  const int K1 = D / 2 + 1;  // ceil((D + 1) / 2): observation + the bias input
  const int64_t total = pm_packed_floats(K1);
  const int grid = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
  k_policy_pack<<<grid, 256, 0, st>>>(W1, b1, W2, b2, W3, b3, D, N3, K1, P);
  return hipGetLastError();
}

template <int K1>
static hipError_t launch_fwd_t(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                               hipStream_t st) {
  const int64_t tiles = (E + 31) / 32;
  // persistent: at most one 4-wave workgroup per CU (one wave per SIMD), >= 1 tile per wave
  static int cus = 0;  // CU count of the (single) device this process drives, queried once
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int64_t want = (tiles + 3) / 4;
  const int grid = (int)(want < cus ? want : cus);
  if (N3 <= 16) k_policy_forward<K1, true><<<grid, 256, 0, st>>>(P, obs, E, D, N3, logits);
  else k_policy_forward<K1, false><<<grid, 256, 0, st>>>(P, obs, E, D, N3, logits);
  return hipGetLastError();
}

hipError_t launch_policy_forward(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                                 hipStream_t st) {
  if (E <= 0) return hipSuccess;
  switch (D / 2 + 1) {
    case 1: return launch_fwd_t<1>(P, obs, E, D, N3, logits, st);
    case 2: return launch_fwd_t<2>(P, obs, E, D, N3, logits, st);
    case 3: return launch_fwd_t<3>(P, obs, E, D, N3, logits, st);
    case 4: return launch_fwd_t<4>(P, obs, E, D, N3, logits, st);
    case 5: return launch_fwd_t<5>(P, obs, E, D, N3, logits, st);
    case 6: return launch_fwd_t<6>(P, obs, E, D, N3, logits, st);
    case 7: return launch_fwd_t<7>(P, obs, E, D, N3, logits, st);
    case 8: return launch_fwd_t<8>(P, obs, E, D, N3, logits, st);
    case 9: return launch_fwd_t<9>(P, obs, E, D, N3, logits, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mh
