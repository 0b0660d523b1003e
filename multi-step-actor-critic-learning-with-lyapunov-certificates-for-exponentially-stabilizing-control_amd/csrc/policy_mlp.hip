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
#include <type_traits>

#include "rollout.h"
#include "policy_x3.h"

namespace mh {


// One thread per packed float.
__global__ __launch_bounds__(256) void k_policy_pack(const float* __restrict__ W1, const float* __restrict__ b1,
                                                     const float* __restrict__ W2, const float* __restrict__ b2,
                                                     const float* __restrict__ W3, const float* __restrict__ b3,
                                                     int D, int N3, int K1, float* __restrict__ P) {
  const int64_t total = pm_off_w2x6(K1);  // the f32 regions (the split copies have their own packers)
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
  // the atomic-max slots of k_policy_scales (which runs next) start from zero. Written here, not by a
  // hipMemsetAsync: captured into a HIP graph, that memset node left the slots dirty from the second
  // replay on (measured: garbage scales -> logits off by 1e-2 on replays >= 2)
  if (blockIdx.x == 0 && threadIdx.x < 8) P[pm_off_scal(K1) + threadIdx.x] = 0.0f;
}

// Exact three-way bf16 split: a = hi + mid + lo with every part a bf16 (round-to-nearest-even
// each time; the two remainders are exact in f32 and the last one has at most 8 significant bits,
// so the sum is exact for normal a).
__device__ __forceinline__ void split3(float a, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)a;
  const float r1 = a - (float)hi;
  mid = (__bf16)r1;
  lo = (__bf16)(r1 - (float)mid);
}

__global__ __launch_bounds__(256) void k_policy_pack_x6(const float* __restrict__ W2, int K1, float* __restrict__ P) {
  __bf16* dst = reinterpret_cast<__bf16*>(P + pm_off_w2x6(K1));
  const int64_t total = PM_X6_FLOATS * 2;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int j = (int)(q & 7), l = (int)((q >> 3) & 63);
    const int64_t f = q >> 9;  // fragment index over all chunks
    const int split = (int)(f % 3), s = (int)((f / 3) % 2), ob = (int)((f / 6) % PM_NB), ib = (int)(f / (6 * PM_NB));
    const int k = ib * 32 + (j & 3) + 8 * (j >> 2) + 16 * s + 4 * (l >> 5);
    __bf16 parts[3];
    split3(W2[(int64_t)(ob * 32 + (l & 31)) * PM_H + k], parts[0], parts[1], parts[2]);
    dst[q] = parts[split];
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

// ----------------------------------------------------------------------------------------------
// Split-bf16 variant: layer 2 (97 % of the f32 kernel's MFMA cycles) on v_mfma_f32_32x32x16_bf16
// with f32 accuracy. Each f32 operand is split exactly into three bf16 (split3); of the nine
// partial products the six with combined weight >= 2^-18 are accumulated
//     lo*hi, hi*lo, mid*mid, mid*hi, hi*mid, hi*hi        (smallest first)
// and the dropped three are <= 2^-26 |w x|, below f32 rounding: per product the result is
// f32-accurate, at 6 x 32 = 192 MFMA cycles per 32x32x16 step instead of 8 x 64 = 512 for the
// same products on v_mfma_f32_32x32x2_f32 (2.7x fewer matrix cycles for layer 2).
//   * the layer-1 accumulator feeds the bf16 MFMA as its B operand in place: registers
//     8 s .. 8 s + 7 of a 32x32 accumulator are k-step s of the next MFMA (the A operand is
//     packed to that k order, pm_off_w2x6);
//   * loop order ib (layer-2 input block) outer, ob inner: each wave owns NT = 2 env tiles
//     (64 envs), i.e. 16 f32x16 layer-2 accumulators (the 256 AGPRs); layer 1 of block ib is
//     computed and split just before its phase (2 x 16 accumulator values per lane);
//   * the W2 splits (384 KB) go through LDS: chunk ib (48 KB) is staged with
//     global_load_lds_dwordx4 (12 per wave) one phase ahead, double buffered (96 KB), and serves
//     the workgroup's 4 waves x 2 tiles (L2 -> LDS at 8 B/clk/CU); each fragment read from LDS
//     (two steps ahead) feeds 12 MFMAs;
//   * layer 3 is folded into the last phase: output block ob's accumulators are final after its
//     step (ob, 1) and go straight through layer 3, so they die there.
// Measured (tools/policy_bench.py, E = 65,536): 57-60 us vs 84-88 us for the all-f32 kernel.
// The layer-2 MFMA stream alone (no staging, barrier or layer 1) takes ~46 us: under a full
// chip of bf16 MFMAs on random data the clock drops to ~1.45 GHz (tools/mfma_rate.hip:
// 32 shader cycles but 20-22 ns per v_mfma_f32_32x32x16_bf16), so the 6 products cost more
// wall time per useful f32 flop than their cycle count suggests.
// Layers 1 and 3 stay f32 MFMA (as in k_policy_forward). N3 <= 16 only (L3B4 epilogue).
constexpr int PM_X6_TPW = 2;  // env tiles per wave: each W2 fragment read from LDS feeds 12 MFMAs

template <int K1, int NT>
__global__ __launch_bounds__(256, 1) void k_policy_forward_x6(const float* __restrict__ P,
                                                             const float* __restrict__ obs, int64_t E, int D, int N3,
                                                             float* __restrict__ logits) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  constexpr int FPW = PM_X6_FRAGS / 4;  // fragments each wave stages per chunk
  __shared__ uint4 lds[2][PM_X6_FRAGS * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ntiles = (E + 31) / 32;
  const int64_t per_round = (int64_t)gridDim.x * 4 * NT;  // tiles per round over the grid
  const float* W1p = P;
  const float* b2p = P + pm_off_b2(K1);
  const f32x4* W3p = reinterpret_cast<const f32x4*>(P + pm_off_w3(K1));
  const float* b3 = P + pm_off_b3(K1);
  const uint4* W2g = reinterpret_cast<const uint4*>(P + pm_off_w2x6(K1));

  auto load_obs = [&](int64_t t, float* xo) {
    const int64_t brow = min(min(t, ntiles - 1) * 32 + (lane & 31), E - 1);  // padded rows: the last env
#pragma unroll
    for (int s = 0; s < K1; ++s) {
      const int k = 2 * s + (lane >> 5);
      xo[s] = k < D ? obs[brow * D + k] : (k == D ? 1.0f : 0.0f);
    }
  };
  auto stage = [&](int ib, int buf) {  // this wave's 12 of the chunk's 48 fragments -> LDS
    const uint4* src = W2g + (int64_t)ib * PM_X6_FRAGS * 64;
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      const int f = w * FPW + i;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + f * 64 + lane),
                                       (void __attribute__((address_space(3)))*)(&lds[buf][f * 64]), 16, 0, 0);
    }
  };
  auto split_into = [&](float v, bf16x8* ph, bf16x8* pm, bf16x8* pl, int idx) {
    __bf16 a, b, c;
    split3(fmaxf(v, 0.0f), a, b, c);
    ph[idx >> 3][idx & 7] = a;
    pm[idx >> 3][idx & 7] = b;
    pl[idx >> 3][idx & 7] = c;
  };

  int64_t t0 = ((int64_t)blockIdx.x * 4 + w) * NT;  // this wave's first tile in the round
  int64_t wg0 = (int64_t)blockIdx.x * 4 * NT;       // the workgroup's first tile (uniform)
  if (wg0 >= ntiles) return;                         // whole workgroup idle (uniform)
  stage(0, 0);
  int buf = 0;
  float w1c[K1];  // layer-1 fragments of the next block to compute (loaded a phase ahead)
#pragma unroll
  for (int s = 0; s < K1; ++s) w1c[s] = W1p[(1 * K1 + s) * 64 + lane];
  float xo[NT][K1], xn[NT][K1];
  bf16x8 xh[NT][2], xm[NT][2], xl[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    load_obs(t0 + t, xo[t]);
    f32x16 h = {};
#pragma unroll
    for (int s = 0; s < K1; ++s) h = __builtin_amdgcn_mfma_f32_32x32x2f32(W1p[s * 64 + lane], xo[t][s], h, 0, 0, 0);
#pragma unroll
    for (int v = 0; v < 16; ++v) split_into(h[v], xh[t], xm[t], xl[t], v);
  }
  for (; wg0 < ntiles; wg0 += per_round, t0 += per_round) {
    const bool more = wg0 + per_round < ntiles;
    if (more) {
#pragma unroll
      for (int t = 0; t < NT; ++t) load_obs(t0 + per_round + t, xn[t]);  // next round's tiles
    }
    // the bias and W3 fragments are the same every round: launder the pointers so the compiler
    // re-loads them per round (L2 hits) instead of hoisting 256 registers of invariants
    int zero = 0;
    asm volatile("" : "+s"(zero));
    const float* b2r = b2p + zero;
    const f32x4* W3r = W3p + zero;
    f32x16 acc[NT][PM_NB];
#pragma unroll
    for (int ob = 0; ob < PM_NB; ++ob) {  // layer-2 bias as the accumulators' start
      const f32x4* bb = reinterpret_cast<const f32x4*>(b2r + (ob * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 bq = bb[q];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[t][ob][4 * q + j] = bq[j];
      }
    }
    f32x16 o3[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) o3[t] = f32x16{};
    // one block ib of layer 2 for the wave's tiles; in the last block (fold) each output block's
    // accumulator is final after its step (ob, 1) and goes straight through layer 3 (f32,
    // v_mfma_f32_16x16x1_4b as k_policy_forward's L3B4 path), so it dies there
    auto phase = [&](int ib, bool fold) {
      const bool has_next = ib < PM_NB - 1 || more;
      const int nib = (ib + 1) & (PM_NB - 1);
      if (ib > 0) {  // layer 1 of block ib for the tiles (block 0 was done a round ahead)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x16 h = {};
#pragma unroll
          for (int s = 0; s < K1; ++s) h = __builtin_amdgcn_mfma_f32_32x32x2f32(w1c[s], xo[t][s], h, 0, 0, 0);
#pragma unroll
          for (int v = 0; v < 16; ++v) split_into(h[v], xh[t], xm[t], xl[t], v);
        }
      }
#pragma unroll
      for (int s = 0; s < K1; ++s) w1c[s] = W1p[(nib * K1 + s) * 64 + lane];  // a phase ahead
      __syncthreads();  // chunk ib has landed (every wave drained its loads); buf ^ 1 is free
      if (has_next) stage(nib, buf ^ 1);
      const uint4* L = lds[buf] + lane;
      // W2 fragments read two steps ahead (a 3-slot ring): an LDS read has 2 steps of MFMAs
      uint4 ring[3][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        ring[0][p] = L[p * 64];
        ring[1][p] = L[(3 + p) * 64];
      }
#pragma unroll
      for (int st = 0; st < 2 * PM_NB; ++st) {
        const int ob = st >> 1, s = st & 1;
        if (st + 2 < 2 * PM_NB) {
#pragma unroll
          for (int p = 0; p < 3; ++p) ring[(st + 2) % 3][p] = L[((st + 2) * 3 + p) * 64];
        }
        const uint4* cur = ring[st % 3];
        f32x4 w3f[4];
        if (fold && s == 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) w3f[q] = W3r[(ob * 4 + q) * 64 + lane];
        }
        const bf16x8 wh = __builtin_bit_cast(bf16x8, cur[0]);
        const bf16x8 wm = __builtin_bit_cast(bf16x8, cur[1]);
        const bf16x8 wl = __builtin_bit_cast(bf16x8, cur[2]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x16 a = acc[t][ob];
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xm[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, xh[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xm[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh[t][s], a, 0, 0, 0);
          acc[t][ob] = a;
        }
        if (fold && s == 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int t = 0; t < NT; ++t)
                o3[t] = __builtin_amdgcn_mfma_f32_16x16x1f32(w3f[q][j], fmaxf(acc[t][ob][4 * q + j], 0.0f), o3[t], 0,
                                                             0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // one step at a time: bounded live fragments
      }
      buf ^= 1;
    };
#pragma unroll 1
    for (int ib = 0; ib < PM_NB - 1; ++ib) phase(ib, false);
    phase(PM_NB - 1, true);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < K1; ++s) xo[t][s] = xn[t][s];
    if (more) {  // block 0 of the next round's tiles
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x16 h = {};
#pragma unroll
        for (int s = 0; s < K1; ++s) h = __builtin_amdgcn_mfma_f32_32x32x2f32(W1p[s * 64 + lane], xo[t][s], h, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) split_into(h[v], xh[t], xm[t], xl[t], v);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int64_t tile = t0 + t;
      if (tile < ntiles) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int64_t b = tile * 32 + (lane & 15) + 16 * hh;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int oo = 4 * (lane >> 4) + q;
            if (b < E && oo < N3) logits[b * N3 + oo] = (o3[t][4 * hh + q] + o3[t][4 * hh + 8 + q]) + b3[oo];
          }
        }
      }
    }
  }
  __syncthreads();  // no LDS-DMA outstanding when the workgroup retires
}

// ----------------------------------------------------------------------------------------------
// Split-f16 variant: all three layers on v_mfma_f32_32x32x16_f16 with THREE partial products per
// operand pair. f16 carries 11 significant bits (bf16: 8), so a two-way split a = hi + lo holds 22
// bits; keeping hi*hi, hi*lo, lo*hi drops lo*lo (<= 2^-22 |w x|), and the split residual is
// <= 2^-22 |a| per operand: every product is within ~3 * 2^-22 = 7e-7 of exact (f32: 6e-8 per
// rounding; the north star allows 1e-5). f16's narrow exponent range is handled by power-of-two
// scaling, exact in f32: each layer's weights by sw_l (pack time, max |W_l| * sw_l <= 2^14) and
// each env's input column of each layer by a per-env power of two from a bound on its magnitude
// (obs: max |obs|; H1: R1 max(1, max |obs|); H2: R2 max(1, bound(H1))), so every split operand is
// <= 2^14 whatever the observation; accumulators are unscaled exactly (power-of-two products) and
// the biases join after the unscaling (b1 rides in the MFMA as the weight of a constant input).
// The splits' subnormal floor is 2^-25 in scaled units, i.e. <= 2^-39 of the operand bound.
// Layer 2 as k_policy_forward_x6 (LDS-staged W2 chunks, NT = 2 tiles per wave, double-buffered,
// read two steps ahead) with 32 instead of 48 fragments per chunk and half the MFMAs; layer 1 is
// 3 MFMAs per 32-row block (K = 16 covers obs + bias for D <= 15); layer 3 is folded into the
// last phase: output block ob's accumulators are final after its step (ob, 1), go through bias,
// ReLU and the split, and into 2 x 3 16x16x32 MFMAs against W3x3 staged once per kernel in LDS
// (policy_x3.h pm_l3_row_half: N3 <= 8, the policy head 2A of every env; wider heads take the
// f32 kernel).
// The raw magnitudes behind the scales: [0] max |W1, b1|, [1] max |W2|, [2] max |W3|,
// [3] R1 = max_k (sum_j |W1[k][j]| + |b1[k]|), [4] R2 = max_o (sum_k |W2[o][k]| + |b2[o]|).
// PM_SC_WG workgroups of 8 waves, one row of W2 per wave (a float4 per lane, wave max / sum by
// butterflies), W1 row / W3 column of the same hidden unit on its lanes; each workgroup stores its
// five maxima to the partial slots scal[8 + 5 wg + q] with plain stores (no atomics: 256 workgroups
// combining by atomic max on five words serialised at the L2, 17.5 us; one workgroup alone took
// 11 us, 8 workgroups of 16 waves with two rows per wave 6.5 us); k_policy_pack_x3 reduces them.
__global__ __launch_bounds__(512) void k_policy_scales(const float* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       const float* __restrict__ W3, int D, int N3, int K1,
                                                       float* __restrict__ P) {
  static_assert(PM_SC_WG * 8 == PM_H, "one W2 row per wave");
  __shared__ float red[5][8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int row = blockIdx.x * 8 + wv;
  const float4 x = reinterpret_cast<const float4*>(W2 + (int64_t)row * PM_H)[lane];
  // hidden unit `row`: its W1 row on lanes j < D, its W3 column on lanes 32 + o, o < N3 — one
  // load per lane, all in flight together (a serial per-element loop on one lane waited out
  // ~40 L2 latencies per wave: 12 us for the kernel)
  const int j = lane & 31;
  const float u1 = lane < 32 && j < D ? fabsf(W1[(int64_t)row * D + j]) : 0.0f;
  const float u3 = lane >= 32 && j < N3 ? fabsf(W3[(int64_t)j * PM_H + row]) : 0.0f;
  const float bb1 = fabsf(b1[row]), bb2 = fabsf(b2[row]);
  const float a = fabsf(x.x), b = fabsf(x.y), c = fabsf(x.z), d = fabsf(x.w);
  float m2 = fmaxf(fmaxf(a, b), fmaxf(c, d)), s2 = (a + b) + (c + d);
  float m1 = u1, r1 = u1, m3 = u3;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m2 = fmaxf(m2, __shfl_xor(m2, off, 64));
    s2 += __shfl_xor(s2, off, 64);
    m1 = fmaxf(m1, __shfl_xor(m1, off, 64));
    r1 += __shfl_xor(r1, off, 64);
    m3 = fmaxf(m3, __shfl_xor(m3, off, 64));
  }
  if (lane == 0) {
    red[0][wv] = fmaxf(m1, bb1);
    red[1][wv] = m2;
    red[2][wv] = m3;
    red[3][wv] = r1 + bb1;
    red[4][wv] = s2 + bb2;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    float m = 0.0f;
#pragma unroll
    for (int w = 0; w < 8; ++w) m = fmaxf(m, red[threadIdx.x][w]);
    P[pm_off_scal(K1) + 8 + 5 * blockIdx.x + threadIdx.x] = m;
  }
}

// The final magnitudes from k_policy_scales' partials (every workgroup of k_policy_pack_x3 forms
// them; its workgroup 0 stores them to scal[0..4] for the forward kernel)
__device__ __forceinline__ void pm_reduce_scales(float* P, int K1, float* out5) {
  __shared__ float s5[5];
  float* scal = P + pm_off_scal(K1);
  if (threadIdx.x < 5) {
    float m = 0.0f;
#pragma unroll
    for (int w = 0; w < PM_SC_WG; ++w) m = fmaxf(m, scal[8 + 5 * w + threadIdx.x]);
    s5[threadIdx.x] = m;
    if (blockIdx.x == 0) scal[threadIdx.x] = m;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 5; ++q) out5[q] = s5[q];
}

// The split-f16 operands, one thread per (fragment pair, lane): the lane's eight weights of a
// fragment (two 16-byte runs of a W2 / W3 row, or eight W1 entries), scaled by the layer's power
// of two and split, stored as the hi and the lo fragment's 16-byte records (the split index is
// the fragment index's low bit in every region). Fragment pairs: W2x3 PM_NB * 16 (pair P: k-step
// P & 1, output block (P >> 1) % PM_NB, input block P / (2 PM_NB)), W1x3 PM_NB (pair = block),
// W3x3 PM_NB * 2 (k-step P & 1, output block P >> 1).
// with_bias: also the f32 layer-2 / layer-3 bias regions the split-f16 forward reads (k_policy_pack's
// layout), so the default kernel needs no f32 pack launch
constexpr int PM_X3_PAIRS_W2 = PM_NB * 16, PM_X3_PAIRS_W1 = PM_NB, PM_X3_PAIRS_W3 = PM_NB * 2;
constexpr int PM_X3_PACK_THREADS = (PM_X3_PAIRS_W2 + PM_X3_PAIRS_W1 + PM_X3_PAIRS_W3) * 64;
static_assert(PM_X3_PAIRS_W2 * 2 * 64 * 4 == PM_X3_FLOATS && PM_X3_PAIRS_W1 * 2 * 64 * 4 == PM_X3_W1_FLOATS &&
                  PM_X3_PAIRS_W3 * 2 * 64 * 4 == PM_X3_W3_FLOATS,
              "fragment pairs cover the split regions");
__global__ __launch_bounds__(256) void k_policy_pack_x3(const float* __restrict__ W1, const float* __restrict__ b1,
                                                        const float* __restrict__ W2, const float* __restrict__ b2,
                                                        const float* __restrict__ W3, const float* __restrict__ b3,
                                                        int D, int N3, int K1, int with_bias, float* __restrict__ P) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int l = t & 63, pr = t >> 6;
  // the weights first (independent of the scales): their loads and the partial-scale loads of
  // pm_reduce_scales are in flight together
  float x[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  int region = -1, idx = 0;
  if (pr < PM_X3_PAIRS_W2) {
    const int s = pr & 1, ob = (pr >> 1) % PM_NB, ib = pr / (2 * PM_NB);
    const int k0 = ib * 32 + 16 * s + 4 * (l >> 5);  // elements j: k0 + (j & 3) + 8 (j >> 2)
    const float* src = W2 + (int64_t)(ob * 32 + (l & 31)) * PM_H + k0;
    const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 8);
    x[0] = x0.x; x[1] = x0.y; x[2] = x0.z; x[3] = x0.w; x[4] = x1.x; x[5] = x1.y; x[6] = x1.z; x[7] = x1.w;
    region = 1;
    idx = pr;
  } else if (pr < PM_X3_PAIRS_W2 + PM_X3_PAIRS_W1) {
    const int blk = pr - PM_X3_PAIRS_W2, row = blk * 32 + (l & 31);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * (l >> 5) + j;
      x[j] = k < D ? W1[(int64_t)row * D + k] : (k == D ? b1[row] : 0.0f);
    }
    region = 0;
    idx = blk;
  } else if (pr < PM_X3_PAIRS_W2 + PM_X3_PAIRS_W1 + PM_X3_PAIRS_W3) {
    // the 16x16x32 A operand (policy_x3.h pm_l3_row_half): row l & 15, k-group l >> 4
    const int p3 = pr - PM_X3_PAIRS_W2 - PM_X3_PAIRS_W1;
    const int s = p3 & 1, ob = p3 >> 1, o = l & 7;
    if (pm_l3_row_half(l) && o < N3) {
      const float* src = W3 + (int64_t)o * PM_H + ob * 32 + 16 * s + 4 * (l >> 5);
      const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 8);
      x[0] = x0.x; x[1] = x0.y; x[2] = x0.z; x[3] = x0.w; x[4] = x1.x; x[5] = x1.y; x[6] = x1.z; x[7] = x1.w;
    }
    region = 2;
    idx = p3;
  }
  if (with_bias) {  // b2 as [blk][lane][16] (pm_row order) and b3 (N3 values, zero padded)
    const int nb2 = (int)(pm_off_w3(K1) - pm_off_b2(K1));
    for (int o = t; o < nb2 + 32; o += gridDim.x * 256) {
      if (o < nb2) {
        const int r = o % 16, ll = (o / 16) % 64, blk = o / (16 * 64);
        P[pm_off_b2(K1) + o] = b2[blk * 32 + pm_row(r, ll)];
      } else {
        const int i = o - nb2;
        P[pm_off_b3(K1) + i] = i < N3 ? b3[i] : 0.0f;
      }
    }
  }
  float raw5[5];
  pm_reduce_scales(P, K1, raw5);  // (a workgroup barrier: every thread of the workgroup reaches it)
  if (region < 0) return;
  const PmScales sc = pm_scales(raw5);
  const float sw = sc.sw[region];
  uint4* dst = reinterpret_cast<uint4*>(P + (region == 1 ? pm_off_w2x3(K1) : region == 0 ? pm_off_w1x3(K1)
                                                                                          : pm_off_w3x3(K1))) +
               (int64_t)idx * 128;
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    _Float16 h0, l0, h1, l1;
    split2h(x[2 * q] * sw, h0, l0);
    split2h(x[2 * q + 1] * sw, h1, l1);
    hw[q] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    lw[q] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  }
  dst[l] = uint4{hw[0], hw[1], hw[2], hw[3]};       // fragment 2 idx: hi
  dst[64 + l] = uint4{lw[0], lw[1], lw[2], lw[3]};  // fragment 2 idx + 1: lo
}

// WAVES = 4 (one wave per SIMD, NT = 2 tiles each) or 8 (two waves per SIMD, NT = 1: the
// accumulators fit in 128 AGPRs, so two waves share each SIMD and hide each other's VALU and
// barrier time behind MFMAs). Either way a workgroup covers 8 tiles per staged W2 chunk.
template <int NT, int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES / 4, WAVES / 4)))
void k_policy_forward_x3(const float* __restrict__ P,
                                                             const float* __restrict__ obs, int64_t E, int D, int N3,
                                                             int K1, float* __restrict__ logits) {
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  constexpr int FPW = PM_X3_FRAGS / WAVES;  // W2x3 fragments each wave stages per chunk
  constexpr int FOPW = PM_NB * 4 / WAVES;  // fold-operand records per wave (per array)
  // two distinct LDS arrays (not one [2][...]): with the buffer known at compile time in every
  // phase, alias analysis proves the next chunk's LDS-DMA writes disjoint from this phase's
  // ds_reads, so the reads do not wait for the staging to land
  __shared__ uint4 lds0[PM_X3_FRAGS * 64];
  __shared__ uint4 lds1[PM_X3_FRAGS * 64];
  // the fold operands, staged once per kernel: W3x3 [ob][s][split][lane] and the layer-2 bias
  // as [ob][q][lane] (lane-contiguous 16-B records)
  __shared__ uint4 lds_w3[PM_NB * 4 * 64];
  __shared__ uint4 lds_b2[PM_NB * 4 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ntiles = (E + 31) / 32;
  const int64_t per_round = (int64_t)gridDim.x * WAVES * NT;
  const float* b3 = P + pm_off_b3(K1);
  const uint4* W2g = reinterpret_cast<const uint4*>(P + pm_off_w2x3(K1));
  const uint4* W1g = reinterpret_cast<const uint4*>(P + pm_off_w1x3(K1));
  const float* scal = P + pm_off_scal(K1);
  const PmScales scs = pm_scales(scal);
  const float isw1 = scs.isw[0], isw2 = scs.isw[1], isw3 = scs.isw[2], R1 = scs.R1, R2 = scs.R2;

  // per lane: the 8 inputs k = 8 (lane >> 5) + j of env column lane & 31 (obs, then the
  // constant-1 bias input at k = D), scaled by 2^ex[0] and split; ex = the env's three exponents
  auto load_split_obs = [&](int64_t t, f16x8& xh, f16x8& xl, int* ex) {
    const int64_t brow = min(min(t, ntiles - 1) * 32 + (lane & 31), E - 1);  // padded rows: the last env
    float x[8];
    float m = 1.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * (lane >> 5) + j;
      x[j] = k < D ? obs[brow * D + k] : (k == D ? 1.0f : 0.0f);
      m = fmaxf(m, fabsf(x[j]));
    }
    m = fmaxf(m, __shfl_xor(m, 32));  // lanes l and l ^ 32 hold the same env
    ex[0] = pm_scale_exp(m);
    const float b1v = R1 * m;
    ex[1] = pm_scale_exp(b1v);
    ex[2] = pm_scale_exp(R2 * fmaxf(1.0f, b1v));
    const float sx = pm_pow2(ex[0]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 a, b;
      split2h(x[j] * sx, a, b);
      xh[j] = a;
      xl[j] = b;
    }
  };
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the wave index, in an SGPR
  auto stage = [&](int ib, uint4* dstbuf) {
    // scalar base + lane offset + immediate fragment offset; the laundered base keeps the compiler
    // from precomputing (and spilling) one 64-bit address per fragment and phase
    const uint4* src = W2g + ((int64_t)ib * PM_X3_FRAGS + wu * FPW) * 64;
    asm volatile("" : "+s"(src));
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + i * 64 + lane),
                                       (void __attribute__((address_space(3)))*)(&dstbuf[(wu * FPW + i) * 64]), 16,
                                       0, 0);
    }
  };
  // layer 1 of one 32-row block for one tile: 3 MFMAs (l1_mfma), then ReLU, rescale to the H1
  // exponent and split into the layer-2 B operands, registers 8 s .. 8 s + 7 = k-step s (l1_split)
  auto l1_mfma = [&](const uint4* wf, const f16x8& xh, const f16x8& xl) {
    const f16x8 wh = __builtin_bit_cast(f16x8, wf[0]), wl = __builtin_bit_cast(f16x8, wf[1]);
    f32x16 h = {};
    h = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, h, 0, 0, 0);
    h = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, h, 0, 0, 0);
    h = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, h, 0, 0, 0);
    return h;
  };
  auto l1_split = [&](const f32x16& h, float rescale, f16x8* ph, f16x8* pl) {
    uint32_t hp[8], lp[8];
#pragma unroll
    for (int p = 0; p < 8; ++p)  // rescale (a power of two) commutes with the ReLU
      split2h_relu_scaled(h[2 * p], h[2 * p + 1], rescale, hp[p], lp[p]);
    ph[0] = __builtin_bit_cast(f16x8, uint4{hp[0], hp[1], hp[2], hp[3]});
    ph[1] = __builtin_bit_cast(f16x8, uint4{hp[4], hp[5], hp[6], hp[7]});
    pl[0] = __builtin_bit_cast(f16x8, uint4{lp[0], lp[1], lp[2], lp[3]});
    pl[1] = __builtin_bit_cast(f16x8, uint4{lp[4], lp[5], lp[6], lp[7]});
  };
  auto layer1 = [&](const uint4* wf, const f16x8& xh, const f16x8& xl, float rescale, f16x8* ph, f16x8* pl) {
    l1_split(l1_mfma(wf, xh, xl), rescale, ph, pl);
  };

  int64_t t0 = ((int64_t)blockIdx.x * WAVES + w) * NT;
  int64_t wg0 = (int64_t)blockIdx.x * WAVES * NT;
  if (wg0 >= ntiles) return;  // whole workgroup idle (uniform)
  {  // fold operands: 2 x 2,048 lane-16-B records over the waves
    const uint4* w3g = reinterpret_cast<const uint4*>(P + pm_off_w3x3(K1));
    const uint4* b2g = reinterpret_cast<const uint4*>(P + pm_off_b2(K1));
#pragma unroll
    for (int i = 0; i < FOPW; ++i) {
      const int r = w * FOPW + i;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(w3g + r * 64 + lane),
                                       (void __attribute__((address_space(3)))*)(&lds_w3[r * 64]), 16, 0, 0);
      // b2p is [ob][lane][16 floats]: lane-strided source, lane-contiguous destination
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(b2g + ((r >> 2) * 64 + lane) * 4 + (r & 3)),
                                       (void __attribute__((address_space(3)))*)(&lds_b2[r * 64]), 16, 0, 0);
    }
  }
  stage(0, lds0);
  uint4 w1c[2];  // layer-1 fragments of the next block (loaded a phase ahead)
  w1c[0] = W1g[(1 * 2 + 0) * 64 + lane];
  w1c[1] = W1g[(1 * 2 + 1) * 64 + lane];
  f16x8 xoh[NT], xol[NT];
  int ex[NT][3];
  f16x8 xh[NT][2], xl[NT][2];
  {
    uint4 w10[2] = {W1g[lane], W1g[64 + lane]};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      load_split_obs(t0 + t, xoh[t], xol[t], ex[t]);
      layer1(w10, xoh[t], xol[t], pm_pow2(ex[t][1] - ex[t][0]) * isw1, xh[t], xl[t]);
    }
  }
  for (; wg0 < ntiles; wg0 += per_round, t0 += per_round) {
    const bool more = wg0 + per_round < ntiles;
    float k23[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) k23[t] = isw2 * pm_pow2(ex[t][2] - ex[t][1]);
    // layer 2 accumulates onto its bias b2 * sw2 * 2^ex1 (set in phase 0, once lds_b2 is visible);
    // the H2 split is then relu(acc) * k23 (the fused sampler's expressions: the same bits)
    f32x16 acc[NT][PM_NB];
    // phase ib reads chunk ib from lds<ib & 1> and stages chunk ib + 1 into the other array
    auto phase = [&](auto bufc, int ib, bool fold) {
      constexpr int B = decltype(bufc)::value;
      uint4* cur_lds = B ? lds1 : lds0;
      uint4* nxt_lds = B ? lds0 : lds1;
      const bool has_next = ib < PM_NB - 1 || more;
      const int nib = (ib + 1) & (PM_NB - 1);
#ifndef MH_X3_NOBAR  // timing experiments only (tools/ab_libs.sh): parts compiled out
      // LDS DMA completes on vmcnt: drain this wave's share of chunk ib, then the barrier makes
      // the whole chunk (and the fold operands) visible to every wave
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      __syncthreads();
      if (has_next) stage(nib, nxt_lds);
#endif
      if (ib == 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float cb = pm_bias_unit(scs.sw[1], ex[t][1]);
#pragma unroll
          for (int ob = 0; ob < PM_NB; ++ob)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x4 bq = __builtin_bit_cast(f32x4, lds_b2[(ob * 4 + q) * 64 + lane]);
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[t][ob][4 * q + j] = bq[j] * cb;
            }
        }
      }
      // layer 1 of block ib + 1 is software-pipelined into this phase's MFMA stream (issued at
      // step 0, split at step 3, into a second operand set), so no wave idles on it at a barrier
      const bool pipe = !fold;
      f32x16 hn[NT];
      f16x8 xh2[NT][2], xl2[NT][2];
      const uint4* L = cur_lds + lane;
      uint4 ring[3][2];  // W2 fragments read two steps ahead
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        ring[0][p] = L[p * 64];
        ring[1][p] = L[(2 + p) * 64];
      }
#pragma unroll
      for (int st = 0; st < 2 * PM_NB; ++st) {
        const int ob = st >> 1, s = st & 1;
        if (st + 2 < 2 * PM_NB) {
#pragma unroll
          for (int p = 0; p < 2; ++p) ring[(st + 2) % 3][p] = L[((st + 2) * 2 + p) * 64];
        }
        const uint4* cur = ring[st % 3];
#ifndef MH_X3_NOL1
        if (pipe && st == 0) {
#pragma unroll
          for (int t = 0; t < NT; ++t) hn[t] = l1_mfma(w1c, xoh[t], xol[t]);
          if (ib + 2 < PM_NB) {  // fragments of block ib + 2, a phase ahead
            w1c[0] = W1g[((ib + 2) * 2 + 0) * 64 + lane];
            w1c[1] = W1g[((ib + 2) * 2 + 1) * 64 + lane];
          }
        }
        if (pipe && st == 3) {
#pragma unroll
          for (int t = 0; t < NT; ++t) l1_split(hn[t], pm_pow2(ex[t][1] - ex[t][0]) * isw1, xh2[t], xl2[t]);
        }
#endif
        uint4 w3f[4];
        if (fold && s == 1) {
#pragma unroll
          for (int q = 0; q < 4; ++q) w3f[q] = lds_w3[(ob * 4 + q) * 64 + lane];
        }
        const f16x8 wh = __builtin_bit_cast(f16x8, cur[0]);
        const f16x8 wl = __builtin_bit_cast(f16x8, cur[1]);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x16 a = acc[t][ob];
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl[t][s], a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh[t][s], a, 0, 0, 0);
          acc[t][ob] = a;
        }
        if (fold && s == 1) {  // H2 block ob is final: bias, ReLU, rescale, split, layer 3
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            // h2 * 2^e3 = relu(acc * (2^(e3 - e2) / sw2) + b2 * 2^e3): one packed fma per pair
            // (powers of two commute with the ReLU and with rounding)
            uint32_t hp[8], lp[8];
#pragma unroll
            for (int p = 0; p < 8; ++p)
              split2h_relu_scaled(acc[t][ob][2 * p], acc[t][ob][2 * p + 1], k23[t], hp[p], lp[p]);
            const f16x8 hh[2] = {__builtin_bit_cast(f16x8, uint4{hp[0], hp[1], hp[2], hp[3]}),
                                 __builtin_bit_cast(f16x8, uint4{hp[4], hp[5], hp[6], hp[7]})};
            const f16x8 hl[2] = {__builtin_bit_cast(f16x8, uint4{lp[0], lp[1], lp[2], lp[3]}),
                                 __builtin_bit_cast(f16x8, uint4{lp[4], lp[5], lp[6], lp[7]})};
            // layer 3 on 16x16x32 (policy_x3.h pm_l3_row_half); its accumulator lives in registers
            // 0..3 of acc[t][0] once block 0 has been folded (free from then on)
            f32x16 o = ob == 0 ? f32x16{} : acc[t][0];
            f32x4 o3 = {o[0], o[1], o[2], o[3]};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              const f16x8 vh = __builtin_bit_cast(f16x8, w3f[2 * ks]);
              const f16x8 vl = __builtin_bit_cast(f16x8, w3f[2 * ks + 1]);
              o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, hh[ks], o3, 0, 0, 0);
              o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, hl[ks], o3, 0, 0, 0);
              o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, hh[ks], o3, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = o3[i];
            acc[t][0] = o;
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one step at a time: bounded live fragments
      }
#ifndef MH_X3_NOL1
      if (pipe) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          xh[t][0] = xh2[t][0];
          xh[t][1] = xh2[t][1];
          xl[t][0] = xl2[t][0];
          xl[t][1] = xl2[t][1];
        }
      }
#endif
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
#pragma unroll 1
    for (int ib = 0; ib < PM_NB - 2; ib += 2) {
      phase(B0{}, ib, false);
      phase(B1{}, ib + 1, false);
    }
    phase(B0{}, PM_NB - 2, false);
    phase(B1{}, PM_NB - 1, true);
    // logits: registers 0..3 of acc[t][0] hold outputs 4 ((lane >> 4) & 1) + i of env column
    // pm_l3_env(lane), in units of sw3 * 2^ex[2] of that env (its exponents live on that env's lane)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int e = pm_l3_env(lane);
      const float iu = __shfl(isw3 * pm_pow2(-ex[t][2]), e);
      const int o0 = 4 * ((lane >> 4) & 1);
      const int64_t b = (t0 + t) * 32 + e;
      if (t0 + t < ntiles && b < E && o0 < N3) {
        if ((N3 & 3) == 0) {
          // one 16-byte store per lane (whole lines: 4-byte stores at the row stride wrote every
          // line 4 times, PMC WRITE_SIZE 9.5x the logits' bytes)
          const float4 bb = *reinterpret_cast<const float4*>(b3 + o0);
          *reinterpret_cast<float4*>(logits + b * N3 + o0) =
              make_float4(acc[t][0][0] * iu + bb.x, acc[t][0][1] * iu + bb.y, acc[t][0][2] * iu + bb.z,
                          acc[t][0][3] * iu + bb.w);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (o0 + i < N3) logits[b * N3 + o0 + i] = acc[t][0][i] * iu + b3[o0 + i];
        }
      }
    }
    if (more) {  // the next round's tiles (loaded here, not a round ahead: registers) and their block 0
      uint4 w10[2] = {W1g[lane], W1g[64 + lane]};
      w1c[0] = W1g[(1 * 2 + 0) * 64 + lane];
      w1c[1] = W1g[(1 * 2 + 1) * 64 + lane];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        load_split_obs(t0 + per_round + t, xoh[t], xol[t], ex[t]);
        layer1(w10, xoh[t], xol[t], pm_pow2(ex[t][1] - ex[t][0]) * isw1, xh[t], xl[t]);
      }
    }
  }
  __syncthreads();  // no LDS-DMA outstanding when the workgroup retires
}

int64_t policy_packed_floats(int D) { return pm_packed_floats(D / 2 + 1); }

// MH_POLICY_KERNEL (A/B measurements): f32 = the all-f32 kernel (0), x6 = split-bf16 layer 2 (1);
// default split-f16 (x3, 2)
static int policy_mode() {
  static int mode = -1;
  if (mode < 0) {
    const char* m = getenv("MH_POLICY_KERNEL");
    mode = (m && m[0] == 'f') ? 0 : ((m && m[0] == 'x' && m[1] == '6') ? 1 : 2);
  }
  return mode;
}

hipError_t launch_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                              const float* b3, int D, int N3, float* P, hipStream_t st) {
  const int K1 = D / 2 + 1;  // ceil((D + 1) / 2): observation + the bias input
  // k_policy_scales / k_policy_pack_x3 read 16-byte runs of W2 and W3 rows
  if ((reinterpret_cast<uintptr_t>(W2) | reinterpret_cast<uintptr_t>(W3)) & 15) return hipErrorInvalidValue;
  const int64_t total = pm_off_w2x6(K1);
  const int grid = (int)((total + 255) / 256 < 1024 ? (total + 255) / 256 : 1024);
  // the default kernel (split-f16, layer 3 on 8 + 8 output rows) reads only b2 / b3 in f32
  const bool split_only = policy_mode() == 2 && D <= 15 && N3 <= 8;
  if (!split_only) {
    k_policy_pack<<<grid, 256, 0, st>>>(W1, b1, W2, b2, W3, b3, D, N3, K1, P);
    if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
  }
  if (policy_mode() == 1) {  // the split-bf16 copy of W2 only for that (A/B) kernel
    k_policy_pack_x6<<<(int)(PM_X6_FLOATS * 2 / 256), 256, 0, st>>>(W2, K1, P);
    if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
  }
  k_policy_scales<<<PM_SC_WG, 512, 0, st>>>(W1, b1, W2, b2, W3, D, N3, K1, P);
  if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
  k_policy_pack_x3<<<(PM_X3_PACK_THREADS + 255) / 256, 256, 0, st>>>(W1, b1, W2, b2, W3, b3, D, N3, K1,
                                                                     split_only ? 1 : 0, P);
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
  const int mode = policy_mode();
  if (D <= 15 && N3 <= 8 && mode == 2) {  // K = 16 holds the observation and the bias input
    // default (round 4): one wave per SIMD with 2 tiles (k_policy_forward_x3<2, 4>, 512 registers,
    // nothing spilled); MH_POLICY_WAVES=8: two waves per SIMD with 1 tile each, whose 256-register
    // budget spilled 32 VGPRs to scratch in every phase — the 9x WRITE_SIZE of the logits' bytes
    // (profiles/r03_pmc_traffic_v4.json) was those spill stores, not the 16-byte logits rows. The
    // two measured equal at the kernel in round 2 (27.9-28.1 vs 27.9 us, profiles/r02_policy_waves4_ab.jsonl).
    static int w8 = -1;
    if (w8 < 0) {
      const char* v = getenv("MH_POLICY_WAVES");
      w8 = (v && atoi(v) == 8) ? 1 : 0;
    }
    const int64_t want3 = (tiles + 7) / 8;  // 8 tiles per workgroup either way
    const int grid3 = (int)(want3 < cus ? want3 : cus);
    if (w8) k_policy_forward_x3<1, 8><<<grid3, 512, 0, st>>>(P, obs, E, D, N3, K1, logits);
    else k_policy_forward_x3<2, 4><<<grid3, 256, 0, st>>>(P, obs, E, D, N3, K1, logits);
  } else if (N3 <= 16 && mode == 1) {
    static int tpw = 0;  // env tiles per wave (MH_POLICY_TPW, for A/B): default PM_X6_TPW
    if (tpw == 0) {
      const char* v = getenv("MH_POLICY_TPW");
      tpw = (v && atoi(v) == 1) ? 1 : PM_X6_TPW;
    }
    const int64_t want6 = (tiles + 4 * tpw - 1) / (4 * tpw);
    const int grid6 = (int)(want6 < cus ? want6 : cus);
    if (tpw == 1) k_policy_forward_x6<K1, 1><<<grid6, 256, 0, st>>>(P, obs, E, D, N3, logits);
    else k_policy_forward_x6<K1, 2><<<grid6, 256, 0, st>>>(P, obs, E, D, N3, logits);
  }
  else if (N3 <= 16) k_policy_forward<K1, true><<<grid, 256, 0, st>>>(P, obs, E, D, N3, logits);
  else k_policy_forward<K1, false><<<grid, 256, 0, st>>>(P, obs, E, D, N3, logits);
  return hipGetLastError();
}

hipError_t launch_policy_forward(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                                 hipStream_t st) {
  if (E <= 0) return hipSuccess;
  // rows of 4k logits are stored as 16-byte vectors (and b3 read as such from the packed block)
  if ((N3 & 3) == 0 && ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(P)) & 15))
    return hipErrorInvalidValue;
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
