// gemm.hip — f32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32) for the update phase's
// MLP layers (gfx950).
//
//   C[M][N] = act(op(A)[M][K] . op(B)[K][N] + bias[N])
//   op(A)(m, k) = TA ? A[k * lda + m] : A[m * lda + k]
//   op(B)(k, n) = TB ? B[n * ldb + k] : B[k * ldb + n]
//
// The actor / critic / Lyapunov MLPs of RL/apprfunc/mlp.py (nn.Linear 256 x 256 layers on a
// replay batch of B x n rows) run their forward (x W^T + b, ReLU/tanh epilogue), input gradient
// (g W) and weight gradient (g^T x) through this kernel instead of the BLAS library, whose
// kernels for these shapes are tuned for large problems: a 256 x 256 x 256 product ran on ONE
// workgroup for 47 us (profiles/r01_update_mix_v2.txt). Here every shape fills the chip:
//   * workgroup = 4 waves; wave tile 32 x 32 (2 x 2 accumulators of 16 x 16, 4 independent MFMA
//     chains: the 40-cycle dependent latency hides behind the 32-cycle issue);
//   * the 4 waves tile the workgroup's (32 WM) x (32 WN) block and split each 32-deep K chunk
//     KS = 4 / (WM WN) ways, reduced through LDS in fixed order;
//   * small output grids split K across workgroups (S-way): each writes its partial tile and
//     k_gemm_reduce sums the S partials in split order with the epilogue (deterministic);
//   * operands are staged through LDS per 32-deep chunk, the next chunk's global loads in flight
//     during the current chunk's MFMAs (register double buffer); the loads go through raw buffer
//     resources with 32-bit byte offsets (one VGPR per thread and operand instead of a 64-bit
//     address per element: 80-110 VGPRs, two workgroups per CU), and an element outside the
//     matrix gets an out-of-range offset, which the buffer unit returns as 0 (no branches).
// Numerics: each output is an f32 fma chain over k (MFMA f32 is exact per product, one rounding
// per accumulate), split partials added in order; agrees with the BLAS result to f32
// summation-order rounding.
#include <cstring>

#include "rollout.h"

namespace mh {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
  const float* A;
  const float* B;
  const float* bias;
  float* C;
  int64_t M, N, K, lda, ldb, ldc;
  int act;           // 0 identity, 1 ReLU, 2 tanh
  int S;             // K splits across workgroups
  int64_t kc_per;    // KC-deep chunks per split
  float* partial;    // [S][M][N] when S > 1
  // fused layer backward (launch_linear_backward): op(A) = act'(Y) * A elementwise (A = dy,
  // Y = the layer output, same leading dimension), and in the deep kernel the column sums of
  // that op(A) over K (the bias gradient): into db directly, or per split into dbp [S][M]
  const float* Y;
  int act_a;         // -1: A as is; 0 identity, 1 ReLU, 2 tanh
  float* db;
  float* dbp;        // [dbn][M] partial column sums (split-major, then column tile), or null
  int dbn;
  // grouped launches (the twin critics' layers as one launch): blockIdx.y = group q, and every
  // operand pointer of group q is its group-0 pointer + q x its stride (floats; 0 = shared)
  int64_t gsA, gsB, gsC, gsBias, gsY, gsPart, gsDb, gsDbp;
  // deep kernel, dbB set: dbp [S][N] holds the column sums of B over each split's K slice (the
  // bias gradient of a layer whose dW is computed transposed, x^T g: g is the B operand)
  int dbB;
};

// this workgroup's group (blockIdx.y) of a grouped launch: the operand pointers advanced
__device__ __forceinline__ void gemm_group(GemmArgs& g) {
  const int64_t q = blockIdx.y;
  if (q == 0) return;
  g.A += q * g.gsA;
  g.B += q * g.gsB;
  g.C += q * g.gsC;
  if (g.bias) g.bias += q * g.gsBias;
  if (g.Y) g.Y += q * g.gsY;
  if (g.partial) g.partial += q * g.gsPart;
  if (g.db) g.db += q * g.gsDb;
  if (g.dbp) g.dbp += q * g.gsDbp;
}

// g = dy * act'(y) exactly as k_act_grad_colsum forms it (mlp_grad.hip)
__device__ __forceinline__ float act_grad(float d, float t, int act) {
  if (act == 1) return t > 0.0f ? d : 0.0f;
  if (act == 2) return d * (1.0f - t * t);
  return d;
}

constexpr int KC = 32;  // K depth of one LDS stage

__device__ __forceinline__ float gemm_act(float v, int act) {
  if (act == 1) return v < 0.0f ? 0.0f : v;  // relu (NaN passes through, as torch.relu)
  if (act == 2) return tanhf(v);
  return v;
}

template <int WM, int WN, bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  constexpr int TM = 32 * WM, TN = 32 * WN, KS = 4 / (WM * WN);
  constexpr int LA = TM + 1, LB = TN + 1;
  constexpr int TILE_LDS = KC * LA + KC * LB;
  constexpr int RED_LDS = (KS - 1) * WM * WN * 1024;
  __shared__ float lds[TILE_LDS > RED_LDS ? TILE_LDS : RED_LDS];
  float* As = lds;
  float* Bs = lds + KC * LA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = (wave / WM) % WN, ks = wave / (WM * WN);
  const int64_t tiles_m = (g.M + TM - 1) / TM;
  const int64_t tiles = tiles_m * ((g.N + TN - 1) / TN);
  const int64_t tile = (int64_t)blockIdx.x % tiles;
  const int s = (int)((int64_t)blockIdx.x / tiles);
  const int64_t m0 = (tile % tiles_m) * TM, n0 = (tile / tiles_m) * TN;
  const int64_t nchunks = (g.K + KC - 1) / KC;
  const int64_t c_begin = (int64_t)s * g.kc_per;
  const int64_t c_end = c_begin + g.kc_per < nchunks ? c_begin + g.kc_per : nchunks;

  constexpr int NA = TM * KC / 256, NB = TN * KC / 256;
  float ra[NA], rb[NB];
  // element i of this thread's share of a chunk: (row/col within the tile, k within the chunk),
  // the contiguous global dimension running fastest across the lanes
  auto a_idx = [&](int i, int& m, int& k) {
    const int idx = tid + 256 * i;
    if (TA) { m = idx % TM; k = idx / TM; } else { k = idx % KC; m = idx / KC; }
  };
  auto b_idx = [&](int i, int& n, int& k) {
    const int idx = tid + 256 * i;
    if (TB) { k = idx % KC; n = idx / KC; } else { n = idx % TN; k = idx / TN; }
  };
  const __amdgpu_buffer_rsrc_t ra_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.A), (short)0, (int)((TA ? g.K : g.M) * g.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.B), (short)0, (int)((TB ? g.N : g.K) * g.ldb * 4), 0x00020000);
  constexpr int OOB = 0x7ffffff0;  // beyond every buffer (host keeps them below 2 GiB): reads 0
  auto load_chunk = [&](int64_t c) {
    const int k0 = (int)(c * KC);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int m, k;
      a_idx(i, m, k);
      const int gm = (int)m0 + m, gk = k0 + k;
      const int off = TA ? (gk * (int)g.lda + gm) * 4 : (gm * (int)g.lda + gk) * 4;
      const bool ok = gm < (int)g.M && gk < (int)g.K;
      ra[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra_rs, ok ? off : OOB, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int n, k;
      b_idx(i, n, k);
      const int gn = (int)n0 + n, gk = k0 + k;
      const int off = TB ? (gn * (int)g.ldb + gk) * 4 : (gk * (int)g.ldb + gn) * 4;
      const bool ok = gn < (int)g.N && gk < (int)g.K;
      rb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb_rs, ok ? off : OOB, 0, 0));
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if (c_begin < c_end) load_chunk(c_begin);
  for (int64_t c = c_begin; c < c_end; ++c) {
    __syncthreads();  // every wave is done reading the previous chunk
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int m, k;
      a_idx(i, m, k);
      As[k * LA + m] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int n, k;
      b_idx(i, n, k);
      Bs[k * LB + n] = rb[i];
    }
    __syncthreads();
    if (c + 1 < c_end) load_chunk(c + 1);
#pragma unroll
    for (int t = 0; t < KC / 4 / KS; ++t) {
      const int kr = (t * KS + ks) * 4 + (lane >> 4);
      const float a0 = As[kr * LA + wm * 32 + (lane & 15)];
      const float a1 = As[kr * LA + wm * 32 + 16 + (lane & 15)];
      const float b0 = Bs[kr * LB + wn * 32 + (lane & 15)];
      const float b1 = Bs[kr * LB + wn * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }

  // intra-workgroup K reduction (waves ks = 1.. add into ks = 0, in ks order)
  if constexpr (KS > 1) {
    __syncthreads();
    const int slot = wn * WM + wm;
    if (ks > 0) {
      float* r = lds + ((ks - 1) * WM * WN + slot) * 1024;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) r[((i * 2 + j) * 4 + q) * 64 + lane] = acc[i][j][q];
    }
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int w = 1; w < KS; ++w) {
        const float* r = lds + ((w - 1) * WM * WN + slot) * 1024;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[i][j][q] += r[((i * 2 + j) * 4 + q) * 64 + lane];
      }
    }
  }

  // C/D map of the 16x16 MFMA: column = lane & 15, row = 4 (lane >> 4) + q
  if (g.S == 1) {
    if (ks == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
          if (col >= g.N) continue;
          const float bv = g.bias ? g.bias[col] : 0.0f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + q;
            if (row < g.M) g.C[row * g.ldc + col] = gemm_act(g.bias ? acc[i][j][q] + bv : acc[i][j][q], g.act);
          }
        }
    }
    return;
  }

  // cross-workgroup split: this split's partial product, [S][M][N]; k_gemm_reduce finishes
  if (ks == 0) {
    float* part = g.partial + (int64_t)s * g.M * g.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (col >= g.N) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + q;
          if (row < g.M) part[row * g.N + col] = acc[i][j][q];
        }
      }
  }
}

// C = act(sum_s partial[s] + bias), splits added in order (and db = sum_s dbp[s] when set);
// block b of nb strides over the elements. transC: C is written transposed (C[col][row], ldc).
__device__ __forceinline__ void gemm_reduce_body(const GemmArgs& g, int64_t b, int64_t nb, bool transC = false) {
  const int64_t MN = g.M * g.N;
  if (g.dbp) {
    const int64_t dlen = g.dbB ? g.N : g.M;
    // dbn = splits x column tiles partials per output (64 for a 256 x 256 layer): sixteen loads
    // in flight per batch, added in partial order (a load-add loop paid one round trip per
    // partial: 18.8 us for this reduce)
    for (int64_t i = b * 256 + threadIdx.x; i < dlen; i += nb * 256) {
      float v = 0.0f;
      for (int s0 = 0; s0 < g.dbn; s0 += 16) {
        float x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = s0 + u < g.dbn ? g.dbp[(int64_t)(s0 + u) * dlen + i] : 0.0f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (s0 + u < g.dbn) v = (s0 + u == 0) ? x[u] : v + x[u];
      }
      g.db[i] = v;
    }
  }
  if (g.S <= 1) return;
  for (int64_t i = b * 256 + threadIdx.x; i < MN; i += nb * 256) {
    // eight partials in flight per batch (a load-add loop waits one round trip per split)
    float v = 0.0f;
    for (int s0 = 0; s0 < g.S; s0 += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = s0 + u < g.S ? g.partial[(int64_t)(s0 + u) * MN + i] : 0.0f;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s0 + u < g.S) v = (s0 + u == 0) ? x[u] : v + x[u];
    }
    const int64_t row = i / g.N, col = i - row * g.N;
    g.C[transC ? col * g.ldc + row : row * g.ldc + col] = gemm_act(g.bias ? v + g.bias[col] : v, g.act);
  }
}

__global__ __launch_bounds__(256) void k_gemm_reduce(GemmArgs g) {
  gemm_group(g);
  gemm_reduce_body(g, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------ tall products
// C = act(A[M][K] . op(B) + bias) for M >> N (the B x n = 5,120-row layers of the update:
// forward x W^T and input gradient g W, N = 256): the output is only M x 256, so a 64 x 64 or
// 128 x 128 tiling leaves most of the 256 CUs idle or runs two uneven rounds (the BLAS kernels
// for these shapes: 160 workgroups, 10.5-14 us). Here
//   * workgroup = 4 waves = (16 RB rows) x 64 columns, wave w owning columns 16w..16w+15 over all
//     RB row blocks (RB chosen so that the workgroup count fills whole rounds of 256 CUs: RB = 5,
//     80 x 64 tiles, 256 workgroups at M = 5,120, N = 256);
//   * 64-deep k chunks staged through LDS (double buffered, one barrier per chunk): the global
//     loads are row-contiguous float4 (a quarter-wave reads 256 B of one row), issued two
//     chunks ahead (two register sets), so each chunk's loads have two chunks' MFMAs (2 x 80
//     per wave) to land. Loading the MFMA
//     fragments straight from global memory instead puts 16 rows under every quarter-wave: 64
//     cache-line lookups per load instruction, and the vector L1 then takes 17 us for what the
//     MFMAs do in 5;
//   * fragments are read from LDS as float4 along k: MFMA j of a 16-deep group takes, in lane l,
//     k = 4 (l >> 4) + j for both operands (the k order inside a group is permuted, the same way
//     for A and B); op(B) is stored [n][k] in LDS whatever its global layout;
//   * blockIdx -> tile is XCD-aware: each XCD (blockIdx mod 8) gets whole row tiles, so an A row
//     block is fetched into one L2 only.
// K % 4 == 0, N % 64 == 0, 16-B aligned rows (A, op(B), C, bias), operands below 1 GiB.
constexpr int TK = 64;       // k depth of one LDS stage
constexpr int TLD = TK + 4;  // LDS row stride (floats): 16 rows of a b128 read hit distinct banks

template <int RB, bool TB, int NCH, bool AG>
__global__ __launch_bounds__(256) void k_gemm_tall(GemmArgs g, int tiles_n) {
  gemm_group(g);
  constexpr int RM = 16 * RB;
  constexpr int NA = RM * TK / 4 / 256;  // float4 loads of A per thread per chunk
  constexpr int NB = 64 * TK / 4 / 256;  // ... of op(B)
  static_assert(RM * TK / 4 % 256 == 0, "A chunk must split evenly over 256 threads");
  __shared__ float lds[2][(RM + 64) * TLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = (int)gridDim.x;
  const int bid = (int)blockIdx.x;
  const int t = (T % 8 == 0) ? (bid % 8) * (T / 8) + bid / 8 : bid;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * RM, n0 = tn * 64;
  const int M = (int)g.M, K = (int)g.K, lda = (int)g.lda, ldb = (int)g.ldb;
  const __amdgpu_buffer_rsrc_t ra_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.A), (short)0, (int)(g.M * g.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.B), (short)0, (int)((TB ? g.N : g.K) * g.ldb * 4), 0x00020000);
  // rows past M start at 1 GiB, beyond the buffer (the host keeps operands below 1 GiB): they
  // read 0 with no per-load select
  constexpr int OOB_ROW = 0x40000000;
  // this thread's float4 slots of a chunk: A slot f -> (row f / 16, k 4 (f % 16)); op(B) slot f
  // -> TB: (n f / 16, k 4 (f % 16)), !TB: (k f / 16, n 4 (f % 16))
  int aoff[NA], boff[NB];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    const int f = tid + 256 * s, m = m0 + f / 16;
    aoff[s] = m < M ? m * lda * 4 + (f % 16) * 16 : OOB_ROW;
  }
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int f = tid + 256 * s;
    boff[s] = TB ? ((n0 + f / 16) * ldb * 4 + (f % 16) * 16) : ((f / 16) * ldb * 4 + (n0 + 4 * (f % 16)) * 4);
  }
  // epilogue slots: float4 f = tid + 256 s of the RM x 64 tile -> (row f / 16, cols 4 (f % 16)..);
  // the bias of those columns (the same for every s) is fetched now, used after the last chunk
  const f32x4 bv = g.bias ? *reinterpret_cast<const f32x4*>(g.bias + n0 + 4 * (tid % 16)) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  f32x4 ra[2][NA], rb[2][NB];  // two chunks in flight ahead of the LDS stage
  f32x4 ry[AG ? 2 : 1][AG ? NA : 1];
  const __amdgpu_buffer_rsrc_t ry_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(AG && g.Y ? g.Y : g.A), (short)0, (int)(g.M * g.lda * 4), 0x00020000);
  auto load = [&](int c, int p) {
#ifdef MH_TALL_EXP_NOLOAD  // cost-attribution experiment only
    if (g.K > 0) return;
#endif
#pragma unroll
    for (int s = 0; s < NA; ++s)
      ra[p][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra_rs, aoff[s] + c * TK * 4, 0, 0));
    if constexpr (AG) {
      if (g.act_a > 0) {
#pragma unroll
        for (int s = 0; s < NA; ++s)
          ry[p][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry_rs, aoff[s] + c * TK * 4, 0, 0));
      }
    }
#pragma unroll
    for (int s = 0; s < NB; ++s)
      rb[p][s] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb_rs, boff[s] + (TB ? c * TK * 4 : c * TK * ldb * 4), 0, 0));
  };
  auto stage = [&](int c, int p) {
    if (NCH == 0 && c * TK + TK > K) {  // k >= K: A (and op(B) of TB) read the next row there
#pragma unroll
      for (int s = 0; s < NA; ++s)
        if (c * TK + 4 * ((tid + 256 * s) % 16) >= K) ra[p][s] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (TB) {
#pragma unroll
        for (int s = 0; s < NB; ++s)
          if (c * TK + 4 * ((tid + 256 * s) % 16) >= K) rb[p][s] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      // !TB: rows k >= K lie past the buffer end and read 0
    }
    float* As = lds[c & 1];
    float* Bs = lds[c & 1] + RM * TLD;
    if constexpr (AG) {
      if (g.act_a > 0) {
#pragma unroll
        for (int s = 0; s < NA; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) ra[p][s][q] = act_grad(ra[p][s][q], ry[p][s][q], g.act_a);
      }
    }
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int f = tid + 256 * s;
      *reinterpret_cast<f32x4*>(As + (f / 16) * TLD + 4 * (f % 16)) = ra[p][s];
    }
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int f = tid + 256 * s;
      // TB: [n][k] rows; !TB: [k][n] rows (the MFMA loop reads the fragment per k there)
      *reinterpret_cast<f32x4*>(Bs + (f / 16) * TLD + 4 * (f % 16)) = rb[p][s];
    }
  };
  f32x4 acc[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int nch = NCH > 0 ? NCH : (K + TK - 1) / TK;
  const int r = lane & 15, kk = lane >> 4;
  auto mma = [&](int c) {
#ifdef MH_TALL_EXP_NOMMA  // cost-attribution experiment only
    if (g.K > 0) return;
#endif
    const float* As = lds[c & 1];
    const float* Bs = lds[c & 1] + RM * TLD;
#pragma unroll
    for (int gq = 0; gq < TK / 16; ++gq) {
      f32x4 bf;
      if (TB) {
        bf = *reinterpret_cast<const f32x4*>(Bs + (wave * 16 + r) * TLD + gq * 16 + 4 * kk);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = Bs[(gq * 16 + 4 * kk + j) * TLD + wave * 16 + r];
      }
      f32x4 af[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i) af[i] = *reinterpret_cast<const f32x4*>(As + (16 * i + r) * TLD + gq * 16 + 4 * kk);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][j], bf[j], acc[i], 0, 0, 0);
    }
  };
  // chunk c: loads of c + 2 issued, MFMAs on LDS buffer c & 1, chunk c + 1 staged into the other
  // buffer (last read in chunk c - 1), one barrier
  auto body = [&](int c, int p) {
    if (c + 2 < nch) load(c + 2, p);
    mma(c);
    if (c + 1 < nch) stage(c + 1, p ^ 1);
    __syncthreads();
  };
  load(0, 0);
  if (nch > 1) load(1, 1);
  stage(0, 0);
  __syncthreads();
  if constexpr (NCH > 0) {
    // K known: straight-line code, so each stage waits only for its own chunk's loads
#pragma unroll
    for (int c = 0; c < NCH; ++c) body(c, c & 1);
  } else {
    for (int c = 0; c < nch; c += 2) {
      body(c, 0);
      if (c + 1 < nch) body(c + 1, 1);
    }
  }
  // C tile through LDS (both buffers are free after the last barrier) so that each quarter-wave
  // stores 256 contiguous bytes of one row instead of 16 scattered columns of four rows
  float* Cs = lds[0];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) Cs[(16 * i + 4 * kk + q) * TLD + wave * 16 + r] = acc[i][q];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < RM * 16 / 256; ++s) {
    const int f = tid + 256 * s, row = m0 + f / 16;
    f32x4 v = *reinterpret_cast<const f32x4*>(Cs + (f / 16) * TLD + 4 * (f % 16));
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = gemm_act(g.bias ? v[q] + bv[q] : v[q], g.act);
#ifdef MH_TALL_EXP_NOSTORE  // cost-attribution experiment only
    if (!(v[0] != v[0])) continue;
#endif
    if (row < M) *reinterpret_cast<f32x4*>(g.C + (int64_t)row * g.ldc + n0 + 4 * (f % 16)) = v;
  }
}

// ------------------------------------------------------------------ deep products
// C[M][N] = A^T B with A [K][M], B [K][N] and K >> M, N: the weight gradients g^T x of the
// update's layers (M = N = 256, K = B x n = 5,120). The BLAS kernel for this shape runs 18.6 us.
// Here the K range splits S ways (S x (M/64)(N/64) ~ deep_target() workgroups: S = 8 at 256 x 256) and
// each workgroup forms a 64 x 64 partial over its K slice:
//   * 64-deep chunks of both operands staged through LDS as [k][64] rows (row-contiguous float4
//     global loads: a quarter-wave reads 256 B of one k row), two chunks ahead in registers;
//   * wave w owns the 32 x 32 quadrant (w & 1, w >> 1): 2 x 2 MFMAs per 4-deep k step, the
//     fragments read from LDS per k row (row stride 80 floats: the four k rows of one read land
//     in distinct banks);
//   * partials go to [S][M][N] and k_gemm_reduce adds them in split order (deterministic).
// M % 64 == 0, N % 64 == 0, 16-B aligned rows, no bias / activation (a weight gradient).
constexpr int DLD = 80;

template <int NCH, bool AG>
__device__ __forceinline__ void gemm_deep_body(const GemmArgs& g, int tiles_m, int bid, float (*lds)[2 * TK * DLD]) {
  constexpr int NF = 64 * TK / 4 / 256;  // float4 loads per operand per thread per chunk (4)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (int)((g.N + 63) / 64);  // column tiles (one, partly used, when N < 64)
  const int tiles = tiles_m * ntn;
  const int tile = bid % tiles, split = bid / tiles;
  const int m0 = (tile % tiles_m) * 64, n0 = (tile / tiles_m) * 64;
  const int K = (int)g.K, lda = (int)g.lda, ldb = (int)g.ldb;
  const int c0 = split * (int)g.kc_per;
  const int nchunks = (K + TK - 1) / TK;
  const int nch = NCH > 0 ? NCH : (c0 + (int)g.kc_per < nchunks ? (int)g.kc_per : nchunks - c0);
  const __amdgpu_buffer_rsrc_t ra_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.A), (short)0, (int)(g.K * g.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.B), (short)0, (int)(g.K * g.ldb * 4), 0x00020000);
  // slot f = tid + 256 s of a chunk -> (k row f / 16, cols 4 (f % 16)..); k rows past K lie
  // beyond the buffers (read 0)
  int aoff[NF], boff[NF];
#pragma unroll
  for (int s = 0; s < NF; ++s) {
    const int f = tid + 256 * s;
    aoff[s] = (f / 16) * lda * 4 + (m0 + 4 * (f % 16)) * 4;
    // columns past N (a narrow layer, N < 64) read from beyond the buffer: zeros
    boff[s] = n0 + 4 * (f % 16) < (int)g.N ? (f / 16) * ldb * 4 + (n0 + 4 * (f % 16)) * 4 : (1 << 30);
  }
  f32x4 ra[2][NF], rb[2][NF];
  f32x4 ry[AG ? 2 : 1][AG ? NF : 1];
  const __amdgpu_buffer_rsrc_t ry_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(AG && g.Y ? g.Y : g.A), (short)0, (int)(g.K * g.lda * 4), 0x00020000);
  auto load = [&](int c, int p) {
    const int kb = (c0 + c) * TK;
#pragma unroll
    for (int s = 0; s < NF; ++s) {
      ra[p][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra_rs, aoff[s] + kb * lda * 4, 0, 0));
      rb[p][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb_rs, boff[s] + kb * ldb * 4, 0, 0));
    }
    if constexpr (AG) {
      if (g.act_a > 0) {
#pragma unroll
        for (int s = 0; s < NF; ++s)
          ry[p][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry_rs, aoff[s] + kb * lda * 4, 0, 0));
      }
    }
  };
  auto stage = [&](int c, int p) {
    float* As = lds[c & 1];
    float* Bs = lds[c & 1] + TK * DLD;
    if constexpr (AG) {
      if (g.act_a > 0) {
#pragma unroll
        for (int s = 0; s < NF; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) ra[p][s][q] = act_grad(ra[p][s][q], ry[p][s][q], g.act_a);
      }
    }
#pragma unroll
    for (int s = 0; s < NF; ++s) {
      const int f = tid + 256 * s;
      *reinterpret_cast<f32x4*>(As + (f / 16) * DLD + 4 * (f % 16)) = ra[p][s];
      *reinterpret_cast<f32x4*>(Bs + (f / 16) * DLD + 4 * (f % 16)) = rb[p][s];
    }
  };
  const int r = lane & 15, kk = lane >> 4, wm = wave & 1, wn = wave >> 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  // bias gradient (AG with db): every workgroup of an (m tile, split) pair holds the same A
  // chunk, so the ntn column tiles share its column sums: tile tn sums the k rows
  // tn, tn + ntn, ... (thread: column tid & 63, every fourth of those rows from tid >> 6), in
  // order, in a register
  const int tn = tile / tiles_m;
  const bool colsum = AG && g.dbp && !g.dbB;
  // dbB: the column sums of B instead, formed by the first row tile of each column tile (the
  // others hold the same B chunk); thread: column tid & 63, every fourth k row from tid >> 6
  const bool colsumB = AG && g.dbp && g.dbB && tile % tiles_m == 0;
  float cs = 0.0f;
  auto mma = [&](int c) {
    const float* As = lds[c & 1];
    const float* Bs = lds[c & 1] + TK * DLD;
    if (colsum) {
      for (int kr = tn + ntn * (tid >> 6); kr < TK; kr += 4 * ntn) cs = cs + As[kr * DLD + (tid & 63)];
    }
    if (colsumB) {
      for (int kr = tid >> 6; kr < TK; kr += 4) cs = cs + Bs[kr * DLD + (tid & 63)];
    }
#pragma unroll
    for (int t = 0; t < TK / 4; ++t) {
      const int kr = (4 * t + kk) * DLD;
      const float a0 = As[kr + 32 * wm + r], a1 = As[kr + 32 * wm + 16 + r];
      const float b0 = Bs[kr + 32 * wn + r], b1 = Bs[kr + 32 * wn + 16 + r];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  };
  auto body = [&](int c, int p) {
    if (c + 2 < nch) load(c + 2, p);
    mma(c);
    if (c + 1 < nch) stage(c + 1, p ^ 1);
    __syncthreads();
  };
  if (nch > 0) {
    load(0, 0);
    if (nch > 1) load(1, 1);
    stage(0, 0);
    __syncthreads();
    if constexpr (NCH > 0) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) body(c, c & 1);
    } else {
      for (int c = 0; c < nch; c += 2) {
        body(c, 0);
        if (c + 1 < nch) body(c + 1, 1);
      }
    }
  }
  // the 64 x 64 result through LDS (free after the last barrier): each quarter-wave then stores
  // 256 contiguous bytes of one row
  float* out = g.S > 1 ? g.partial + (int64_t)split * g.M * g.N : g.C;
  const int64_t ld = g.S > 1 ? g.N : g.ldc;
  float* Cs = lds[0];
  if (nch == 0) __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) Cs[(32 * wm + 16 * i + 4 * kk + q) * DLD + 32 * wn + 16 * j + r] = acc[i][j][q];
  if (colsum || colsumB) lds[1][tid] = cs;
  __syncthreads();
  if ((colsum || colsumB) && tid < 64) {  // the four row groups of this workgroup's share, in order
    const float v = ((lds[1][tid] + lds[1][64 + tid]) + lds[1][128 + tid]) + lds[1][192 + tid];
    if (colsum)
      g.dbp[((int64_t)split * ntn + tn) * g.M + m0 + tid] = v;
    else if (n0 + tid < (int)g.N)
      g.dbp[(int64_t)split * g.N + n0 + tid] = v;
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = tid + 256 * s;
    if (n0 + 4 * (f % 16) < (int)g.N)
      *reinterpret_cast<f32x4*>(out + (int64_t)(m0 + f / 16) * ld + n0 + 4 * (f % 16)) =
          *reinterpret_cast<const f32x4*>(Cs + (f / 16) * DLD + 4 * (f % 16));
  }
}

template <int NCH, bool AG>
__global__ __launch_bounds__(256) void k_gemm_deep(GemmArgs g, int tiles_m) {
  gemm_group(g);
  __shared__ float lds[2][2 * TK * DLD];
  gemm_deep_body<NCH, AG>(g, tiles_m, (int)blockIdx.x, lds);
}

// ------------------------------------------------------------------ several weight gradients at once
// Up to MULTI_MAX deep products (dW = g^T x with the bias gradient) in ONE launch and their split
// reduces in one more: the three layers of an MLP backward (and both twin critics') are independent
// once the input-gradient chain has formed their left operands (mh_mlp3_backward). Product p owns
// workgroups [start[p], start[p + 1]); every product is split over its rows (S >= 2) so its result
// always goes through the reduce, which may write it transposed (dW3 computed as h2^T g3 = dW3^T
// when the layer has fewer than 64 outputs; its bias gradient is then the column sums of the B
// operand g3, formed per split in the deep kernel: GemmArgs::dbB).
constexpr int MULTI_MAX = 6;
struct DeepMulti {
  GemmArgs g[MULTI_MAX];
  int tiles_m[MULTI_MAX];
  int start[MULTI_MAX + 1];
  int rstart[MULTI_MAX + 1];  // reduce blocks
  int trans[MULTI_MAX];
  int n;
};

__global__ __launch_bounds__(256) void k_gemm_deep_multi(DeepMulti d) {
  __shared__ float lds[2][2 * TK * DLD];
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < d.n && b >= d.start[p + 1]) ++p;
  gemm_deep_body<0, true>(d.g[p], d.tiles_m[p], b - d.start[p], lds);
}

__global__ __launch_bounds__(256) void k_gemm_reduce_multi(DeepMulti d) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < d.n && b >= d.rstart[p + 1]) ++p;
  const int rb = b - d.rstart[p], nrb = d.rstart[p + 1] - d.rstart[p];
  gemm_reduce_body(d.g[p], rb, nrb, d.trans[p] != 0);
}

static bool deep_ok(const float* A, const float* B, const float* bias, int64_t M, int64_t N, int64_t K, int64_t lda,
                    int64_t ldb, int ta, int tb, int act) {
#ifdef MH_NO_DEEP_GEMM
  return false;
#endif
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return ta && !tb && !bias && act == 0 && M % 64 == 0 && N % 64 == 0 && K >= 1024 && lda % 4 == 0 &&
         ldb % 4 == 0 && al16(A) && al16(B) && (K + TK) * lda * 4 < ((int64_t)1 << 30) &&
         (K + TK) * ldb * 4 < ((int64_t)1 << 30);
}

// K splits: about 128 workgroups per product, slices of >= 2 chunks. Workgroups a deep product
// aims for (MH_DEEP_WGS overrides for A/B measurements): the weight gradients run beside the other
// update branch's launches, where fewer, longer workgroups (less prologue / partial-tile work per
// CU) win although alone 256 is as fast or faster: bench 1.154-1.161 B env-steps/s at 128 vs
// 1.149-1.151 at 256, 1.139-1.141 at 96, 1.119 at 64; alone, the Lyapunov layers' 52.5 vs 54.7 us
// and the critics' 28.1 vs 25.1 us (tools/r04_deepwgs.sh, r04_deepwgs2.sh)
static int64_t deep_target() {
  static const int64_t t = [] {
    const char* e = getenv("MH_DEEP_WGS");
    const int64_t v = e ? atoll(e) : 0;
    return v > 0 ? v : 128;
  }();
  return t;
}

static int deep_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = (M / 64) * ((N + 63) / 64);
  const int64_t chunks = (K + TK - 1) / TK;
  int64_t S = (deep_target() + tiles - 1) / tiles;
  if (S > chunks / 2) S = chunks / 2;
  if (S < 1) S = 1;
  const int64_t per = (chunks + S - 1) / S;
  return (int)((chunks + per - 1) / per);
}

// row blocks per workgroup for a tall product: fewest (rounds of 256 workgroups) x RB
static int tall_rb(int64_t M, int64_t N) {
#ifdef MH_TALL_RB
  return MH_TALL_RB;
#endif
  const int64_t tn = N / 64;
  int best = 0;
  int64_t best_cost = INT64_MAX;
  for (int rb = 1; rb <= 8; ++rb) {
    const int64_t wgs = ((M + 16 * rb - 1) / (16 * rb)) * tn;
    const int64_t cost = ((wgs + 255) / 256) * (rb + 1);  // + 1: per-workgroup fixed cost
    if (cost < best_cost) {
      best_cost = cost;
      best = rb;
    }
  }
  return best;
}

static bool tall_ok(const float* A, const float* B, const float* bias, const float* C, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int ta) {
#ifdef MH_NO_TALL_GEMM
  return false;
#endif
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return !ta && M >= 2048 && N % 64 == 0 && K % 4 == 0 && K > 0 && lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 &&
         al16(A) && al16(B) && al16(C) && al16(bias) && M * lda * 4 < ((int64_t)1 << 30) &&
         K * 4 < ((int64_t)1 << 28);
}

template <int RB>
static hipError_t launch_tall(const GemmArgs& g, bool tb, hipStream_t st, int groups = 1) {
  const int tiles_n = (int)(g.N / 64);
  const dim3 grid((unsigned)(((g.M + 16 * RB - 1) / (16 * RB)) * tiles_n), (unsigned)groups);
  if (g.act_a >= 0) {  // fused layer backward: dx = (dy * act'(y)) W
    if (tb) return hipErrorInvalidValue;
    if (g.K == 256) k_gemm_tall<RB, false, 4, true><<<grid, 256, 0, st>>>(g, tiles_n);
    else k_gemm_tall<RB, false, 0, true><<<grid, 256, 0, st>>>(g, tiles_n);
  } else if (g.K == 256) {  // the hidden layers of every reference MLP: 4 chunks, unrolled
    if (tb) k_gemm_tall<RB, true, 4, false><<<grid, 256, 0, st>>>(g, tiles_n);
    else k_gemm_tall<RB, false, 4, false><<<grid, 256, 0, st>>>(g, tiles_n);
  } else {
    if (tb) k_gemm_tall<RB, true, 0, false><<<grid, 256, 0, st>>>(g, tiles_n);
    else k_gemm_tall<RB, false, 0, false><<<grid, 256, 0, st>>>(g, tiles_n);
  }
  return hipGetLastError();
}

static hipError_t launch_tall_rb(const GemmArgs& g, bool tb, hipStream_t st, int groups) {
  switch (tall_rb(g.M, g.N)) {
    case 1: return launch_tall<1>(g, tb, st, groups);
    case 2: return launch_tall<2>(g, tb, st, groups);
    case 3: return launch_tall<3>(g, tb, st, groups);
    case 4: return launch_tall<4>(g, tb, st, groups);
    case 5: return launch_tall<5>(g, tb, st, groups);
    case 6: return launch_tall<6>(g, tb, st, groups);
    case 7: return launch_tall<7>(g, tb, st, groups);
    default: return launch_tall<8>(g, tb, st, groups);
  }
}

// ------------------------------------------------------------------ launch plan
struct GemmPlan {
  int wm, wn, S;
  int64_t tiles, kc_per;
};

static GemmPlan gemm_plan(int64_t M, int64_t N, int64_t K) {
  const int64_t chunks = (K + KC - 1) / KC;
  const int cfg[4][2] = {{2, 2}, {2, 1}, {1, 2}, {1, 1}};
  GemmPlan best{1, 1, 1, 0, 0};
  double best_cost = 1e300;
  for (auto& c : cfg) {
    const int TM = 32 * c[0], TN = 32 * c[1], KS = 4 / (c[0] * c[1]);
    const int64_t tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
    int64_t S = 1;
    if (tiles < 192 && chunks >= 4) {  // split only K ranges of >= 2 chunks (128)
      S = (256 + tiles - 1) / tiles;
      if (S > chunks / 2) S = chunks / 2;
      if (S > 32) S = 32;
      if (S < 1) S = 1;
    }
    const int64_t kc_per = (chunks + S - 1) / S;
    S = (chunks + kc_per - 1) / kc_per;
    const int64_t wgs = tiles * S;
    // rounds of resident workgroups x per-wave work (MFMA issue + chunk staging latency)
    const double rounds = (double)((wgs + 1023) / 1024);  // <= 110 VGPRs: 4 workgroups per CU
    const double per_chunk = (KC / 4.0 / KS) * 4.0 * 32.0 + 1500.0;
    const double cost = rounds * (double)kc_per * per_chunk + (S > 1 ? 6000.0 : 0.0) + (KS > 1 ? 300.0 : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = GemmPlan{c[0], c[1], (int)S, tiles, kc_per};
    }
  }
  return best;
}

int64_t gemm_workspace_floats(int64_t M, int64_t N, int64_t K) {
  const GemmPlan p = gemm_plan(M, N, K);
  int64_t S = p.S;
  if (M % 64 == 0 && N % 64 == 0 && K >= 1024) {  // the deep-product path may take this shape
    const int64_t sd = deep_splits(M, N, K);
    S = sd > S ? sd : S;
  }
  return S > 1 ? S * M * N : 0;
}

// One-output products C[M][1] = act(A[M][K] . b + bias) (the critics' / value nets' last layer:
// 5,120 x 256 in the MSACL update): one wave per row, each lane a float4 of every 256-wide K chunk
// in order, the 64 lane sums added by a butterfly; no split-K partials or finishing launch
// (k_gemm + k_gemm_reduce took 9 + 4 us for this shape).
__global__ __launch_bounds__(256) void k_gemv_n1(GemmArgs g, int64_t bstride) {
  gemm_group(g);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= g.M) return;
  const float* a = g.A + row * g.lda;
  float acc = 0.0f;
  for (int64_t k0 = 0; k0 < g.K; k0 += 256) {
    const int64_t k = k0 + 4 * lane;
    if (k + 3 < g.K && bstride == 1) {
      const float4 av = *reinterpret_cast<const float4*>(a + k);
      const float4 bv = *reinterpret_cast<const float4*>(g.B + k);
      acc = acc + av.x * bv.x;
      acc = acc + av.y * bv.y;
      acc = acc + av.z * bv.z;
      acc = acc + av.w * bv.w;
    } else {
      for (int u = 0; u < 4; ++u)
        if (k + u < g.K) acc = acc + a[k + u] * g.B[(k + u) * bstride];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
  if (lane == 0) g.C[row * g.ldc] = gemm_act(g.bias ? acc + g.bias[0] : acc, g.act);
}

// Short-K products C[M][N] = act(A[M][K] B[N][K]^T + bias), K <= 32 (the first layers of the
// update's MLPs: observations / observation + action, K = 12 or 16, into 256 hidden units over
// 5,120-10,240 rows): write-bound, not MFMA-bound. Workgroup = 32 rows x 64 columns with both
// operand tiles in LDS; thread = one column x 8 rows, the K products summed in k order, bias and
// activation applied, 64 consecutive columns per store instruction (k_gemm_tall's 64-deep chunk
// and the library's tile both took 7-14 us for these shapes).
constexpr int SK_MAX = 32;
__global__ __launch_bounds__(256) void k_gemm_shortk(GemmArgs g) {
  __shared__ float As[32][SK_MAX + 1];
  __shared__ float Bs[64][SK_MAX + 1];
  const int tid = threadIdx.x, tx = tid & 63, ty = tid >> 6;
  const int tiles_n = (int)((g.N + 63) / 64);
  const int64_t m0 = (int64_t)(blockIdx.x / tiles_n) * 32;
  const int64_t n0 = (int64_t)(blockIdx.x % tiles_n) * 64;
  const int K = (int)g.K;
  for (int q = tid; q < 32 * K; q += 256) {
    const int r = q / K, k = q - r * K;
    As[r][k] = m0 + r < g.M ? g.A[(m0 + r) * g.lda + k] : 0.0f;
  }
  for (int q = tid; q < 64 * K; q += 256) {
    const int c = q / K, k = q - c * K;
    Bs[c][k] = n0 + c < g.N ? g.B[(n0 + c) * g.ldb + k] : 0.0f;
  }
  __syncthreads();
  const int64_t col = n0 + tx;
  if (col >= g.N) return;
  const float bv = g.bias ? g.bias[col] : 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = ty + 4 * i;
    if (m0 + r >= g.M) break;
    float acc = As[r][0] * Bs[tx][0];
    for (int k = 1; k < K; ++k) acc = acc + As[r][k] * Bs[tx][k];
    g.C[(m0 + r) * g.ldc + col] = gemm_act(g.bias ? acc + bv : acc, g.act);
  }
}

template <int WM, int WN>
static hipError_t launch_gemm_cfg(const GemmArgs& g, int64_t grid, bool ta, bool tb, hipStream_t st) {
  if (!ta && !tb) k_gemm<WM, WN, false, false><<<(unsigned)grid, 256, 0, st>>>(g);
  else if (!ta && tb) k_gemm<WM, WN, false, true><<<(unsigned)grid, 256, 0, st>>>(g);
  else if (ta && !tb) k_gemm<WM, WN, true, false><<<(unsigned)grid, 256, 0, st>>>(g);
  else k_gemm<WM, WN, true, true><<<(unsigned)grid, 256, 0, st>>>(g);
  return hipGetLastError();
}

hipError_t launch_gemm(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                       int64_t lda, int64_t ldb, int64_t ldc, int ta, int tb, int act, float* workspace,
                       hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  // 32-bit buffer offsets (load_chunk): both operands below 2 GiB
  if ((ta ? K : M) * lda * 4 >= ((int64_t)1 << 31) - 64 || (tb ? N : K) * ldb * 4 >= ((int64_t)1 << 31) - 64)
    return hipErrorInvalidValue;
  if (deep_ok(A, B, bias, M, N, K, lda, ldb, ta, tb, act) && ((uintptr_t)C & 15) == 0 && ldc % 4 == 0 &&
      (deep_splits(M, N, K) == 1 || (workspace && ((uintptr_t)workspace & 15) == 0))) {
    const int S = deep_splits(M, N, K);
    const int64_t chunks = (K + TK - 1) / TK;
    const int64_t per = (chunks + S - 1) / S;
    GemmArgs g{A, B, nullptr, C, M, N, K, lda, ldb, ldc, 0, S, per, workspace, nullptr, -1, nullptr, nullptr};
    const int tiles_m = (int)(M / 64);
    const unsigned grid = (unsigned)(tiles_m * (N / 64) * S);
    // every split full (the common case: 5,120 = 16 x 5 chunks) -> unrolled 5-chunk body
    if (per == 5 && chunks == per * S) k_gemm_deep<5, false><<<grid, 256, 0, st>>>(g, tiles_m);
    else k_gemm_deep<0, false><<<grid, 256, 0, st>>>(g, tiles_m);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || S == 1) return e;
    const int64_t want = (M * N + 255) / 256;
    k_gemm_reduce<<<(unsigned)(want < 2048 ? want : 2048), 256, 0, st>>>(g);
    return hipGetLastError();
  }
  if (!ta && tb && K >= 1 && K <= SK_MAX && M >= 256 && N >= 64) {
    GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, 1, 0, nullptr, nullptr, -1, nullptr, nullptr};
    const int64_t grid = ((M + 31) / 32) * ((N + 63) / 64);
    k_gemm_shortk<<<(unsigned)grid, 256, 0, st>>>(g);
    return hipGetLastError();
  }
  if (tall_ok(A, B, bias, C, M, N, K, lda, ldb, ldc, ta) && (tb ? N : K) * ldb * 4 < ((int64_t)1 << 30)) {
    GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, 1, 0, nullptr, nullptr, -1, nullptr, nullptr};
    switch (tall_rb(M, N)) {
      case 1: return launch_tall<1>(g, tb, st);
      case 2: return launch_tall<2>(g, tb, st);
      case 3: return launch_tall<3>(g, tb, st);
      case 4: return launch_tall<4>(g, tb, st);
      case 5: return launch_tall<5>(g, tb, st);
      case 6: return launch_tall<6>(g, tb, st);
      case 7: return launch_tall<7>(g, tb, st);
      default: return launch_tall<8>(g, tb, st);
    }
  }
  if (N == 1 && !ta && M >= 256 && K > 0 && lda % 4 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0) {
    GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, 1, 0, nullptr, nullptr, -1, nullptr, nullptr};
    k_gemv_n1<<<(unsigned)((M + 3) / 4), 256, 0, st>>>(g, tb ? 1 : ldb);
    return hipGetLastError();
  }
  const GemmPlan p = gemm_plan(M, N, K > 0 ? K : 1);
  GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, p.S, p.kc_per, workspace, nullptr, -1, nullptr, nullptr};
  const int64_t grid = p.tiles * p.S;
  hipError_t e;
  if (p.wm == 2 && p.wn == 2) e = launch_gemm_cfg<2, 2>(g, grid, ta, tb, st);
  else if (p.wm == 2 && p.wn == 1) e = launch_gemm_cfg<2, 1>(g, grid, ta, tb, st);
  else if (p.wm == 1 && p.wn == 2) e = launch_gemm_cfg<1, 2>(g, grid, ta, tb, st);
  else e = launch_gemm_cfg<1, 1>(g, grid, ta, tb, st);
  if (e != hipSuccess || p.S == 1) return e;
  const int64_t want = (M * N + 255) / 256;
  k_gemm_reduce<<<(unsigned)(want < 2048 ? want : 2048), 256, 0, st>>>(g);
  return hipGetLastError();
}

// ------------------------------------------------------------------ fused layer backward
// For y = act(x W^T + b) over `rows` rows (W [n_out][n_in]): dx = g W, dW = g^T x, db = sum_rows g
// with g = dy * act'(y) formed on the fly inside the two GEMMs' A-operand staging (the tall
// kernel for dx, the deep kernel for dW and db), instead of k_act_grad_colsum writing g and the
// bias gradient first: one launch fewer and g never written to or re-read from HBM.
static bool lb_dx_ok(int64_t rows, int64_t n_out, int64_t n_in) {
  return rows >= 2048 && n_in % 64 == 0 && n_out % 4 == 0 && n_out >= 64 && rows * n_out * 4 < ((int64_t)1 << 30) &&
         n_out * n_in * 4 < ((int64_t)1 << 30) && n_out * 4 < ((int64_t)1 << 28);
}
// n_in below 64 (the first layer's observation / observation+action inputs): one column tile,
// its columns past n_in read as zeros and not stored (dW and db only: the tall dx kernel needs
// n_in % 64 == 0)
static bool lb_dw_ok(int64_t rows, int64_t n_out, int64_t n_in) {
  return n_out % 64 == 0 && (n_in % 64 == 0 || (n_in < 64 && n_in % 4 == 0)) && rows >= 1024 &&
         (rows + TK) * n_out * 4 < ((int64_t)1 << 30) &&
         (rows + TK) * n_in * 4 < ((int64_t)1 << 30);
}

bool linear_backward_plan(int64_t rows, int64_t n_out, int64_t n_in, bool dx, bool dw, bool db, int64_t* ws) {
  *ws = 0;
  if ((!dx && !dw) || (db && !dw)) return false;
  if (dx && !lb_dx_ok(rows, n_out, n_in)) return false;
  if (dw && !lb_dw_ok(rows, n_out, n_in)) return false;
  if (dw) {
    const int S = deep_splits(n_out, n_in, rows);
    *ws = (S > 1 ? (int64_t)S * n_out * n_in : 0) + (db ? (int64_t)S * ((n_in + 63) / 64) * n_out : 0);
  }
  return true;
}

hipError_t launch_linear_backward(const float* dy, const float* y, int act, const float* x, const float* W,
                                  int64_t rows, int64_t n_out, int64_t n_in, float* dx, float* dw, float* db,
                                  float* workspace, hipStream_t st) {
  if (dx) {  // dx[rows][n_in] = g[rows][n_out] . W[n_out][n_in]
    GemmArgs g{dy, W, nullptr, dx, rows, n_in, n_out, n_out, n_in, n_in, 0, 1, 0, nullptr, y, act, nullptr, nullptr};
    hipError_t e;
    switch (tall_rb(rows, n_in)) {
      case 1: e = launch_tall<1>(g, false, st); break;
      case 2: e = launch_tall<2>(g, false, st); break;
      case 3: e = launch_tall<3>(g, false, st); break;
      case 4: e = launch_tall<4>(g, false, st); break;
      case 5: e = launch_tall<5>(g, false, st); break;
      case 6: e = launch_tall<6>(g, false, st); break;
      case 7: e = launch_tall<7>(g, false, st); break;
      default: e = launch_tall<8>(g, false, st); break;
    }
    if (e != hipSuccess) return e;
  }
  if (dw) {  // dW[n_out][n_in] = g^T x over the rows; db[n_out] = column sums of g
    const int S = deep_splits(n_out, n_in, rows);
    const int64_t chunks = (rows + TK - 1) / TK;
    const int64_t per = (chunks + S - 1) / S;
    float* dbp = db ? workspace + (S > 1 ? (int64_t)S * n_out * n_in : 0) : nullptr;
    const int ntn = (int)((n_in + 63) / 64);
    GemmArgs g{dy, x, nullptr, dw, n_out, n_in, rows, n_out, n_in, n_in, 0, S, per, workspace, y, act, db, dbp,
               S * ntn};
    const int tiles_m = (int)(n_out / 64);
    const unsigned grid = (unsigned)(tiles_m * ntn * S);
    if (per == 5 && chunks == per * S) k_gemm_deep<5, true><<<grid, 256, 0, st>>>(g, tiles_m);
    else k_gemm_deep<0, true><<<grid, 256, 0, st>>>(g, tiles_m);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || (S == 1 && !db)) return e;
    const int64_t want = (n_out * n_in + 255) / 256;
    k_gemm_reduce<<<(unsigned)(want < 2048 ? want : 2048), 256, 0, st>>>(g);
    return hipGetLastError();
  }
  return hipSuccess;
}

// ------------------------------------------------------------------ several weight gradients
// product p: dw[n_out][n_in] = g^T x over `rows`, db = column sums of g. Returns false when a
// product does not fit (the caller takes the per-layer path); ws_floats: workspace needed.
static bool wgrad_plan(const WgradSpec* ps, int n, int64_t rows, DeepMulti* d, int64_t* ws_floats, float* ws) {
  if (n < 1 || n > MULTI_MAX || rows < 1024) return false;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  int64_t off = 0;
  int start = 0, rstart = 0;
  if (d) std::memset(d, 0, sizeof(*d));
  for (int i = 0; i < n; ++i) {
    const WgradSpec& q = ps[i];
    if (q.ld_g % 4 || q.ld_x % 4 || !al16(q.g) || !al16(q.x) || !q.dw) return false;
    const bool normal = q.n_out % 64 == 0 && q.n_in % 4 == 0;
    const bool swapped = !normal && q.n_out < 64 && q.n_out % 4 == 0 && q.n_in % 64 == 0;
    if (!normal && !swapped) return false;
    const int64_t M = swapped ? q.n_in : q.n_out, N = swapped ? q.n_out : q.n_in;
    if ((rows + TK) * (swapped ? q.ld_x : q.ld_g) * 4 >= ((int64_t)1 << 30) ||
        (rows + TK) * (swapped ? q.ld_g : q.ld_x) * 4 >= ((int64_t)1 << 30))
      return false;
    int S = deep_splits(M, N, rows);
    const int64_t chunks = (rows + TK - 1) / TK;
    if (S < 2) S = chunks >= 2 ? 2 : 1;
    if (S < 2) return false;
    const int64_t per = (chunks + S - 1) / S;
    S = (int)((chunks + per - 1) / per);
    if (S < 2) return false;
    const int ntn = (int)((N + 63) / 64), tiles_m = (int)(M / 64);
    const bool dbp = q.db != nullptr;  // normal: column sums of A = g; swapped: of B = g
    const int64_t need = (int64_t)S * M * N + (dbp ? (normal ? (int64_t)S * ntn * M : (int64_t)S * N) : 0);
    if (d) {
      GemmArgs g{};
      g.A = swapped ? q.x : q.g;
      g.B = swapped ? q.g : q.x;
      g.C = q.dw;
      g.M = M; g.N = N; g.K = rows;
      g.lda = swapped ? q.ld_x : q.ld_g;
      g.ldb = swapped ? q.ld_g : q.ld_x;
      g.ldc = swapped ? M : N;  // transposed write: dw[n_out][n_in] = C^T, row length n_in = M
      g.act = 0; g.S = S; g.kc_per = per; g.partial = ws + off;
      g.act_a = 0;
      g.db = dbp ? q.db : nullptr;
      g.dbp = dbp ? ws + off + (int64_t)S * M * N : nullptr;
      g.dbn = normal ? S * ntn : S;
      g.dbB = swapped ? 1 : 0;
      d->g[i] = g;
      d->tiles_m[i] = tiles_m;
      d->start[i] = start;
      d->rstart[i] = rstart;
      d->trans[i] = swapped ? 1 : 0;
    }
    off += need;
    start += tiles_m * ntn * S;
    const int64_t rb = (M * N + 255) / 256;
    rstart += (int)(rb < 512 ? rb : 512);
  }
  if (d) {
    d->start[n] = start;
    d->rstart[n] = rstart;
    d->n = n;
  }
  *ws_floats = off;
  return true;
}

bool weight_grads_plan(const WgradSpec* ps, int n, int64_t rows, int64_t* ws_floats) {
  return wgrad_plan(ps, n, rows, nullptr, ws_floats, nullptr);
}

hipError_t launch_weight_grads(const WgradSpec* ps, int n, int64_t rows, float* ws, hipStream_t st) {
  DeepMulti d;
  int64_t need = 0;
  if (!wgrad_plan(ps, n, rows, &d, &need, ws)) return hipErrorInvalidValue;
  k_gemm_deep_multi<<<(unsigned)d.start[n], 256, 0, st>>>(d);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  k_gemm_reduce_multi<<<(unsigned)d.rstart[n], 256, 0, st>>>(d);
  return hipGetLastError();
}

// ------------------------------------------------------------------ grouped launches
// `groups` independent products of one shape in ONE launch (blockIdx.y = group), group q's
// operands at the group-0 pointers + q x the strides (floats): the twin critics' hidden and
// output layers, whose two networks read the two halves of one [rows][2H] activation buffer.
// Routes: the tall kernel (forward x W^T / g W on >= 2,048 rows) and the one-output GEMV;
// hipErrorInvalidValue for any other shape (the caller runs the groups one by one).
hipError_t launch_gemm_grouped(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N,
                               int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int ta, int tb, int act, int groups,
                               int64_t sA, int64_t sB, int64_t sBias, int64_t sC, hipStream_t st) {
  if (M <= 0 || N <= 0 || groups <= 0) return hipSuccess;
  if (groups > 65535) return hipErrorInvalidValue;
  auto al16 = [](int64_t x) { return (x & 3) == 0; };  // a float stride that keeps 16-byte alignment
  if (tall_ok(A, B, bias, C, M, N, K, lda, ldb, ldc, ta) && (tb ? N : K) * ldb * 4 < ((int64_t)1 << 30) &&
      al16(sA) && al16(sB) && al16(sC) && (!bias || al16(sBias))) {
    GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, 1, 0, nullptr, nullptr, -1, nullptr, nullptr, 0,
               sA, sB, sC, sBias, 0, 0, 0, 0};
    return launch_tall_rb(g, tb, st, groups);
  }
  if (N == 1 && !ta && M >= 256 && K > 0 && lda % 4 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
      al16(sA) && (tb ? al16(sB) : true)) {
    GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, 1, 0, nullptr, nullptr, -1, nullptr, nullptr, 0,
               sA, sB, sC, sBias, 0, 0, 0, 0};
    k_gemv_n1<<<dim3((unsigned)((M + 3) / 4), (unsigned)groups), 256, 0, st>>>(g, tb ? 1 : ldb);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

// The fused layer backward (launch_linear_backward) of `groups` layers of one shape in one launch
// per GEMM: dy / y rows of leading dimension ld_dy, x of ld_x, dx of ld_dx; group q's operands at
// q x the strides. Workspace: groups x linear_backward_plan's per-group floats.
hipError_t launch_linear_backward_grouped(const float* dy, const float* y, int act, const float* x, const float* W,
                                          int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x,
                                          int64_t ld_dx, int groups, int64_t s_dy, int64_t s_x, int64_t s_W,
                                          int64_t s_dx, int64_t s_dw, int64_t s_db, float* dx, float* dw, float* db,
                                          float* workspace, hipStream_t st) {
  if (groups <= 0) return hipSuccess;
  if (groups > 65535 || ld_dy % 4 || ld_x % 4 || ld_dx % 4 || s_dy % 4 || s_x % 4 || s_dx % 4 || s_W % 4 ||
      s_dw % 4)
    return hipErrorInvalidValue;
  if (dx) {  // dx[rows][n_in] = g[rows][n_out] . W[n_out][n_in], per group
    if (!lb_dx_ok(rows, n_out, n_in) || rows * ld_dy * 4 >= ((int64_t)1 << 30)) return hipErrorInvalidValue;
    GemmArgs g{dy, W, nullptr, dx, rows, n_in, n_out, ld_dy, n_in, ld_dx, 0, 1, 0, nullptr, y, act, nullptr, nullptr, 0,
               s_dy, s_W, s_dx, 0, s_dy, 0, 0, 0};
    const hipError_t e = launch_tall_rb(g, false, st, groups);
    if (e != hipSuccess) return e;
  }
  if (dw) {  // dW[n_out][n_in] = g^T x over the rows; db[n_out] = column sums of g, per group
    if (!lb_dw_ok(rows, n_out, n_in) || (rows + TK) * ld_dy * 4 >= ((int64_t)1 << 30) ||
        (rows + TK) * ld_x * 4 >= ((int64_t)1 << 30))
      return hipErrorInvalidValue;
    const int S = deep_splits(n_out, n_in, rows);
    const int64_t chunks = (rows + TK - 1) / TK;
    const int64_t per = (chunks + S - 1) / S;
    const int ntn = (int)((n_in + 63) / 64);
    const int64_t part = S > 1 ? (int64_t)S * n_out * n_in : 0;
    const int64_t wsg = part + (db ? (int64_t)S * ntn * n_out : 0);  // per group
    float* dbp = db ? workspace + part : nullptr;
    GemmArgs g{dy, x, nullptr, dw, n_out, n_in, rows, ld_dy, ld_x, n_in, 0, S, per, workspace, y, act, db, dbp,
               S * ntn, s_dy, s_x, s_dw, 0, s_dy, wsg, s_db, wsg};
    const int tiles_m = (int)(n_out / 64);
    const dim3 grid((unsigned)(tiles_m * ntn * S), (unsigned)groups);
    if (per == 5 && chunks == per * S) k_gemm_deep<5, true><<<grid, 256, 0, st>>>(g, tiles_m);
    else k_gemm_deep<0, true><<<grid, 256, 0, st>>>(g, tiles_m);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || (S == 1 && !db)) return e;
    const int64_t want = (n_out * n_in + 255) / 256;
    k_gemm_reduce<<<dim3((unsigned)(want < 2048 ? want : 2048), (unsigned)groups), 256, 0, st>>>(g);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace mh
