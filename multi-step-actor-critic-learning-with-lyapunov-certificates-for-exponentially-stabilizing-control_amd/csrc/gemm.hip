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
};

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

// C = act(sum_s partial[s] + bias), splits added in order
__global__ __launch_bounds__(256) void k_gemm_reduce(GemmArgs g) {
  const int64_t MN = g.M * g.N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < MN; i += (int64_t)gridDim.x * 256) {
    float v = g.partial[i];
    for (int sp = 1; sp < g.S; ++sp) v += g.partial[(int64_t)sp * MN + i];
    const int64_t row = i / g.N, col = i - row * g.N;
    g.C[row * g.ldc + col] = gemm_act(g.bias ? v + g.bias[col] : v, g.act);
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
  return p.S > 1 ? (int64_t)p.S * M * N : 0;
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
  const GemmPlan p = gemm_plan(M, N, K > 0 ? K : 1);
  GemmArgs g{A, B, bias, C, M, N, K, lda, ldb, ldc, act, p.S, p.kc_per, workspace};
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

}  // namespace mh
