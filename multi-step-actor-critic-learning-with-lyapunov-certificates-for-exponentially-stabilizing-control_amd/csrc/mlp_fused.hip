// mlp_fused.hip — the update's 3-layer MLPs (RL/apprfunc/mlp.py:18-30: Linear -> act -> Linear ->
// act -> Linear -> act) forward in ONE launch (gfx950, f32-input MFMA).
//
//   h1 = act1(x W1^T + b1)   [M][H]      x [M][K1], K1 <= 32
//   h2 = act2(h1 W2^T + b2)  [M][H]      H = 256
//   y  = act3(h2 W3^T + b3)  [M][N3]     N3 <= 16, or N3 a multiple of 64 (<= 256)
//
// The per-layer path is three launches (the BLAS short-K GEMM, the tall kernel, a GEMV / narrow
// GEMM: 30-35 us at 5,120 rows, most of it per-launch ramp and drain), and it writes h1 to HBM and
// reads it back. Here a workgroup owns TM = 16 rows through all three layers:
//   * 4 waves; in each hidden layer wave w computes output columns [64 w, 64 w + 64) as four
//     16 x 16 accumulators (v_mfma_f32_16x16x4_f32);
//   * the layer's input rows sit in LDS; every 16-deep K group is one ds_read_b128 per lane (the
//     A operand of four MFMAs) and four global float4 loads of weight rows (the B operands), the
//     loads issued three groups ahead. The K order inside a group is permuted consistently on
//     both operands: in MFMA t of group u, lane group g = lane >> 4 contracts k = 16 u + 4 g + t,
//     so one 16-byte load per lane and operand feeds four MFMAs;
//   * the epilogue (bias, activation) writes the layer's output tile to LDS for the next layer,
//     and (when the caller keeps them for the backward) as row-contiguous float4 stores to h1 / h2;
//   * narrow output layers (N3 <= 16: the policy head, the critics' single output) split K over
//     the four waves and add the four partial tiles in wave order through LDS.
// Numerics: f32 MFMA products (exact) accumulated in f32 in k order within each 4-deep step; the
// same f32 results as the per-layer kernels up to summation order.
// Grouped launches (the twin critics, apprfunc/_twin.py): blockIdx.y = group q; every pointer is
// advanced by q x its group stride (floats; 0 = shared).
#include <cstring>

#include "policy_x3.h"
#include "rollout.h"

namespace mh {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// a + b element by element as four scalar adds: a vector `+` on f32x4 is selected as two packed
// v_pk_add_f32, which no kernel of the library carries (tests/test_build_isa.py; csrc/Makefile)
__device__ __forceinline__ f32x4 add4_scalar(f32x4 a, f32x4 b) {
  float r0 = a[0] + b[0], r1 = a[1] + b[1], r2 = a[2] + b[2], r3 = a[3] + b[3];
  asm volatile("" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));  // keep them scalar (no v2f32 re-pairing)
  return f32x4{r0, r1, r2, r3};
}
__device__ __forceinline__ f32x4 mul4_scalar(f32x4 a, float k) {
  float r0 = a[0] * k, r1 = a[1] * k, r2 = a[2] * k, r3 = a[3] * k;
  asm volatile("" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
  return f32x4{r0, r1, r2, r3};
}

constexpr int TM = 16;        // rows per workgroup
constexpr int HID = 256;      // hidden width
constexpr int SH = HID + 4;   // LDS row stride of a hidden tile (floats): rows 16 B apart in the banks
constexpr int K1P = 32;       // first-layer K padded
constexpr int SX = K1P + 4;
#ifndef MH_MLP_PF
#define MH_MLP_PF 2
#endif
#ifndef MH_MLP_PFT
#define MH_MLP_PFT 3
#endif
// weight groups in the load ring: PF - 1 in flight behind the MFMAs. One group ahead (PF = 2) is
// the fastest at the update's shapes (round 5, tools/r05_pf_probe.sh, r05_pf_bench.sh): a group's
// MFMAs (32 at two row tiles, ~1 k cycles) cover its loads' L2 latency, and every deeper ring was
// slower (PF = 4 / 5 / 6 / 8: +3 / +5 / +7 / +15 % on the 10,240-row forward): each load touches
// 16 half-used 128-byte lines whose other halves the NEXT group reads, and with more groups in
// flight those lines are evicted from the vector L1 before that read
constexpr int PF = MH_MLP_PF;

// The load ring is enforced with scheduling barriers: left to itself the scheduler regroups the
// fully unrolled loop and waits on each group's loads right after issuing them (one L2 latency per
// 16-deep group — the r04 first cut measured 41 us at 5,120 rows, latency-bound).
#define MH_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

template <int ACT>
__device__ __forceinline__ float act_t(float v) {
  if constexpr (ACT == 1) return v < 0.0f ? 0.0f : v;  // as torch.relu / gemm_act (NaN passes through)
  if constexpr (ACT == 2) return tanhf(v);
  return v;
}

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == 1) return act_t<1>(v);
  if (act == 2) return act_t<2>(v);
  return v;
}

// One hidden-width layer for this wave's 64 output columns: out[16][64] += in[16][K] W[n][K]^T,
// K = 16 G. `in` is the LDS tile (row stride SIN floats), W rows [n0, n0 + 64) of a row-major [N][K]
// matrix behind a buffer resource (rows past N read 0). Group u's four weight float4s are issued
// PF - 1 groups before its MFMAs; its A operand (one ds_read_b128) one group before.
// layer_cols_pre issues the ring's first PF - 1 groups (the caller may do so long before the layer:
// the forward issues layer 2's at kernel start, beside layer 1's weights), layer_cols_run the rest.
template <int G>
__device__ __forceinline__ void wring_load(__amdgpu_buffer_rsrc_t wr, int n0, int lane, int u, f32x4 (&dst)[4]) {
  constexpr int K = 16 * G;
  const int r = lane & 15, g = lane >> 4;
  const int voff = ((n0 + r) * K + 4 * g) * 4;
#ifdef MH_MLP_EXP_PACKED  // cost-attribution experiment only: fragment-ordered addresses (wrong results)
  for (int j = 0; j < 4; ++j)
    dst[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           wr, (((n0 / 16 + j) * G + u) * 64 + lane) * 16, 0, 0));
  return;
#endif
#ifdef MH_MLP_EXP_NOLOAD  // cost-attribution experiment only: no weight loads (wrong results)
  for (int j = 0; j < 4; ++j) dst[j] = f32x4{(float)voff, 0.f, 1.f, (float)u};
  return;
#endif
#pragma unroll
  for (int j = 0; j < 4; ++j)
    dst[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, voff + (16 * j * K + 16 * u) * 4, 0, 0));
}

template <int G>
__device__ __forceinline__ void layer_cols_pre(__amdgpu_buffer_rsrc_t wr, int n0, int lane, f32x4 (&wb)[PF][4]) {
#pragma unroll
  for (int p = 0; p < PF - 1; ++p)
    if (p < G) wring_load<G>(wr, n0, lane, p, wb[p]);
}

// RT row tiles of 16 (the workgroup's TM = 16 RT rows): each weight fragment feeds RT MFMAs, so a
// workgroup streams the layer's weights once per 16 RT rows.
template <int SIN, int G, int RT = 1>
__device__ __forceinline__ void layer_cols_run(const float* in, __amdgpu_buffer_rsrc_t wr, int n0, int lane,
                                               f32x4 (&acc)[RT][4], f32x4 (&wb)[PF][4]) {
  const int r = lane & 15, g = lane >> 4;
  const float* arow = in + r * SIN + 4 * g;
  f32x4 a_cur[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) a_cur[rt] = *reinterpret_cast<const f32x4*>(arow + 16 * rt * SIN);
#pragma unroll
  for (int u = 0; u < G; ++u) {
    if (u + PF - 1 < G) wring_load<G>(wr, n0, lane, u + PF - 1, wb[(u + PF - 1) % PF]);
    f32x4 a_nxt[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      a_nxt[rt] = u + 1 < G ? *reinterpret_cast<const f32x4*>(arow + 16 * rt * SIN + 16 * (u + 1)) : a_cur[rt];
    MH_SCHED_FENCE();
#ifdef MH_MLP_EXP_NOMFMA  // cost-attribution experiment only: operands consumed, no MFMA (wrong results)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[rt][j] += a_cur[rt] * wb[u % PF][j];
#else
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[rt][t], wb[u % PF][j][t], acc[rt][j], 0, 0, 0);
#endif
    MH_SCHED_FENCE();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a_cur[rt] = a_nxt[rt];
  }
}

template <int SIN, int G, int RT = 1>
__device__ __forceinline__ void layer_cols(const float* in, __amdgpu_buffer_rsrc_t wr, int n0, int lane,
                                           f32x4 (&acc)[RT][4]) {
  f32x4 wb[PF][4];
  layer_cols_pre<G>(wr, n0, lane, wb);
  layer_cols_run<SIN, G, RT>(in, wr, n0, lane, acc, wb);
}

// ---- the split-f16 form of a hidden-width layer (round 6): out[16 RT][64] += in[.][K] W[n][K]^T with
// v_mfma_f32_16x16x32_f16 on two-way f16 splits, three products per f32 product (lo.hi, hi.lo,
// hi.hi: policy_x3.h's scheme), i.e. 16-cycle 16x16x32 MFMAs, three per 32-deep K-step, instead of
// eight 32-cycle 16x16x4 f32 MFMAs: the f32 layer kept a wave's SIMD 16 k cycles in MFMA issue at
// two row tiles. Operands, per lane l (16x16x32: A[row l & 15][k = 8 (l >> 4) + j], B[k][col l & 15]):
//   A: eight consecutive floats of its row from the LDS tile, times the row tile's power of two
//      2^e (from the tile's max |value|: every scaled value <= 2^14), then split;
//   B: eight consecutive floats of weight row n (W [N][K] row-major: two global float4 loads per
//      16-column block and 32-deep K-step), times the fixed WX = 2^10, then split: the f16 lo of a
//      weight in [2^-13, 64) is a normal number, so hi + lo keeps 22 bits of it; a weight of 64 or
//      more overflows its f16 hi, the tile's accumulators come out non-finite, and that row tile
//      is recomputed by the f32 layer (x3_redo_nonfinite: cold, the bits of the f32 path);
// the accumulators carry 2^e WX, undone exactly (powers of two) before the bias and activation.
// A value is split in one rounding each way: hi = f16(v k), lo = f16(v k - hi) (v_fma_mix, the
// product and difference exact inside the fused multiply-add).
// The K-step's weights are loaded PF - 1 steps ahead (as layer_cols's ring), its A operand one ahead.
constexpr int KS32 = HID / 32;  // 32-deep K-steps of a hidden-width layer
constexpr float WX = 1024.0f, IWX = 1.0f / 1024.0f;
typedef _Float16 f16x8m __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split2h_pair_k(float a, float b, float k, uint32_t& hi, uint32_t& lo) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(a), "v"(b), "v"(k));
}

// eight floats -> (hi, lo) f16x8 of the values times k
__device__ __forceinline__ void split8(const f32x4& p, const f32x4& q, float k, f16x8m& hi, f16x8m& lo) {
  uint32_t h[4], l[4];
  split2h_pair_k(p[0], p[1], k, h[0], l[0]);
  split2h_pair_k(p[2], p[3], k, h[1], l[1]);
  split2h_pair_k(q[0], q[1], k, h[2], l[2]);
  split2h_pair_k(q[2], q[3], k, h[3], l[3]);
  hi = __builtin_bit_cast(f16x8m, uint4{h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(f16x8m, uint4{l[0], l[1], l[2], l[3]});
}

template <int PFX>
__device__ __forceinline__ void wring_load_x3(__amdgpu_buffer_rsrc_t wr, int n0, int lane, int ks, f32x4 (&dst)[4][2]) {
  const int r = lane & 15, g = lane >> 4;
  const int voff = ((n0 + r) * HID + 32 * ks + 8 * g) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      dst[j][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, voff + (16 * j * HID + 4 * h) * 4, 0, 0));
}

template <int RT>
__device__ __forceinline__ void layer_cols_pre_x3(__amdgpu_buffer_rsrc_t wr, int n0, int lane, f32x4 (&wb)[PF][4][2]) {
#pragma unroll
  for (int p = 0; p < PF - 1; ++p) wring_load_x3<PF>(wr, n0, lane, p, wb[p]);
}

template <int SIN, int RT>
__device__ __forceinline__ void layer_cols_run_x3(const float* in, const float (&sc)[RT], __amdgpu_buffer_rsrc_t wr,
                                                  int n0, int lane, f32x4 (&acc)[RT][4], f32x4 (&wb)[PF][4][2]) {
  const int r = lane & 15, g = lane >> 4;
  const float wx = WX;
  const float* arow = in + r * SIN + 8 * g;
  f32x4 a_cur[RT][2];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int h = 0; h < 2; ++h) a_cur[rt][h] = *reinterpret_cast<const f32x4*>(arow + 16 * rt * SIN + 4 * h);
#pragma unroll
  for (int ks = 0; ks < KS32; ++ks) {
    if (ks + PF - 1 < KS32) wring_load_x3<PF>(wr, n0, lane, ks + PF - 1, wb[(ks + PF - 1) % PF]);
    f32x4 a_nxt[RT][2];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        a_nxt[rt][h] = ks + 1 < KS32 ? *reinterpret_cast<const f32x4*>(arow + 16 * rt * SIN + 32 * (ks + 1) + 4 * h)
                                     : a_cur[rt][h];
    MH_SCHED_FENCE();
    f16x8m ah[RT], al[RT], wh[4], wl[4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) split8(a_cur[rt][0], a_cur[rt][1], sc[rt], ah[rt], al[rt]);
#pragma unroll
    for (int j = 0; j < 4; ++j) split8(wb[ks % PF][j][0], wb[ks % PF][j][1], wx, wh[j], wl[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[rt], wh[j], acc[rt][j], 0, 0, 0);
        acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], wl[j], acc[rt][j], 0, 0, 0);
        acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt], wh[j], acc[rt][j], 0, 0, 0);
      }
    MH_SCHED_FENCE();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int h = 0; h < 2; ++h) a_cur[rt][h] = a_nxt[rt][h];
  }
}

// the largest |value| of each row tile of an epilogue's output, over the workgroup (LDS atomic max
// on the bits: non-negative floats order as their bit patterns; NaN stays the max)
template <int RT>
__device__ __forceinline__ void tile_max_publish(const float (&m)[RT], uint32_t* smax) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float v = m[rt];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(smax + rt, __float_as_uint(v));
  }
}
// the A scale of each row tile (a power of two, every scaled value <= 2^14) and the accumulators'
// unscale (2^-e / WX)
template <int RT>
__device__ __forceinline__ void tile_scales(const uint32_t* smax, float (&sc)[RT], float (&isc)[RT]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const float m = __uint_as_float(smax[rt]);
    const int e = pm_scale_exp(m);  // 0 for 0 / NaN
    sc[rt] = pm_pow2(e);
    isc[rt] = pm_pow2(-e) * IWX;  // exact: 2^-(e + 10) >= 2^-50
  }
}

// The row tiles whose split-f16 accumulators came out non-finite (a weight of 64 or more, or a
// non-finite input, which the f32 layer turns into the same non-finite values) are recomputed by
// the f32 layer, 2^e WX-scaled so the epilogue's unscale applies unchanged. Wave-uniform and cold.
struct Acc4 {
  f32x4 v[4];
};
template <int SIN>
__device__ __noinline__ Acc4 x3_redo_tile(const float* in, __amdgpu_buffer_rsrc_t wr, int n0, int lane, float s) {
  f32x4 a1[1][4] = {};
  layer_cols<SIN, HID / 16, 1>(in, wr, n0, lane, a1);
  Acc4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r.v[j] = mul4_scalar(a1[0][j], s);
  return r;
}
template <int SIN, int RT>
__device__ __forceinline__ void x3_redo_nonfinite(const float* in, __amdgpu_buffer_rsrc_t wr, int n0, int lane,
                                                  f32x4 (&acc)[RT][4], const float (&isc)[RT]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) bad |= !__builtin_isfinite(acc[rt][j][q]);
    if (__builtin_expect(__any(bad), 0)) {
      const Acc4 r = x3_redo_tile<SIN>(in + 16 * rt * SIN, wr, n0, lane, 1.0f / isc[rt]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[rt][j] = r.v[j];
    }
  }
}

// bias + activation of this wave's 64 columns into the LDS tile `out` (row stride SH), row tiles
// 0 .. RT - 1; the MFMA's C map: column = lane & 15, rows 16 rt + 4 (lane >> 4) + q
template <int ACT, int RT>
__device__ __forceinline__ void epilogue_lds_t(const f32x4 (&acc)[RT][4], const float (&bias)[4], int n0, int lane,
                                               float* out, const float* isc = nullptr, float* mx = nullptr) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float m = 0.0f;
    const float u = isc ? isc[rt] : 1.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 16 * j + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = act_t<ACT>((isc ? acc[rt][j][q] * u : acc[rt][j][q]) + bias[j]);
        out[(16 * rt + 4 * g + q) * SH + n] = v;
        m = fmaxf(m, fabsf(v));
      }
    }
    if (mx) mx[rt] = m;
  }
}

// bias[j] = the bias of column n0 + 16 j + (lane & 15), loaded up front
template <int RT>
__device__ __forceinline__ void epilogue_lds(const f32x4 (&acc)[RT][4], const float (&bias)[4], int act, int n0,
                                             int lane, float* out, const float* isc = nullptr, float* mx = nullptr) {
  if (act == 1)
    epilogue_lds_t<1, RT>(acc, bias, n0, lane, out, isc, mx);
  else if (act == 2)
    epilogue_lds_t<2, RT>(acc, bias, n0, lane, out, isc, mx);
  else
    epilogue_lds_t<0, RT>(acc, bias, n0, lane, out, isc, mx);
}

// the LDS tile (rows x HID) to global rows m0.. (ld floats), row-contiguous float4 stores
__device__ __forceinline__ void store_tile(const float* tile, float* dst, int64_t ld, int64_t m0, int64_t M, int cols,
                                           int rows = TM) {
  const int per_row = cols / 4;
  for (int i = threadIdx.x; i < rows * per_row; i += 256) {
    const int rr = i / per_row, c4 = i - rr * per_row;
    if (m0 + rr < M)
      *reinterpret_cast<f32x4*>(dst + (m0 + rr) * ld + 4 * c4) = *reinterpret_cast<const f32x4*>(tile + rr * SH + 4 * c4);
  }
}

// X3: layer 2 and a wide layer 3 in the split-f16 form (layer_cols_run_x3), layer 1 and a narrow
// layer 3 in f32 MFMA either way
template <int RT, bool X3>
__global__ __launch_bounds__(256) void k_mlp3_fwd(Mlp3Args a) {
  constexpr int TR = 16 * RT;  // rows per workgroup
  __shared__ float xs[TR * SX];
  __shared__ float hs1[TR * SH];
  __shared__ float hs2[TR * SH];
  __shared__ f32x4 red[4][RT][64];
  __shared__ uint32_t smax[2][RT];  // X3: max |h1|, |h2| of each row tile (float bits)
  {
    int64_t q = blockIdx.y;
    if (q >= a.groups_a) {  // the second network set (its activations are not kept)
      q -= a.groups_a;
      a.x = a.x_b;
      a.W1 = a.W1_b;
      a.b1 = a.b1_b;
      a.W2 = a.W2_b;
      a.b2 = a.b2_b;
      a.W3 = a.W3_b;
      a.b3 = a.b3_b;
      a.y = a.y_b;
      a.h1 = nullptr;
      a.h2 = nullptr;
    }
    a.x += q * a.gs_x;
    a.W1 += q * a.gs_W1;
    a.b1 += q * a.gs_b1;
    a.W2 += q * a.gs_W2;
    a.b2 += q * a.gs_b2;
    a.W3 += q * a.gs_W3;
    a.b3 += q * a.gs_b3;
    if (a.h1) a.h1 += q * a.gs_h;
    if (a.h2) a.h2 += q * a.gs_h;
    a.y += q * a.gs_y;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * TR;
  const int K1 = a.K1, K1p = (K1 + 15) & ~15;
  const int n0 = wave * 64;
  const int r = lane & 15, g = lane >> 4;

  // layer 2's first weight groups go out first: they depend on nothing, and layer 2 then starts
  // without a round trip
  const __amdgpu_buffer_rsrc_t wr2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.W2), (short)0, HID * HID * 4, 0x00020000);
  f32x4 wb2[PF][X3 ? 1 : 4];
  f32x4 wx2[PF][X3 ? 4 : 1][2];
  if constexpr (X3)
    layer_cols_pre_x3<RT>(wr2, n0, lane, wx2);
  else
    layer_cols_pre<HID / 16>(wr2, n0, lane, wb2);
  if (X3 && tid < 2 * RT) smax[tid / RT][tid % RT] = 0u;
  // ---- the hidden layers' biases and layer 1's weights (their latency overlaps the input
  // staging): W1 [H][K1], lane group g of column n reads k = 16 u + 4 g + t; k >= K1 lands past
  // the buffer's end and reads 0
  float w1[2][4][4], bias1[4], bias2[4];
  {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bias1[j] = a.b1[n0 + 16 * j + r];
      bias2[j] = a.b2[n0 + 16 * j + r];
    }
    const __amdgpu_buffer_rsrc_t wr1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.W1), (short)0, HID * K1 * 4, 0x00020000);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = 16 * u + 4 * g + t, n = n0 + 16 * j + r;
          w1[u][j][t] = (u * 16 < K1p)
                            ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                            wr1, k < K1 ? (n * K1 + k) * 4 : 0x7ffffff0, 0, 0))
                            : 0.0f;
        }
  }

  // ---- the input rows, zero-padded to K1p columns (rows past M: zeros); TR x K1p <= 512 RT
  // elements: a thread's loads all issued before its stores
  {
    float xv[2 * RT];
#pragma unroll
    for (int s = 0; s < 2 * RT; ++s) {
      const int i = tid + 256 * s, rr = i / K1p, k = i - rr * K1p;
      xv[s] = (i < TR * K1p && m0 + rr < a.M && k < K1) ? a.x[(m0 + rr) * a.ldx + k] : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < 2 * RT; ++s) {
      const int i = tid + 256 * s, rr = i / K1p, k = i - rr * K1p;
      if (i < TR * K1p) xs[rr * SX + k] = xv[s];
    }
  }
  __syncthreads();

  // ---- layer 1: K1p <= 32
  {
    f32x4 acc[RT][4] = {};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u * 16 < K1p) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(xs + (16 * rt + r) * SX + 16 * u + 4 * g);
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], w1[u][j][t], acc[rt][j], 0, 0, 0);
        }
      }
    }
    if constexpr (X3) {
      float mx[RT];
      epilogue_lds<RT>(acc, bias1, a.act1, n0, lane, hs1, nullptr, mx);
      tile_max_publish<RT>(mx, smax[0]);
    } else {
      epilogue_lds<RT>(acc, bias1, a.act1, n0, lane, hs1);
    }
  }
  __syncthreads();
  if (a.h1) store_tile(hs1, a.h1, a.ldh, m0, a.M, HID, TR);

  // ---- layer 2
  const int N3 = a.N3;
  const __amdgpu_buffer_rsrc_t wr3 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.W3), (short)0, N3 * HID * 4, 0x00020000);
  f32x4 w3[4];  // the narrow output layer's weights (N3 <= 16), issued before layer 2's epilogue
  {
    f32x4 acc[RT][4] = {};
    float sc[RT], isc[RT];
    if constexpr (X3) {
      tile_scales<RT>(smax[0], sc, isc);
      layer_cols_run_x3<SH, RT>(hs1, sc, wr2, n0, lane, acc, wx2);
      x3_redo_nonfinite<SH, RT>(hs1, wr2, n0, lane, acc, isc);
    } else {
      layer_cols_run<SH, HID / 16, RT>(hs1, wr2, n0, lane, acc, reinterpret_cast<f32x4(&)[PF][4]>(wb2));
    }
    if (N3 <= 16) {
#pragma unroll
      for (int uu = 0; uu < 4; ++uu)
        w3[uu] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr3, (r * HID + 16 * (wave * 4 + uu) + 4 * g) * 4, 0, 0));
    }
    MH_SCHED_FENCE();
    if constexpr (X3) {
      float mx[RT];
      epilogue_lds<RT>(acc, bias2, a.act2, n0, lane, hs2, isc, mx);
      if (N3 > 16) tile_max_publish<RT>(mx, smax[1]);
    } else {
      epilogue_lds<RT>(acc, bias2, a.act2, n0, lane, hs2);
    }
  }
  __syncthreads();
  if (a.h2) store_tile(hs2, a.h2, a.ldh, m0, a.M, HID, TR);

  // ---- layer 3
  if (N3 <= 16) {
    // one 16-column block; wave w contracts k in [64 w, 64 w + 64), the four partial tiles added
    // in wave order
    f32x4 acc[RT] = {};
#pragma unroll
    for (int uu = 0; uu < 4; ++uu) {
      const int u = wave * 4 + uu;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(hs2 + (16 * rt + r) * SH + 16 * u + 4 * g);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], w3[uu][t], acc[rt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) red[wave][rt][lane] = acc[rt];
    __syncthreads();
    if (wave < RT) {  // wave rt sums row tile rt's four partials
      const int rt = wave;
      f32x4 sum = red[0][rt][lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) sum = add4_scalar(sum, red[w][rt][lane]);
      const int n = lane & 15;
      if (n < N3) {
        const float bv = a.b3[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t row = m0 + 16 * rt + 4 * g + q;
          if (row < a.M) a.y[row * a.ldy + n] = act_f(sum[q] + bv, a.act3);
        }
      }
    }
  } else {
    // N3 = 64 c: wave w takes output columns [N3 / 4 * w, ...) in 16-column blocks of 64-wide passes
    // (with sqsum: also into the free hs1 tile, N3 <= HID)
    float sc3[RT], isc3[RT];
    if constexpr (X3) tile_scales<RT>(smax[1], sc3, isc3);
    for (int nb = wave * 64; nb < N3; nb += 256) {
      f32x4 acc[RT][4] = {};
      if constexpr (X3) {
        f32x4 wx3[PF][4][2];
        layer_cols_pre_x3<RT>(wr3, nb, lane, wx3);
        layer_cols_run_x3<SH, RT>(hs2, sc3, wr3, nb, lane, acc, wx3);
        x3_redo_nonfinite<SH, RT>(hs2, wr3, nb, lane, acc, isc3);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[rt][j] = mul4_scalar(acc[rt][j], isc3[rt]);
      } else {
        layer_cols<SH, HID / 16, RT>(hs2, wr3, nb, lane, acc);
      }
      const int c = lane & 15;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nb + 16 * j + c;
          const float bv = a.b3[n];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t row = m0 + 16 * rt + 4 * g + q;
            const float v = act_f(acc[rt][j][q] + bv, a.act3);
            if (row < a.M) a.y[row * a.ldy + n] = v;
            if (a.sqsum) hs1[(16 * rt + 4 * g + q) * SH + n] = v;
          }
        }
    }
    if (a.sqsum) {
      // V = sum_n y^2 per row in k_square_sum's order (lane l: columns 4l .. 4l + 3 of each
      // 256-column pass, in order; then the xor butterfly 32 .. 1): its bits
      __syncthreads();
      for (int rr = wave; rr < TR; rr += 4) {
        float s = 0.0f;
        for (int c0 = 0; c0 < N3; c0 += 256) {
          const int cc = c0 + 4 * lane;
          if (cc + 3 < N3) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(hs1 + rr * SH + cc);
            s = s + v[0] * v[0];
            s = s + v[1] * v[1];
            s = s + v[2] * v[2];
            s = s + v[3] * v[3];
          }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s = s + __shfl_xor(s, off, 64);
        if (lane == 0 && m0 + rr < a.M) a.sqsum[m0 + rr] = s;
      }
    }
  }
}

// ------------------------------------------------------------------ backward: the input-gradient chain
// The contraction of a backward product runs over the weight's OUTPUT index (dh = g W, W [N][K]):
// in MFMA t of group u, lane group g contracts weight row 16 u + 4 g + t, so each lane's four B
// values lie in four rows (scalar loads, 64 consecutive bytes per 16 lanes). Rows past `nrows` read 0.
// (the weight rows are HID floats long; rows at or past `nrows` lie beyond the buffer resource)
// Same load ring as layer_cols (depth PFT: sixteen scalars a group), group u issued PFT - 1 groups ahead.
constexpr int PFT = MH_MLP_PFT;
template <int G>
__device__ __forceinline__ void wring_t_load(__amdgpu_buffer_rsrc_t wr, int n0, int lane, int u, float (&dst)[4][4]) {
  const int c = lane & 15, g = lane >> 4;
  const int voff = ((4 * g) * HID + n0 + c) * 4;  // + (t HID + 16 j) 4: immediate offsets
  const int soff = u * 16 * HID * 4;
#ifdef MH_MLP_EXP_PACKED  // cost-attribution experiment only: fragment-ordered addresses (wrong results)
  for (int j = 0; j < 4; ++j) {
    const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  wr, (((n0 / 16 + j) * G + u) * 64 + lane) * 16, 0, 0));
    for (int t = 0; t < 4; ++t) dst[j][t] = v[t];
  }
  return;
#endif
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t)
      dst[j][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, voff + (t * HID + 16 * j) * 4,
                                                                               soff, 0));
}

template <int G, int D = PFT>
__device__ __forceinline__ void layer_cols_t_pre(__amdgpu_buffer_rsrc_t wr, int n0, int lane, float (&wb)[D][4][4]) {
#pragma unroll
  for (int p = 0; p < D - 1; ++p)
    if (p < G) wring_t_load<G>(wr, n0, lane, p, wb[p]);
}

template <int G, int D = PFT, int RT = 1>
__device__ __forceinline__ void layer_cols_t_run(const float* in, int sin, __amdgpu_buffer_rsrc_t wr, int n0, int lane,
                                                 f32x4 (&acc)[RT][4], float (&wb)[D][4][4]) {
  const int c = lane & 15, g = lane >> 4;
  const float* arow = in + c * sin + 4 * g;
  f32x4 a_cur[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) a_cur[rt] = *reinterpret_cast<const f32x4*>(arow + 16 * rt * sin);
#pragma unroll
  for (int u = 0; u < G; ++u) {
    if (u + D - 1 < G) wring_t_load<G>(wr, n0, lane, u + D - 1, wb[(u + D - 1) % D]);
    f32x4 a_nxt[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      a_nxt[rt] = u + 1 < G ? *reinterpret_cast<const f32x4*>(arow + 16 * rt * sin + 16 * (u + 1)) : a_cur[rt];
    MH_SCHED_FENCE();
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[rt][t], wb[u % D][j][t], acc[rt][j], 0, 0, 0);
    MH_SCHED_FENCE();
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a_cur[rt] = a_nxt[rt];
  }
}

template <int G, int D = PFT, int RT = 1>
__device__ __forceinline__ void layer_cols_t(const float* in, int sin, __amdgpu_buffer_rsrc_t wr, int n0, int lane,
                                             f32x4 (&acc)[RT][4]) {
  float wb[D][4][4];
  layer_cols_t_pre<G, D>(wr, n0, lane, wb);
  layer_cols_t_run<G, D, RT>(in, sin, wr, n0, lane, acc, wb);
}

// the output-gradient contraction over W3's N3 rows, N3 a multiple of 64
template <int RT>
__device__ __forceinline__ void layer_cols_t_n3(const float* in, __amdgpu_buffer_rsrc_t wr, int N3, int n0, int lane,
                                                f32x4 (&acc)[RT][4]) {
  if (N3 == 64)
    layer_cols_t<4, 3, RT>(in, SH, wr, n0, lane, acc);
  else if (N3 == 128)
    layer_cols_t<8, 3, RT>(in, SH, wr, n0, lane, acc);
  else if (N3 == 192)
    layer_cols_t<12, 3, RT>(in, SH, wr, n0, lane, acc);
  else
    layer_cols_t<16, 3, RT>(in, SH, wr, n0, lane, acc);
}

// this wave's 64 columns of the forward activations h (rows m0.., row stride ldh) in row tiles
// 0 .. RT - 1, for the gradient epilogue; issued before the layer's MFMAs so that their latency
// hides behind them (rows past M read 0)
template <int RT>
__device__ __forceinline__ void load_h_tile(const float* h, int64_t ldh, int64_t m0, int64_t M, int n0, int lane,
                                            float (&hv)[RT][4][4]) {
  const int c = lane & 15, g = lane >> 4;
  const int64_t rows = M - m0 < 16 * RT ? M - m0 : 16 * RT;
  const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(h + m0 * ldh), (short)0, (int)(((rows - 1) * ldh + HID) * 4), 0x00020000);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 16 * rt + 4 * g + q;
        hv[rt][j][q] = rr < rows ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                 hr, (int)((rr * ldh + n0 + 16 * j + c) * 4), 0, 0))
                                 : 0.0f;
      }
}

template <int ACT>
__device__ __forceinline__ float act_grad_t(float d, float t) {  // gemm.hip act_grad
  if constexpr (ACT == 1) return t > 0.0f ? d : 0.0f;
  if constexpr (ACT == 2) return d * (1.0f - t * t);
  return d;
}

// dh = acc (this wave's 64 columns) -> g = dh * act'(h) into the LDS tile `out`; rows past M: 0
template <int ACT, int RT>
__device__ __forceinline__ void grad_epilogue_t(const f32x4 (&acc)[RT][4], const float (&hv)[RT][4][4], int n0,
                                                int lane, int64_t m0, int64_t M, float* out) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 16 * j + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = 16 * rt + 4 * g + q;
        out[rr * SH + n] = m0 + rr < M ? act_grad_t<ACT>(acc[rt][j][q], hv[rt][j][q]) : 0.0f;
      }
    }
}

template <int RT>
__device__ __forceinline__ void grad_epilogue(const f32x4 (&acc)[RT][4], const float (&hv)[RT][4][4], int act, int n0,
                                              int lane, int64_t m0, int64_t M, float* out) {
  if (act == 1)
    grad_epilogue_t<1, RT>(acc, hv, n0, lane, m0, M, out);
  else if (act == 2)
    grad_epilogue_t<2, RT>(acc, hv, n0, lane, m0, M, out);
  else
    grad_epilogue_t<0, RT>(acc, hv, n0, lane, m0, M, out);
}

// The output layer's weight / bias gradient partials per 16-row block (Mlp3BwdArgs::pdw3) from the
// staged output gradient (g3 rows, LDS) and this wave's 64 columns of h2 (hv, the MFMA C layout:
// rows 4 g + q in lane group g): each lane gathers its column's 16 rows by shuffles and adds
// g3[r][o] h2[r][n] over the block's rows in order, k_head_backward's expression and order.
template <int RT>
__device__ __forceinline__ void w3_partials(const float* gs3, const float (&hv)[RT][4][4], int N3, int n0, int lane,
                                            int wave, int64_t m0, int64_t M, float* pdw, float* pdb) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int64_t r0 = m0 + 16 * rt;
    if (r0 >= M) break;
    const int nr = M - r0 < 16 ? (int)(M - r0) : 16;
    const int64_t blk = r0 / 16;
    const float* gr = gs3 + 16 * rt * SH;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float hc[16];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) hc[4 * gg + qq] = __shfl(hv[rt][j][qq], c + 16 * gg, 64);
      for (int o = 0; o < N3; ++o) {
        float s = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (r < nr) s = s + gr[r * SH + o] * hc[r];
        if (g == (o & 3)) pdw[(blk * N3 + o) * HID + n0 + 16 * j + c] = s;
      }
    }
    if (pdb && wave == 0 && lane < N3) {
      float s = 0.0f;
      for (int r = 0; r < nr; ++r) s = s + gr[r * SH + lane];
      pdb[blk * N3 + lane] = s;
    }
  }
}

// NARROW (N3 <= 16): the W2 product's weight ring is issued before the W3 product; the wide form
// (N3 a multiple of 64) has no registers for that beside the W3 product's own ring. RT row tiles
// of 16 per wave (the workgroup's 16 RT rows): each weight fragment feeds RT MFMAs.
template <bool NARROW, int RT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT == 1 ? 2 : 1))) void k_mlp3_bwd(
    Mlp3BwdArgs a) {
  constexpr int TR = 16 * RT;
  __shared__ float gs3[TR * SH];  // the output gradient tile (N3 <= 256 columns)
  __shared__ float gs2[TR * SH];
  __shared__ float gs1[TR * SH];
  __shared__ f32x4 red[4][RT][2][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * TR;
  const int N3 = a.N3, K1 = a.K1, n0 = wave * 64;
  const int N3p = (N3 + 15) & ~15;
  f32x4 dxa[RT][2] = {};
  for (int q = 0; q < a.groups; ++q) {
    const float* dy = a.dy + q * a.gs_dy;
    const float* h1 = a.h1 + q * a.gs_h;
    const float* h2 = a.h2 + q * a.gs_h;
    const float* W1 = a.W1 + q * a.gs_W1;
    const float* W2 = a.W2 + q * a.gs_W2;
    const float* W3 = a.W3 + q * a.gs_W3;
    if (q > 0) __syncthreads();  // the previous group's tiles are read
    // the W2 product's first weight groups and the h2 tile go out before the output-gradient
    // staging: they depend on nothing, and their round trip overlaps it and the W3 product
    const __amdgpu_buffer_rsrc_t wr2 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W2), (short)0, HID * HID * 4, 0x00020000);
    float wb2[PFT][4][4];
    if constexpr (NARROW) layer_cols_t_pre<HID / 16>(wr2, n0, lane, wb2);
    float hv2[RT][4][4];
    load_h_tile<RT>(h2, a.ldh, m0, a.M, n0, lane, hv2);
    if (a.sq_dv) {  // LyapunovValue: dy = dV (2 y) (k_square_sum_bwd's expression), kept in g3
      for (int i = tid; i < TR * N3p; i += 256) {
        const int rr = i / N3p, k = i - rr * N3p;
        float v = 0.0f;
        if (m0 + rr < a.M && k < N3) {
          v = a.sq_dv[m0 + rr] * (2.0f * dy[(m0 + rr) * a.ldy + k]);
          a.g3[(m0 + rr) * a.ldy + k] = v;
        }
        gs3[rr * SH + k] = v;
      }
    } else {
      for (int i = tid; i < TR * N3p; i += 256) {
        const int rr = i / N3p, k = i - rr * N3p;
        gs3[rr * SH + k] = (m0 + rr < a.M && k < N3) ? dy[(m0 + rr) * a.ldy + k] : 0.0f;
      }
    }
    __syncthreads();
    // dh2 = g3 W3 (contraction over W3's N3 rows), g2 = dh2 * act2'(h2)
    {
      const __amdgpu_buffer_rsrc_t wr =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W3), (short)0, N3 * HID * 4, 0x00020000);
      f32x4 acc[RT][4] = {};
      if constexpr (NARROW)
        layer_cols_t<1, PFT, RT>(gs3, SH, wr, n0, lane, acc);
      else
        layer_cols_t_n3<RT>(gs3, wr, N3, n0, lane, acc);
      grad_epilogue<RT>(acc, hv2, a.act2, n0, lane, m0, a.M, gs2);
      if constexpr (NARROW) {
        if (a.pdw3) w3_partials<RT>(gs3, hv2, N3, n0, lane, wave, m0, a.M, a.pdw3 + q * a.s_part3,
                                    a.pdb3 ? a.pdb3 + q * a.s_part3 : nullptr);
      }
    }
    __syncthreads();
    if (a.g2) store_tile(gs2, a.g2 + q * a.gs_g, a.ldg, m0, a.M, HID, TR);
    // dh1 = g2 W2, g1 = dh1 * act1'(h1)
    {
      float hv[RT][4][4];
      load_h_tile<RT>(h1, a.ldh, m0, a.M, n0, lane, hv);
      f32x4 acc[RT][4] = {};
      if constexpr (NARROW)
        layer_cols_t_run<HID / 16, PFT, RT>(gs2, SH, wr2, n0, lane, acc, wb2);
      else
        layer_cols_t<HID / 16, 3, RT>(gs2, SH, wr2, n0, lane, acc);  // (registers: the wide form keeps depth 3)
      grad_epilogue<RT>(acc, hv, a.act1, n0, lane, m0, a.M, gs1);
    }
    __syncthreads();
    if (a.g1) store_tile(gs1, a.g1 + q * a.gs_g, a.ldg, m0, a.M, HID, TR);
    // dx += g1 W1 (W1 [H][K1]: contraction over its H rows, wave w rows [64 w, 64 w + 64); two
    // 16-column blocks of K1 <= 32)
    if (a.dx) {
      const int c = lane & 15, g = lane >> 4;
      const __amdgpu_buffer_rsrc_t wr =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W1), (short)0, HID * K1 * 4, 0x00020000);
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int u = wave * 4 + uu;
        f32x4 av[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          av[rt] = *reinterpret_cast<const f32x4*>(gs1 + (16 * rt + c) * SH + 16 * u + 4 * g);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          float bv[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int k = 16 * u + 4 * g + t, col = 16 * cb + c;
            bv[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  wr, col < K1 ? (k * K1 + col) * 4 : 0x7ffffff0, 0, 0));
          }
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
              dxa[rt][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rt][t], bv[t], dxa[rt][cb], 0, 0, 0);
        }
      }
    }
  }
  if (a.dx) {  // the four waves' partials (rows of W1 they contracted) added in wave order
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      red[wave][rt][0][lane] = dxa[rt][0];
      red[wave][rt][1][lane] = dxa[rt][1];
    }
    __syncthreads();
    if (wave < RT) {  // wave rt: row tile rt
      const int rt = wave;
      const int c = lane & 15, g = lane >> 4;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        f32x4 sum = red[0][rt][cb][lane];
#pragma unroll
        for (int w = 1; w < 4; ++w) sum = add4_scalar(sum, red[w][rt][cb][lane]);
        const int col = 16 * cb + c;
        if (col < K1) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int64_t row = m0 + 16 * rt + 4 * g + qq;
            if (row < a.M) a.dx[row * a.ldx + col] = sum[qq];
          }
        }
      }
    }
  }
}

}  // namespace

bool mlp3_supported(int64_t M, int K1, int H, int N3) {
  return M > 0 && K1 >= 1 && K1 <= K1P && H == HID && N3 >= 1 && (N3 <= 16 || (N3 % 64 == 0 && N3 <= 256));
}

hipError_t launch_mlp3_backward(const Mlp3BwdArgs& a, hipStream_t st) {
  if (!mlp3_supported(a.M, a.K1, a.H, a.N3) || a.groups < 1) return hipErrorInvalidValue;
  // one row tile per wave: two (MH_MLP_BWD_RT=2, one workgroup per CU for its 116 KB of LDS)
  // measured slower (10,240 rows: 38.7 vs 27.4 us; N3 = 256: 34.7 vs 30.0; tools/mlp3_bench.py)
  static const int force_rt = [] {
    const char* e = getenv("MH_MLP_BWD_RT");
    return e ? atoi(e) : 0;
  }();
  if (force_rt != 2) {
    const int64_t tiles = (a.M + TM - 1) / TM;
    if (a.N3 <= 16)
      k_mlp3_bwd<true, 1><<<(unsigned)tiles, 256, 0, st>>>(a);
    else
      k_mlp3_bwd<false, 1><<<(unsigned)tiles, 256, 0, st>>>(a);
  } else {
    const int64_t tiles = (a.M + 31) / 32;
    if (a.N3 <= 16)
      k_mlp3_bwd<true, 2><<<(unsigned)tiles, 256, 0, st>>>(a);
    else
      k_mlp3_bwd<false, 2><<<(unsigned)tiles, 256, 0, st>>>(a);
  }
  return hipGetLastError();
}

// the forward's row-tile mode for the launches that follow (mh_mlp3_set_row_tiles): 0 the default
// (RT = 2), -1 the CU-count rule, 1 .. 4 fixed. Host state read at launch (and so at capture).
static int g_row_tiles = 0;

void mlp3_set_row_tiles(int mode) { g_row_tiles = mode; }

// CU count of the (single) device this process drives, queried once (256 on the MI355X)
static int64_t device_cus() {
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

hipError_t launch_mlp3_forward(const Mlp3Args& a_in, int groups, hipStream_t st) {
  if (!mlp3_supported(a_in.M, a_in.K1, a_in.H, a_in.N3) || groups < 1 || a_in.groups_b < 0) return hipErrorInvalidValue;
  Mlp3Args a = a_in;
  a.groups_a = groups;
  groups += a.groups_b;
  // Row tiles per wave (RT): a workgroup streams each weight matrix once per 16 RT rows, and
  // costs about (10 + 10 RT) us at the Lyapunov shape (one per CU; two co-resident on a CU take
  // 1.7x one). Alone, the fastest grid is the fewest row tiles per workgroup that still fit one
  // workgroup per CU (MH_MLP_RT=auto): RT = 3 at 10,240 rows (40 vs 50 us at RT = 2 / 4), RT = 3
  // for the twin critics' 2 x 5,120 (24.9 vs 30.6 us), RT = 1 at 2,560 (13.7 vs 16.5)
  // (tools/mlp3_bench.py, tools/r04_rt3.sh, r04_rt3b.sh). Inside the update, though, the critic and
  // Lyapunov branches run these launches side by side, and RT = 3's 119 KB of LDS leaves no room
  // for the other branch's workgroup on the CU (the critics + targets pair took 88 us there beside
  // the Lyapunov forward at RT = 3 vs 49 us at RT = 2): the bench step is 1.2 % faster with RT = 2
  // everywhere (1.120-1.127 vs 1.110-1.112 B env-steps/s, alternating runs on one box,
  // tools/r04_iter13.sh), so RT = 2 (79 KB, two workgroups per CU) is the default.
  // MH_MLP_RT = 1 / 2 / 3 / 4 forces, "auto" selects as above.
  static const int force_rt = [] {
    const char* e = getenv("MH_MLP_RT");
    if (!e) return -1;
    if (std::strcmp(e, "auto") == 0) return 0;
    return atoi(e);
  }();
  // MH_MLP_RT wins; else the caller's mode (mh_mlp3_set_row_tiles: a launch it knows runs alone,
  // such as the policy step's critic forward, takes the "auto" grid); else RT = 2
  int rt = force_rt >= 0 ? force_rt : (g_row_tiles == 0 ? 2 : (g_row_tiles < 0 ? 0 : g_row_tiles));
  if (rt < 1 || rt > 4) {
    const int64_t cus = device_cus();
    auto wgs = [&](int r) { return (a.M + 16 * r - 1) / (16 * r) * (int64_t)groups; };
    rt = 0;
    for (int r = 1; r <= 4 && !rt; ++r)
      if (wgs(r) <= cus) rt = r;
    if (!rt) rt = 2;
  }
  // the split-f16 hidden layers (k_mlp3_fwd<., true>) unless MH_MLP_X3=0
  static const bool x3 = [] {
    const char* e = getenv("MH_MLP_X3");
    return !(e && e[0] == '0');
  }();
  const unsigned gy = (unsigned)groups;
  const dim3 grid((unsigned)((a.M + 16 * rt - 1) / (16 * rt)), gy);
  if (x3) {
    switch (rt) {
      case 1: k_mlp3_fwd<1, true><<<grid, 256, 0, st>>>(a); break;
      case 3: k_mlp3_fwd<3, true><<<grid, 256, 0, st>>>(a); break;
      case 4: k_mlp3_fwd<4, true><<<grid, 256, 0, st>>>(a); break;
      default: k_mlp3_fwd<2, true><<<grid, 256, 0, st>>>(a); break;
    }
  } else {
    switch (rt) {
      case 1: k_mlp3_fwd<1, false><<<grid, 256, 0, st>>>(a); break;
      case 3: k_mlp3_fwd<3, false><<<grid, 256, 0, st>>>(a); break;
      case 4: k_mlp3_fwd<4, false><<<grid, 256, 0, st>>>(a); break;
      default: k_mlp3_fwd<2, false><<<grid, 256, 0, st>>>(a); break;
    }
  }
  return hipGetLastError();
}

}  // namespace mh
