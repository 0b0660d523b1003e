// policy_x3.h — shared device pieces of the split-f16 policy MLP (StochaPolicy 256 x 256,
// RL/apprfunc/mlp.py:111-136): the packed-parameter layout, the power-of-two scaling and the
// hi/lo f16 splits. Used by the standalone policy kernels (policy_mlp.hip) and by the fused
// horizon sampler (sample_fused.hip), which must compute bit-identical logits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mh {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

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
// W2 again, as exact three-way bf16 splits for the split-bf16 layer-2 kernel (k_policy_forward_x6):
// W2x6 [ib 8][ob 8][s 2][split 3][lane 64][8 bf16] — chunk ib (48 fragments of 1 KB, the unit
// one workgroup stages through LDS) holds, for lane l and element j of k-step s, the weight
//   W2[ob*32 + (l & 31)][ib*32 + (j & 3) + 8 (j >> 2) + 16 s + 4 (l >> 5)]
// i.e. the hidden unit that accumulator register 8 s + j of a layer-1 block holds on that lane.
constexpr int PM_X6_FRAGS = 48;                                    // fragments per chunk
constexpr int64_t PM_X6_FLOATS = (int64_t)PM_NB * PM_X6_FRAGS * 64 * 4;  // 8 bf16 = 4 floats per lane
__host__ __device__ constexpr int64_t pm_off_w2x6(int K1) { return (pm_off_b3(K1) + 32 + 63) / 64 * 64; }
// The split-f16 kernel's operands (k_policy_forward_x3), every weight scaled by a power of two
// sw1 / sw2 / sw3 (max |.| of the layer in [2^13, 2^14]) and split into two f16 (hi, lo):
//   W1x3 [blk 8][split 2][lane 64][8 f16]        W1[blk*32 + (l & 31)][8 (l >> 5) + j] * sw1,
//                                                b1 at k = D (constant-1 input), 0 beyond
//   W2x3 [ib 8][ob 8][s 2][split 2][lane 64][8 f16]   the W2x6 k order, * sw2
//   W3x3 [ob 8][s 2][split 2][lane 64][8 f16]    the A operand of layer 3 on v_mfma_f32_16x16x32_f16
//                                                (N3 <= 8): row m = l & 15, k-group g = l >> 4 holds
//                                                W3[m & 7][ob*32 + (j & 3) + 8 (j >> 2) + 16 s + 4 (g >> 1)] * sw3
//                                                when (m < 8) == (g even), else 0 (pm_l3_row_half)
constexpr int PM_X3_FRAGS = 32;                                      // W2x3 fragments per chunk
constexpr int64_t PM_X3_FLOATS = (int64_t)PM_NB * PM_X3_FRAGS * 64 * 4;
constexpr int64_t PM_X3_W1_FLOATS = (int64_t)PM_NB * 2 * 64 * 4;
constexpr int64_t PM_X3_W3_FLOATS = (int64_t)PM_NB * 4 * 64 * 4;
__host__ __device__ constexpr int64_t pm_off_w2x3(int K1) { return pm_off_w2x6(K1) + PM_X6_FLOATS; }
__host__ __device__ constexpr int64_t pm_off_w1x3(int K1) { return pm_off_w2x3(K1) + PM_X3_FLOATS; }
__host__ __device__ constexpr int64_t pm_off_w3x3(int K1) { return pm_off_w1x3(K1) + PM_X3_W1_FLOATS; }
// scalars: the raw layer magnitudes of k_policy_scales (pm_scales() derives sw1..3 and the bounds
// |H1| <= R1 max(1, max |obs|), |H2| <= R2 max(1, |H1|))
__host__ __device__ constexpr int64_t pm_off_scal(int K1) { return pm_off_w3x3(K1) + PM_X3_W3_FLOATS; }
// [0..4] the final magnitudes, [8 + 5 wg + q] k_policy_scales' per-workgroup partials
constexpr int PM_SC_WG = 32;  // k_policy_scales workgroups (8 waves, one W2 row per wave)
__host__ __device__ constexpr int64_t pm_packed_floats(int K1) { return pm_off_scal(K1) + (8 + 5 * PM_SC_WG + 63) / 64 * 64; }

__device__ __forceinline__ int pm_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ float pm_pow2(int e) {  // 2^e for e in [-126, 127]
  return __uint_as_float((uint32_t)(127 + e) << 23);
}
__device__ __forceinline__ int pm_scale_exp(float bound) {  // 14 - ceil(log2(bound)), clamped
  if (!(bound > 0.0f) || bound != bound) return 0;
  int e;
  (void)frexpf(bound, &e);  // bound = m 2^e, m in [0.5, 1): bound <= 2^e
  const int k = 14 - e;
  return k < -40 ? -40 : (k > 40 ? 40 : k);
}

// sw1..3, their inverses, and R1, R2 rounded up (the f32 sums above are upper bounds only up to
// their own rounding) from the raw magnitudes
struct PmScales {
  float sw[3], isw[3], R1, R2;
};
__device__ __forceinline__ PmScales pm_scales(const float* scal) {
  PmScales r;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int e = pm_scale_exp(scal[q]);
    r.sw[q] = pm_pow2(e);
    r.isw[q] = pm_pow2(-e);
  }
  r.R1 = scal[3] * (1.0f + 1.0f / 1024.0f);
  r.R2 = scal[4] * (1.0f + 1.0f / 1024.0f);
  return r;
}

__device__ __forceinline__ void split2h(float a, _Float16& hi, _Float16& lo) {
  hi = (_Float16)a;
  lo = (_Float16)(a - (float)hi);  // the remainder is exact in f32
}

// The kernel's hot splits, three VALU per pair: hi = both values rounded to f16 (one packed
// convert), lo = f16(a - hi) by v_fma_mix (the f16 hi read as a mixed-precision operand; the
// f32 difference is exact, rounded once). Written out because the compiler's lowering of
// (_Float16)(a - (float)hi) spends a convert back, a subtract and a second convert per value.
__device__ __forceinline__ void split2h_pair(float a, float b, float one, uint32_t& hi, uint32_t& lo) {
  asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(a), "v"(b), "v"(one));
}
// max(x, 0) without the canonicalising max(x, x) the compiler adds for values it did not
// produce itself (MFMA results)
__device__ __forceinline__ float relu_raw(float x) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return r;
}
// The layer splits of the split-f16 MLP: hi = f16(relu(a k)), lo = f16(relu(a k) - hi) for a pair
// (a, b), k a power of two (the layer's rescale; relu commutes with it). The products a k are
// plain C++ (compiler-visible VALU): a and b are usually MFMA results, and an inline-asm reader of
// an MFMA destination gets no hazard wait states from the compiler (the round-5 first cut fed them
// straight to the asm max and read unfinished accumulators). Then split2h_pair's three-instruction
// split with the fma_mix multiplier as the inline constant 1.0 (no register). 7 VALU per pair,
// none of them packed-f32.
__device__ __forceinline__ void split2h_relu_scaled(float a, float b, float k, uint32_t& hi, uint32_t& lo) {
  const float ra = relu_raw(a * k), rb = relu_raw(b * k);
  asm("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
      "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(ra), "v"(rb));
}
// The layer-2 accumulator starts at the bias in the accumulator's units: b2 * sw2 * 2^ex1 (the
// products are (W2 sw2)(H1 2^ex1)); cb = sw2 * 2^ex1 (a power of two: exact). The H2 split is then
// split2h_relu_scaled(acc, k23), k23 = 2^(ex2 - ex1) / sw2.
__device__ __forceinline__ float pm_bias_unit(float sw2, int ex1) { return sw2 * pm_pow2(ex1); }

// Layer 3 on v_mfma_f32_16x16x32_f16 without moving the H2 split across lanes. The split of
// k-step s of an H2 block is, read as that MFMA's B operand (lane l = column l & 15, k-group
// g = l >> 4), env l & 31's eight units of row half l >> 5: k-groups 0 and 2 belong to env
// column n = l & 15 and groups 1 and 3 to env 16 + n. W3x3 puts the weights of the even groups in
// output rows 0..7 and those of the odd groups in rows 8..15 (zeros elsewhere), so the 16x16
// result holds outputs 0..7 of env n in rows 0..7 and of env 16 + n in rows 8..15 — every row
// real for N3 = 8, where a 32x32x16 tile pads 32 rows — and lane l ends up with outputs
// 4 ((l >> 4) & 1) + i of env pm_l3_env(l). Per block 2 k-steps x 3 products (lo·hi, hi·lo,
// hi·hi) on one accumulator.
__device__ __forceinline__ int pm_l3_env(int lane) { return 16 * (lane >> 5) + (lane & 15); }
__host__ __device__ constexpr bool pm_l3_row_half(int lane) { return ((lane & 15) < 8) == (((lane >> 4) & 1) == 0); }

}  // namespace mh
