// sample_fused.hip — the sampler's whole horizon (RL/trainer/sampler/base.py:118-222 run for
// `sample_batch_size` lockstep steps) as ONE persistent kernel per sample(), for the default
// StochaPolicy shape (256 x 256, D <= 15).
//
// Why: the two-kernel lockstep (k_policy_forward_x3, MFMA-bound, then k_rollout, latency-bound
// at one wave per SIMD) alternates two phases that each leave the other unit of every SIMD idle,
// and every lockstep re-reads and re-writes the env state through the cache hierarchy. Here each
// workgroup owns 256 envs for the whole horizon, 8 waves:
//   waves 0-3  policy waves: the split-f16 MLP (policy_x3.h, the same MFMA sequence on every
//              accumulator as k_policy_forward_x3, so the same logits bit for bit), one 32-env
//              tile per wave per pass, W2 streamed through LDS by LDS-DMA and shared by the four
//              policy waves (they synchronise among themselves through an LDS counter, not
//              s_barrier, so the env waves never wait on the policy's chunk handoffs);
//   waves 4-7  env waves: one env per lane, the env's state (state, Rd_last, steps, Philox
//              counter, deque length / position) kept in REGISTERS across the horizon; each
//              lockstep samples the TanhGauss action, steps the env, autoresets and pushes the
//              ring record exactly as k_rollout<Env, true> does.
// The 256 envs are two halves H0 (env waves 4, 5) and H1 (6, 7), pipelined so MFMA and VALU
// work of the same CU overlap (the policy waves and the env waves share each SIMD):
//   phase A(t): policy(H0, obs after t-1)  ||  env step t of H1 (logits from B(t-1))
//   phase B(t): policy(H1, obs after t)    ||  env step t of H0 (logits from A(t))
// with one workgroup barrier between phases; observations and logits pass through LDS only.
// Windows: every full deque of lockstep t is recorded as (lane | oldest slot << 6) in a per-wave,
// rank-ordered list; the rings hold n + H - 1 records (mh_nstep_reserve) so every window of the
// horizon is still intact when k_emit_cells copies them, in the reference's order (lockstep major,
// env index within a lockstep: base.py:178-213), into the replay store after the kernel.
#include <type_traits>

#include "policy_x3.h"
#include "reset_draw.h"
#include "rollout.h"
#include "sample_fused.h"

#ifdef MH_FUSED_EXP_NO_MFMA  // cost-attribution experiment: the policy pass without its MFMAs (garbage logits)
#define MH_MFMA(a, b, c) (c)
#elif defined(MH_FUSED_EXP_MFMA16)
// clock experiment (garbage logits): each 32x32x16 product replaced by two v_mfma_f32_16x16x32_f16
// of the same flops into two quarters of the accumulator (the DVFS give-back of the shape)
namespace mh {
typedef float f32x4e __attribute__((ext_vector_type(4)));
template <class V, class A>
__device__ __forceinline__ V mfma16_pair(const A& a, const A& b, V c) {
  f32x4e lo = {c[0], c[1], c[2], c[3]}, hi = {c[4], c[5], c[6], c[7]};
  lo = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, lo, 0, 0, 0);
  hi = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, hi, 0, 0, 0);
  c[0] = lo[0]; c[1] = lo[1]; c[2] = lo[2]; c[3] = lo[3];
  c[4] = hi[0]; c[5] = hi[1]; c[6] = hi[2]; c[7] = hi[3];
  return c;
}
}  // namespace mh
#define MH_MFMA(a, b, c) mfma16_pair(a, b, c)
#else
#define MH_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0)
#endif

namespace mh {

// ------------------------------------------------------------------ policy waves
struct PolicyLds {
  uint4* c0;            // W2 chunk buffers (PM_X3_FRAGS * 64 records each)
  uint4* c1;
  uint32_t c0_lds;      // their LDS byte addresses (the chunk DMA's M0 values)
  uint32_t c1_lds;
  const uint4* w3;      // layer-3 operands [ob][s][split][lane] (16x16x32 A fragments)
  const float* b2;      // layer-2 bias, [256]
  const uint4* w1;      // layer-1 fragments [blk][split][lane] (LDS: no memory loads inside a pass)
  const float* obs;     // [256][D] observations of the workgroup's envs
  float* lgt;           // [256][N3] logits out
  uint32_t* bar;        // policy-wave barrier counter
  int64_t* err;         // device error word (bounded waits that timed out)
};

// 16-byte LDS-DMA (global_load_lds_dwordx4: this lane's 16 bytes at gsrc -> LDS lds_dst + 16 lane) as
// inline asm, M0 written in the same statement (cdna_hip_programming.md's recipe). Not the builtin:
// hipcc books a global_load_lds as a FLAT access to both memory and LDS, and while one is pending
// it widens EVERY later LDS wait to lgkmcnt(0) and every memory wait to vmcnt(0) — with W2 always
// streaming, the ring's two-steps-ahead LDS reads were waited for one step after issue and each
// phase's first W1 register load waited for the chunk DMA just issued. The asm DMA is invisible
// to that bookkeeping: its completion is counted explicitly (pol_sync's vmcnt(0)).
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds_dst) {
  // the destination is wave-uniform at every call site: pinned to an SGPR (M0's source)
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) void*)lds_dst));
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(l)
               : "memory");
}

// The same DMA with the global address as an SGPR base + a 32-bit VGPR offset (the saddr form):
// the per-piece address arithmetic is scalar (the 64-bit VGPR form spent two v_lshl_add_u64 per
// piece), M0 = the wave-uniform LDS byte address of the piece.
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_addr)
               : "memory");
}

#ifdef MH_FUSED_EXP_STAMPS
// diagnostic build only: lane 0 of policy wave w of workgroup b < 4 stores s_memtime at slot `slot`
// of pass `pass` into the debug-logits buffer (reinterpreted as uint64 [4 wg][4 wave][64 pass][32]).
// (Each stamp is a global store: the next vmcnt(0) — the hand-off's — waits for it, so the
// "sync" segments read long; MH_FUSED_EXP_TACC has no such artefact.)
#define MH_STAMP(a, pass, slot)                                                                      \
  do {                                                                                               \
    if (blockIdx.x < 4 && (threadIdx.x & 63) == 0 && (a).lgt_out) {                                  \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();                                              \
      reinterpret_cast<uint64_t*>((a).lgt_out)[((blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + (pass)) * 32 + (slot)] = t_; \
    }                                                                                                \
  } while (0)
#elif defined(MH_FUSED_EXP_TACC)
// diagnostic build only: s_memtime deltas summed per segment kind in registers (no memory traffic
// inside the horizon), stored once at the end: [wg 4][policy wave 4][8] uint64 in the debug-logits
// buffer. Kinds: 0 prologue, 1 hand-offs, 2 phases 0..6, 3 phase 7 layer 2 + splits, 4 layer 3,
// 5 logits store + pass barrier, 6 between passes.
struct TAcc {
  uint64_t t[8];
  uint64_t last;
};
__device__ __forceinline__ void tacc_add(TAcc& c, int kind) {
  const uint64_t now = __builtin_amdgcn_s_memtime();
  const uint64_t d = now - c.last;
  c.last = now;
  if (kind == 0) c.t[0] += d;
  else if (kind == 1) c.t[1] += d;
  else if (kind == 2) c.t[2] += d;
  else if (kind == 3) c.t[3] += d;
  else if (kind == 4) c.t[4] += d;
  else if (kind == 5) c.t[5] += d;
  else c.t[6] += d;
}
// slot -> the kind of the segment it closes (MH_STAMP's slots)
#define MH_STAMP(a, pass, slot)                                                                      \
  do {                                                                                               \
    const int s_ = (slot);                                                                           \
    tacc_add(g_tacc, s_ == 0 ? 6 : s_ == 1 ? 0 : s_ == 17 ? 3 : s_ == 19 ? 4 : s_ == 18 ? 5 :        \
                         ((s_ & 1) == 0 ? 1 : 2));                                                    \
  } while (0)
#else
#define MH_STAMP(a, pass, slot) \
  do {                          \
  } while (0)
#endif

// the four policy waves' barrier: own LDS-DMA landed (vmcnt(0)), arrive, wait for all four. The
// wait is bounded (~1e9 cycles): a wave that gives up records it in *err (read by the tests
// through mh_sample_horizon_errors) instead of hanging the device. Measured and rejected (DESIGN
// §3.2): a split hand-off (separate "landed" / "buffer read" counters, 641-643 vs 606-617 us per
// horizon), loader waves staging the chunks (637-641 vs 585-595 us), three chunk buffers with the
// DMA two phases ahead (645-656 vs 621-625 us).
__device__ __forceinline__ void pol_sync(uint32_t* bar, uint32_t& target, int64_t* err, uint32_t limit) {
#ifdef MH_FUSED_EXP_NOSYNC  // cost-attribution experiment only (races: garbage logits)
  target += 4;
  return;
#endif
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's share of the chunk landed in LDS
  target += 4;
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  uint32_t spins = 0;
  while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    if (++spins >= limit) {  // (LDS polls without a sleep: the hand-off is within one CU)
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(err, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}

// Splits of two accumulator values into the next layer's (hi, lo) f16 operands (policy_x3.h
// split2h_relu_scaled: no packed-f32 VALU — beside MFMAs a v_pk_mul_f32 / v_pk_fma_f32 costs ~22
// cycles more than the two scalar instructions it replaces, MI355X_MICROARCH.md constants):
//   layer 1: relu(h) * rs     (rs = 2^(ex1 - ex0) / sw1; b1 rides in the MFMA as a constant input)
//   layer 2: relu(acc) * k23  (k23 = 2^(ex2 - ex1) / sw2; acc started at b2 * sw2 * 2^ex1)
// k_policy_forward_x3 uses the same expressions: the same bits.

// The layer-3 pair schedule of the last phase (all compile-time). H2 block fb (pairs 8 fb .. 8 fb +
// 7, pair p = accumulator registers 2p, 2p + 1) is final after step 2 fb + 1 of the last phase; its
// pairs are split from step 2 fb + 2 on (its MFMAs retired: no VALU waits on the matrix pipe),
// at most FOLD_K2 per layer-2 step; the rest during the layer-3 MFMAs, at most FOLD_K3 per
// layer-3 block but always every pair of the block the next layer-3 MFMA reads.
#ifndef MH_FOLD_K2  // (overridable for A/B builds, tools/src_variants.sh)
#define MH_FOLD_K2 2
#endif
#ifndef MH_FOLD_K3
#define MH_FOLD_K3 6
#endif
constexpr int FOLD_K2 = MH_FOLD_K2;
constexpr int FOLD_K3 = MH_FOLD_K3;
constexpr int fold_done_l2(int st) {  // pairs split after layer-2 steps 0 .. st
  int done = 0;
  for (int t = 0; t <= st; ++t) {
    const int ready = t >= 2 ? 8 * ((t - 2) / 2 + 1) : 0;
    const int take = ready - done < FOLD_K2 ? ready - done : FOLD_K2;
    done += take > 0 ? take : 0;
  }
  return done;
}
constexpr int fold_done_l3(int fb) {  // pairs split before layer-3 block fb's MFMAs (fb = -1: after layer 2)
  int done = fold_done_l2(2 * PM_NB - 1);
  for (int b = 0; b <= fb; ++b) {
    int want = done + FOLD_K3;
    if (want < 8 * (b + 1)) want = 8 * (b + 1);
    if (want > 8 * PM_NB) want = 8 * PM_NB;
    done = want;
  }
  return done;
}

// One pass: the 32-env tile `row0 .. row0 + 31` (workgroup-local rows) of policy wave pw through
// all three layers (k_policy_forward_x3<1, 8>'s per-tile MFMA sequence) with the observation rows
// and the logits in LDS. `next`: stage chunk 0 of the following pass during the last phase.
// D = 0: the observation width is Drt.
//   phases 0 .. 6: layer 2's input block ib (chunk ib) into all eight H2 blocks; layer 1 of block
//     ib + 1 pipelined into the phase (issued at step 0, split over steps 3 .. 10);
//   phase 7: chunk 7 into the H2 blocks, each finished block split (bias, ReLU, rescale, f16 hi /
//     lo) two steps later beside the remaining layer-2 MFMAs, then layer 3 as one 16x16x32 MFMA
//     run over the split blocks (policy_x3.h pm_l3_row_half; k_policy_forward_x3's layer-3 order:
//     block 0 .. 7, k-step 0, 1, products lo·hi, hi·lo, hi·hi) with the remaining splits beside it.
// The chunk DMA for the next phase is issued one 1-KB piece per step (steps 0 .. 7) rather than all
// at once: a piece's issue costs a policy wave 60-185 cycles, eight in a row idle the matrix pipe.
#ifdef MH_FUSED_EXP_TACC
#define MH_TACC_PARAM , TAcc& g_tacc
#define MH_TACC_ARG , g_tacc
#else
#define MH_TACC_PARAM
#define MH_TACC_ARG
#endif
// N3 = 2A <= 8 (compile-time: the logits rows are stored without per-row branches); b3r: the
// layer-3 bias of the outputs this lane stores (rows 4 (lane >> 5) + 0..3), held in registers.
template <int D, int N3>
__device__ void policy_pass(const FusedArgs& a, const PolicyLds& L, int pw, int row0, bool next, uint32_t& target,
                            const float (&b3r)[4], int pass_no MH_TACC_PARAM, int Drt = 0) {
  static_assert(N3 >= 1 && N3 <= 8, "the fused sampler's policy head has 2A <= 8 outputs");
  const int DD = D > 0 ? D : Drt;
  MH_STAMP(a, pass_no, 0);
  (void)pass_no;
#ifdef MH_FUSED_EXP_NO_POLICY  // cost-attribution experiment only: no policy work (the barriers stay)
  if (a.H > 0) return;
#endif
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  constexpr int FPW = PM_X3_FRAGS / 4;  // W2 fragments each policy wave stages per chunk
  static_assert(FPW <= 2 * PM_NB, "one DMA piece per step");
  const int lane = threadIdx.x & 63;
  const int K1 = a.K1;
  const float* P = a.P;
  const uint4* W2g = reinterpret_cast<const uint4*>(P + pm_off_w2x3(K1));
  const PmScales scs = pm_scales(P + pm_off_scal(K1));
  const float isw1 = scs.isw[0], isw2 = scs.isw[1], isw3 = scs.isw[2], R1 = scs.R1, R2 = scs.R2;

  // piece i (1 KB) of this wave's share of chunk ib into the chunk buffer at LDS address dst
  const uint32_t voff = (uint32_t)lane * 16u;
  auto stage_piece = [&](int ib, uint32_t dst, int i) {
#ifdef MH_FUSED_EXP_NODMA  // cost-attribution experiment only (stale chunks)
    if (a.H > 0) return;
#endif
    const uint4* src = W2g + ((int64_t)ib * PM_X3_FRAGS + pw * FPW + i) * 64;
    glds16s(src, voff, dst + (uint32_t)(pw * FPW + i) * 1024u);
  };
  auto l1_mfma = [&](const uint4* wf, const f16x8& xh, const f16x8& xl) {
    const f16x8 wh = __builtin_bit_cast(f16x8, wf[0]), wl = __builtin_bit_cast(f16x8, wf[1]);
    f32x16 h = {};
    h = MH_MFMA(wl, xh, h);
    h = MH_MFMA(wh, xl, h);
    h = MH_MFMA(wh, xh, h);
    return h;
  };
  auto pack8 = [](const uint32_t* p) {
    return __builtin_bit_cast(f16x8, uint4{p[0], p[1], p[2], p[3]});
  };

  // observations of env column lane & 31 (inputs k = 8 (lane >> 5) + j; the constant-1 bias input
  // at k = D), scaled by 2^ex[0] and split (load_split_obs of k_policy_forward_x3)
  f16x8 xoh, xol;
  int ex[3];
  {
    const int row = row0 + (lane & 31);
    float x[8];
    float m = 1.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * (lane >> 5) + j;
      x[j] = k < DD ? L.obs[row * DD + k] : (k == DD ? 1.0f : 0.0f);
      m = fmaxf(m, fabsf(x[j]));
    }
    m = fmaxf(m, __shfl_xor(m, 32));
    ex[0] = pm_scale_exp(m);
    const float b1v = R1 * m;
    ex[1] = pm_scale_exp(b1v);
    ex[2] = pm_scale_exp(R2 * fmaxf(1.0f, b1v));
    const float sx = pm_pow2(ex[0]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 hi, lo;
      split2h(x[j] * sx, hi, lo);
      xoh[j] = hi;
      xol[j] = lo;
    }
  }
  const float rs1 = pm_pow2(ex[1] - ex[0]) * isw1;
  f16x8 xh[2], xl[2];
  uint4 w1c[2];
  f32x16 hn;  // layer 1 of the next block, issued ahead of the hand-off that precedes its split
  {
    const uint4 w10[2] = {L.w1[lane], L.w1[64 + lane]};
    w1c[0] = L.w1[(1 * 2 + 0) * 64 + lane];
    w1c[1] = L.w1[(1 * 2 + 1) * 64 + lane];
    const f32x16 h = l1_mfma(w10, xoh, xol);
    hn = l1_mfma(w1c, xoh, xol);  // block 1 (split during phase 0)
    uint32_t hp[8], lp[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) split2h_relu_scaled(h[2 * p], h[2 * p + 1], rs1, hp[p], lp[p]);
    xh[0] = pack8(hp);
    xh[1] = pack8(hp + 4);
    xl[0] = pack8(lp);
    xl[1] = pack8(lp + 4);
  }
  const float k23 = isw2 * pm_pow2(ex[2] - ex[1]);
  const float cb = pm_bias_unit(scs.sw[1], ex[1]);
  f32x16 acc[PM_NB];
  f32x4 b2n[4];  // the next block's layer-2 bias (phase 0: the accumulators start at b2 * cb)
  auto load_b2 = [&](int ob) {
#pragma unroll
    for (int q = 0; q < 4; ++q) b2n[q] = *reinterpret_cast<const f32x4*>(L.b2 + ob * 32 + 8 * q + 4 * (lane >> 5));
  };

  // the three split products of one layer-2 step into H2 block ob (k-step s of the phase's block);
  // `first`: the block's first step (phase 0, s = 0) accumulates onto its bias b2 * cb (registers
  // 4q .. 4q + 3 of block ob hold hidden units ob*32 + 8q + 4 (lane >> 5) + 0..3)
  auto l2_step = [&](int ob, int s, const uint4* cur, bool first) {
    const f16x8 wh = __builtin_bit_cast(f16x8, cur[0]);
    const f16x8 wl = __builtin_bit_cast(f16x8, cur[1]);
    f32x16 acc_ob;
    if (first) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc_ob[r] = b2n[r >> 2][r & 3] * cb;
    } else {
      acc_ob = acc[ob];
    }
    acc_ob = MH_MFMA(wl, xh[s], acc_ob);
    acc_ob = MH_MFMA(wh, xl[s], acc_ob);
    acc_ob = MH_MFMA(wh, xh[s], acc_ob);
    acc[ob] = acc_ob;
  };

  // ---- phases 0 .. PM_NB - 2: input block ib; chunk ib + 1 staged, layer 1 of block ib + 1
  auto phase = [&](auto bufc, auto firstc, int ib) {
    constexpr int B = decltype(bufc)::value;
    constexpr bool FIRST = decltype(firstc)::value;  // phase 0: the accumulators start at zero
    uint4* cur_lds = B ? L.c1 : L.c0;
    const uint32_t nxt_lds = B ? L.c0_lds : L.c1_lds;
    MH_STAMP(a, pass_no, 1 + 2 * ib);
    pol_sync(L.bar, target, L.err, a.spin_limit);  // chunk ib landed in every policy wave's share
    MH_STAMP(a, pass_no, 2 + 2 * ib);
    if constexpr (FIRST) load_b2(0);
    uint32_t l1hp[8], l1lp[8];  // the next block's layer-1 split, pair by pair
    const uint4* Lc = cur_lds + lane;
    uint4 ring[3][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      ring[0][p] = Lc[p * 64];
      ring[1][p] = Lc[(2 + p) * 64];
    }
#pragma unroll
    for (int st = 0; st < 2 * PM_NB; ++st) {
      const int ob = st >> 1, s = st & 1;
      if (st + 2 < 2 * PM_NB) {
#pragma unroll
        for (int p = 0; p < 2; ++p) ring[(st + 2) % 3][p] = Lc[((st + 2) * 2 + p) * 64];
      }
      // the next chunk's DMA into the other buffer (every policy wave finished reading it in the
      // previous phase: the pol_sync above), one piece per step
#ifdef MH_FUSED_EXP_DMA_BURST  // experiment: the whole share at step 0 (the round-4 placement)
      if (st == 0)
        for (int i = 0; i < FPW; ++i) stage_piece(ib + 1, nxt_lds, i);
#else
      if (st < FPW) stage_piece(ib + 1, nxt_lds, st);
#endif
      if (st == 0 && ib + 2 < PM_NB) {
        w1c[0] = L.w1[((ib + 2) * 2 + 0) * 64 + lane];
        w1c[1] = L.w1[((ib + 2) * 2 + 1) * 64 + lane];
      }
      // the next block's layer-1 split, one register pair per step over steps 3..10 (its VALU
      // between this phase's MFMAs)
      if (st >= 3 && st < 11) {
        const int p = st - 3;
        split2h_relu_scaled(hn[2 * p], hn[2 * p + 1], rs1, l1hp[p], l1lp[p]);
      }
      l2_step(ob, s, ring[st % 3], FIRST && s == 0);
      if (FIRST && s == 0 && ob + 1 < PM_NB) load_b2(ob + 1);  // the next block's bias, a step ahead
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    xh[0] = pack8(l1hp);
    xh[1] = pack8(l1hp + 4);
    xl[0] = pack8(l1lp);
    xl[1] = pack8(l1lp + 4);
    // layer 1 of block ib + 2 before the next hand-off: its MFMAs keep the matrix pipe busy while
    // the wave waits there (its split runs in the next phase)
    if (ib + 2 < PM_NB) hn = l1_mfma(w1c, xoh, xol);
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using F0 = std::integral_constant<bool, false>;
  using F1 = std::integral_constant<bool, true>;
  phase(B0{}, F1{}, 0);
  phase(B1{}, F0{}, 1);
#pragma unroll 1
  for (int ib = 2; ib < PM_NB - 2; ib += 2) {
    phase(B0{}, F0{}, ib);
    phase(B1{}, F0{}, ib + 1);
  }
  phase(B0{}, F0{}, PM_NB - 2);

  // ---- phase PM_NB - 1 (chunk 7, buffer 1): the last layer-2 input block, the H2 splits, layer 3
  f32x4 o3 = {};  // layer 3: outputs 4 ((lane >> 4) & 1) + i of env pm_l3_env(lane)
  {
    constexpr int ib = PM_NB - 1;
    (void)ib;
    MH_STAMP(a, pass_no, 1 + 2 * ib);
    pol_sync(L.bar, target, L.err, a.spin_limit);
    MH_STAMP(a, pass_no, 2 + 2 * ib);
    const uint4* Lc = L.c1 + lane;
    uint4 ring[3][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      ring[0][p] = Lc[p * 64];
      ring[1][p] = Lc[(2 + p) * 64];
    }
    uint32_t hs[PM_NB][8], ls[PM_NB][8];  // split H2 blocks: pair p of block fb -> (hs, ls)[fb][p]
    // pair q = 8 fb + p: registers 2p, 2p + 1 of block fb (the bias is already in the accumulator)
    auto split_pair = [&](int q) {
      const int fb = q >> 3, p = q & 7, r = 2 * p;
      split2h_relu_scaled(acc[fb][r], acc[fb][r + 1], k23, hs[fb][p], ls[fb][p]);
    };
    // (pairs split in layer-2 step st: [fold_done_l2(st - 1), fold_done_l2(st)))
#pragma unroll
    for (int st = 0; st < 2 * PM_NB; ++st) {
      const int ob = st >> 1, s = st & 1;
      const int q0 = st == 0 ? 0 : fold_done_l2(st - 1), q1 = fold_done_l2(st);
      if (st + 2 < 2 * PM_NB) {
#pragma unroll
        for (int p = 0; p < 2; ++p) ring[(st + 2) % 3][p] = Lc[((st + 2) * 2 + p) * 64];
      }
      if (next && st < FPW) stage_piece(0, L.c0_lds, st);  // chunk 0 of the next pass
      l2_step(ob, s, ring[st % 3], false);
#pragma unroll
      for (int q = q0; q < q1; ++q) split_pair(q);
      // the split VALU between the step's three MFMAs, not bunched after them
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2 * FOLD_K2, 0);  // VALU (6 per pair)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    MH_STAMP(a, pass_no, 17);
    // layer 3 on 16x16x32 (policy_x3.h pm_l3_row_half; k_policy_forward_x3's order): o3 = W3 H2 over
    // the split blocks; the layer-3 operands read one block ahead, the remaining splits beside the MFMAs
    uint4 w3f[2][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w3f[0][q] = L.w3[q * 64 + lane];
#pragma unroll
    for (int fb = 0; fb < PM_NB; ++fb) {
      const int q0 = fold_done_l3(fb - 1), q1 = fold_done_l3(fb);
      if (fb + 1 < PM_NB) {
#pragma unroll
        for (int q = 0; q < 4; ++q) w3f[(fb + 1) & 1][q] = L.w3[((fb + 1) * 4 + q) * 64 + lane];
      }
#pragma unroll
      for (int q = q0; q < q1; ++q) split_pair(q);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 vh = __builtin_bit_cast(f16x8, w3f[fb & 1][2 * ks]);
        const f16x8 vl = __builtin_bit_cast(f16x8, w3f[fb & 1][2 * ks + 1]);
        const f16x8 hh = pack8(&hs[fb][4 * ks]), hl = pack8(&ls[fb][4 * ks]);
        o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, hh, o3, 0, 0, 0);
        o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, hl, o3, 0, 0, 0);
        o3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, hh, o3, 0, 0, 0);
      }
#pragma unroll
      for (int g = 0; g < 6; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);        // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, FOLD_K3, 0);  // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // logits rows, the same expression as k_policy_forward_x3's store: lane l stores outputs
  // 4 ((l >> 4) & 1) + i of env pm_l3_env(l) — one 16-byte (N3 = 8, 4) or 4-byte (N3 = 2, 6) store
  // per lane — with that env's unit 2^-ex[2] / sw3 from the env's own lane
  MH_STAMP(a, pass_no, 19);
  const int erow = pm_l3_env(lane);
  const float iu = __shfl(isw3 * pm_pow2(-ex[2]), erow);
  const int row = row0 + erow;
  const int o0 = 4 * ((lane >> 4) & 1);
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = o3[r] * iu + b3r[r];
  if constexpr (N3 % 4 == 0) {
    if (o0 < N3) *reinterpret_cast<float4*>(L.lgt + row * N3 + o0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (o0 + r < N3) L.lgt[row * N3 + o0 + r] = v[r];
  }
}

// ------------------------------------------------------------------ env waves
template <class Env>
struct EnvLane {  // one env's persistent state, held in registers across the horizon
  float s[Env::S];
  double xs[Env::XS > 0 ? Env::XS : 1];
  int k, len, pos;
  uint32_t ctr;
};

// One lockstep of one env (lane) — k_rollout<Env, true>'s arithmetic: TanhGauss sample from the
// logits in LDS, clip, env step, term/trunc, rew_plus_cost, autoreset, ring record.
template <class Env>
__device__ __forceinline__ void env_lockstep(const FusedArgs& a, EnvLane<Env>& v, int64_t e, bool live, int t,
                                             const float* lg_row, float* obs_row, float4* stage, int* spos,
                                             bool& emit, int& emit_pos) {
  constexpr int D = Env::D, A = Env::A, RS = Env::RS;
  constexpr int F = rec_floats(D, A);
  const int lane = threadIdx.x & 63;
  float rec[F];  // [0, D) unused: the stage holds obs0
  emit = false;
  emit_pos = 0;
  int wpos = 0;
  constexpr int C = F / 4, CP = C + 1;
  float* srec = reinterpret_cast<float*>(stage + lane * CP);  // this lane's record in the stage
  if (live) {
    float lgt[2 * A];
#pragma unroll
    for (int i = 0; i < 2 * A; ++i) lgt[i] = lg_row[i];
#ifdef MH_FUSED_EXP_STAMPS
    if (false) {
#else
    if (a.lgt_out) {
#endif
#pragma unroll
      for (int i = 0; i < 2 * A; ++i) a.lgt_out[((int64_t)t * a.E + e) * 2 * A + i] = lgt[i];
#pragma unroll
      for (int i = 0; i < D; ++i) a.obs_out[((int64_t)t * a.E + e) * D + i] = obs_row[i];
    }
    // the record's pre-step observation goes to the stage now: not held across the env step
#pragma unroll
    for (int i = 0; i < D; ++i) srec[i] = obs_row[i];
    const float noise = a.act_noise ? a.act_noise[t] : 0.0f;
    double rowv[Env::ROWN > 0 ? Env::ROWN : 1];
    if constexpr (Env::ROWN > 0) {
      typedef double f64x2 __attribute__((ext_vector_type(2)));
      const f64x2* rp = reinterpret_cast<const f64x2*>(a.tab + (int64_t)(v.k + 1) * Env::ROWN);
#pragma unroll
      for (int i = 2; i < Env::ROWN; i += 2) {
        const f64x2 q = rp[i / 2];
        rowv[i] = q[0];
        rowv[i + 1] = q[1];
      }
    }
    const Rng rng = make_rng(a.seed, (uint64_t)e, v.ctr);
    float u[A];
    float logp;
    {
      float nz[4];
      rng.normal4f_fast(0, nz);
      float lg = -0.0f, lt = -0.0f;
#pragma unroll
      for (int i = 0; i < A; ++i) {
        const float mu = lgt[i];
        const float c = fminf(fmaxf(lgt[A + i], a.log_std_lo), a.log_std_hi);
        const float sd = __builtin_amdgcn_exp2f(c * 1.44269504088896341f);
        const float log_sd = c;
        const float z = mu + sd * nz[i];
        const float df = z - mu;
        lg = lg + ((-(df * df) * __builtin_amdgcn_rcpf(2.0f * (sd * sd)) - log_sd) - 0.918938533204672742f);
        const float tt = __builtin_amdgcn_exp2f(-2.88539008177792682f * fabsf(z));
        const float rt = __builtin_amdgcn_rcpf(1.0f + tt);
        const float th = copysignf((1.0f - tt) * rt, z);
        lt = lt + __builtin_amdgcn_logf(squash_arg(tt, rt)) * 0.693147180559945309f;
        const float lo = Env::act_lo(i), hi = Env::act_hi(i);
        const float half = (hi - lo) / 2.0f, mid = (hi + lo) / 2.0f;
        float act = half * th + mid;
        if (a.act_noise) act = act + noise;
        act = fminf(fmaxf(act, lo), hi);
        u[i] = act;
      }
      logp = (lg - lt) - a.log_half_sum;
    }
    if (a.act_out) {
#pragma unroll
      for (int i = 0; i < A; ++i) a.act_out[((int64_t)t * a.E + e) * A + i] = u[i];
    }
    if (a.logp_out) a.logp_out[(int64_t)t * a.E + e] = logp;
    float obs2[D], r;
    if constexpr (Env::ROWN > 0)
      Env::step_row(v.s, v.xs, rowv, u, obs2, &r);
    else
      Env::step(v.s, v.xs, v.k, u, a.tab, obs2, &r);
    bool term = false;
#pragma unroll
    for (int i = 0; i < D; ++i) term = term || (obs2[i] < Env::obs_lo(i)) || (obs2[i] > Env::obs_hi(i));
    int k1 = v.k + 1;
    const bool trunc = k1 >= MAX_STEP;
    const bool done = term || trunc;
    float sq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) sq[i] = obs2[i] * obs2[i];
    const float cost = np_sum<D>(sq) * a.cost_scale;
    const float rew = r * a.reward_scale;
    float obsn[D];
    if (done) {
      float rs[RS];
      ResetDraw<Env>::draw(rng, rs);
      Env::reset_from(rs, v.s, v.xs, a.tab, obsn);
      k1 = 0;
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) obsn[i] = obs2[i];
    }
    v.k = k1;
    v.ctr = v.ctr + 1u;
#pragma unroll
    for (int i = 0; i < D; ++i) obs_row[i] = obsn[i];
#pragma unroll
    for (int i = 0; i < A; ++i) rec[D + i] = u[i];
#pragma unroll
    for (int i = 0; i < D; ++i) rec[D + A + i] = obs2[i];
    rec[2 * D + A + 0] = rew;
    rec[2 * D + A + 1] = cost;
    rec[2 * D + A + 2] = done ? 1.0f : 0.0f;
    rec[2 * D + A + 3] = logp;
#pragma unroll
    for (int i = 2 * D + A + 4; i < F; ++i) rec[i] = 0.0f;
    const int n = a.n, R = a.R;
    wpos = v.pos;
    v.pos = v.pos + 1 == R ? 0 : v.pos + 1;
    v.len = v.len + 1 < n ? v.len + 1 : n;
    emit = (v.len == n);
    emit_pos = v.pos - n < 0 ? v.pos - n + R : v.pos - n;
    if (done) v.len = 0;
  }
  // ring record: transposed through this wave's LDS staging so each store instruction writes
  // whole records (k_rollout's ring store); its first D floats (obs0) are already there
#pragma unroll
  for (int i = D; i < F; ++i) srec[i] = rec[i];
  spos[lane] = wpos;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int64_t e0 = e - lane;
  const int64_t nrec = e0 < a.E ? (a.E - e0 < 64 ? a.E - e0 : 64) : 0;
  const int R = a.R;
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc(a.ring + e0 * R * F, (short)0, (int)(nrec * R * F * 4), 0x00020000);
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  float4 vv[C];
  int off[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int c = j * 64 + lane;
    const int rr_ = c / C, q = c % C;
    vv[j] = stage[rr_ * CP + q];
    off[j] = ((rr_ * R + spos[rr_]) * F + 4 * q) * 4;
  }
#pragma unroll
  for (int j = 0; j < C; ++j) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4v, vv[j]), rr, off[j], 0, 0);
  // the stage is rewritten by the next lockstep of a wave sharing it only after a workgroup
  // barrier; within this wave the reads above complete before its next writes (in order)
}

// ------------------------------------------------------------------ loader waves

// ------------------------------------------------------------------ the kernel
template <class Env>
__global__ __launch_bounds__(FUSED_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_sample_fused(FusedArgs a) {
  constexpr int D = Env::D, A = Env::A, S = Env::S, XS = Env::XS;
  constexpr int N3C = 2 * A;
  constexpr int F = rec_floats(D, A), CP = F / 4 + 1;
  __shared__ uint4 lds0[PM_X3_FRAGS * 64];
  __shared__ uint4 lds1[PM_X3_FRAGS * 64];
  __shared__ uint4 lds_w3[PM_NB * 4 * 64];
  __shared__ float lds_b2[PM_H];
  __shared__ uint4 lds_w1[PM_NB * 2 * 64];
  __shared__ float s_obs[FUSED_ENVS * D];
  __shared__ float s_lgt[FUSED_ENVS * N3C];
  __shared__ float4 s_stage[2][64 * CP];
  __shared__ int s_spos[2][64];
  __shared__ uint32_t s_bar;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t E = a.E;
  const int64_t base = (int64_t)blockIdx.x * FUSED_ENVS;
  const int H = a.H;

  // ---- prologue: the workgroup's observations into LDS (rows past E: zeros), the policy's
  // fold operands and layer-2 bias, chunk 0 of W2
  for (int i = threadIdx.x; i < FUSED_ENVS * D; i += FUSED_THREADS) {
    const int64_t g = base * D + i;
    s_obs[i] = g < E * D ? a.obs[g] : 0.0f;
  }
  if (threadIdx.x == 0) {
    s_bar = 0u;
  }
  const bool pol = w < 4;
  if (pol) {
    const uint4* w3g = reinterpret_cast<const uint4*>(a.P + pm_off_w3x3(a.K1));
    constexpr int FOPW = PM_NB * 4 / 4;
#pragma unroll
    for (int i = 0; i < FOPW; ++i) {
      const int r = w * FOPW + i;
      glds16(w3g + r * 64 + lane, &lds_w3[r * 64]);
    }
    const uint4* w1g = reinterpret_cast<const uint4*>(a.P + pm_off_w1x3(a.K1));
#pragma unroll
    for (int i = 0; i < PM_NB * 2 / 4; ++i) {
      const int r = w * (PM_NB * 2 / 4) + i;
      glds16(w1g + r * 64 + lane, &lds_w1[r * 64]);
    }
    // compact b2 from the packed [ob][lane][16] copy: lanes 0 and 32 of each block hold all 32 rows
    const float* b2p = a.P + pm_off_b2(a.K1);
    for (int q = threadIdx.x; q < PM_NB * 2 * 16; q += 256) {
      const int r = q & 15, l = ((q >> 4) & 1) * 32, ob = q >> 5;
      lds_b2[ob * 32 + pm_row(r, l)] = b2p[((int64_t)ob * 64 + l) * 16 + r];
    }
    const uint4* W2g = reinterpret_cast<const uint4*>(a.P + pm_off_w2x3(a.K1));
    constexpr int FPW = PM_X3_FRAGS / 4;
#pragma unroll
    for (int i = 0; i < FPW; ++i) glds16(W2g + (w * FPW + i) * 64 + lane, &lds0[(w * FPW + i) * 64]);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's fold operands landed before the barrier
  }
  __syncthreads();

  if (pol) {
    // ================= policy waves: 2H passes (H1 first, then H0 / H1 alternating)
    const uint32_t lds0_addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds0;
    const uint32_t lds1_addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds1;
    PolicyLds L{lds0, lds1, lds0_addr, lds1_addr, lds_w3, lds_b2, lds_w1, s_obs, s_lgt, &s_bar, a.err};
    // the layer-3 bias of the rows this lane stores (4 ((lane >> 4) & 1) + r; zero past N3)
    float b3r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 4 * ((lane >> 4) & 1) + r;
      b3r[r] = o < N3C ? a.P[pm_off_b3(a.K1) + o] : 0.0f;
    }
    uint32_t target = 0;
    const int total = 2 * H;
#ifdef MH_FUSED_EXP_TACC
    TAcc g_tacc{};
    g_tacc.last = __builtin_amdgcn_s_memtime();
#endif
    int pass = 0;
    ++pass;
    policy_pass<D, N3C>(a, L, w, FUSED_ENVS / 2 + w * 32, pass < total, target, b3r, pass - 1 MH_TACC_ARG);
    __syncthreads();
    for (int t = 0; t < H; ++t) {
      ++pass;
      policy_pass<D, N3C>(a, L, w, w * 32, pass < total, target, b3r, pass - 1 MH_TACC_ARG);  // A(t): H0
      MH_STAMP(a, pass - 1, 18);
      __syncthreads();
      if (t < H - 1) {  // B(t): H1
        ++pass;
        policy_pass<D, N3C>(a, L, w, FUSED_ENVS / 2 + w * 32, pass < total, target, b3r, pass - 1 MH_TACC_ARG);
        MH_STAMP(a, pass - 1, 18);
      }
      __syncthreads();
    }
#ifdef MH_FUSED_EXP_TACC
    if (blockIdx.x < 4 && lane == 0 && a.lgt_out) {
      uint64_t* o = reinterpret_cast<uint64_t*>(a.lgt_out) + (blockIdx.x * 4 + w) * 8;
#pragma unroll
      for (int k = 0; k < 7; ++k) o[k] = g_tacc.t[k];
      o[7] = (uint64_t)total;
    }
#endif
    __builtin_amdgcn_s_waitcnt(0x0F70);
  } else {
#ifdef MH_FUSED_EXP_NO_ENV  // cost-attribution experiment only
    if (false)
#endif
    {
    // ================= env waves: one env per lane, state in registers across the horizon
    const int ew = w - 4;             // 0, 1: half H0; 2, 3: half H1
    const int half = ew >> 1;
    const int row = ew * 64 + lane;   // workgroup-local env row
    const int64_t e = base + row;
    const bool live = e < E;
    EnvLane<Env> v;
    if (live) {
#pragma unroll
      for (int i = 0; i < S; ++i) v.s[i] = a.state[(int64_t)i * E + e];
#pragma unroll
      for (int i = 0; i < XS; ++i) v.xs[i] = a.xstate[(int64_t)i * E + e];
      v.k = a.steps[e];
      v.ctr = a.ctr[e];
      v.len = a.ring_len[e];
      v.pos = a.ring_pos[e];
    }
    const int NW = (int)((E + 63) / 64);
    const int gw = (int)(e / 64);
    float4* stage = s_stage[ew & 1];
    int* spos = s_spos[ew & 1];
    auto step = [&](int t) {
      bool emit;
      int emit_pos;
      env_lockstep<Env>(a, v, e, live, t, s_lgt + row * N3C, s_obs + row * D, stage, spos, emit, emit_pos);
      const unsigned long long m = __ballot(emit);
      if (base + ew * 64 < E) {
        if (lane == 0) {
          const int nw = __popcll(m);
          a.emit_count[(int64_t)t * NW + gw] = nw;
          if (nw) __hip_atomic_fetch_add(a.ts_total + t, nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (emit) a.emit_list[(int64_t)t * E + (int64_t)gw * 64 + __popcll(m & ((1ull << lane) - 1ull))] =
            lane | (emit_pos << 6);
      }
    };
    __syncthreads();  // the policy's first pass (H1)
    // phases A(t) (half H1 steps) and B(t) (half H0 steps), one call site for the step's body; the
    // other half's waves stage the pass's W2 chunks (phase ph runs policy pass ph + 1)
    for (int ph = 0; ph < 2 * H; ++ph) {
      if ((ph & 1) == (half ^ 1)) {
        step(ph >> 1);
      } else {
      }
      __syncthreads();
    }
    if (live) {
#pragma unroll
      for (int i = 0; i < S; ++i) a.state[(int64_t)i * E + e] = v.s[i];
#pragma unroll
      for (int i = 0; i < XS; ++i) a.xstate[(int64_t)i * E + e] = v.xs[i];
      a.steps[e] = v.k;
      a.ctr[e] = v.ctr;
      a.ring_len[e] = v.len;
      a.ring_pos[e] = v.pos;
    }
    }
  }
  // ---- epilogue: the observations after the horizon (both halves final after the last B phase)
  for (int i = threadIdx.x; i < FUSED_ENVS * D; i += FUSED_THREADS) {
    const int64_t g = base * D + i;
    if (g < E * D) a.obs[g] = s_obs[i];
  }
  // ---- the emission's bookkeeping, by the last workgroup to finish (every lockstep count is in):
  // the per-lockstep window prefixes and the total into aux, with the store cursor they start
  // from; the cursor advanced past the horizon's windows; the counts re-zeroed for the next horizon
  // The lockstep totals are agent-scope atomics (performed at the device's coherence point): each
  // wave's adds complete (vmcnt(0)) before the workgroup's RELAXED arrival, and the last
  // workgroup reads them with agent-scope atomic loads; nothing else passes between workgroups
  // here (aux / cursor are read by the next launch), so no agent-scope fence (an L2 writeback +
  // invalidate per workgroup at the kernel's tail).
  // Memory-model basis (LLVM AMDGPUUsage, "Memory Model GFX942" code sequences, which gfx950
  // follows): the lockstep totals are agent-scope atomic RMWs, performed at the coherence point;
  // `s_waitcnt vmcnt(0)` returns once every one of this workgroup's adds is performed (each
  // storing wave waits before the barrier), and the relaxed arrival is issued after the barrier in
  // program order; the last workgroup reads the totals with agent-scope atomic loads (`sc1`, from
  // the coherence point), so it needs no acquire (MI355X_MICROARCH.md, "Hand-offs measured with sc1
  // loads", row 1). aux / cursor are published to the next launch by the kernel boundary.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  __shared__ uint32_t s_last;
  if (threadIdx.x == 0) {
    const uint32_t arrived = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = arrived == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && w == 0) {
    // wave 0: 64 lockstep totals per round, loaded together, an inclusive wave scan, the
    // exclusive prefixes stored and the totals re-zeroed (a lane-serial loop took one L2 round
    // trip per lockstep at the kernel's tail)
    int64_t carry = 0;
    int last = 0;
    for (int t0 = 0; t0 < H; t0 += 64) {
      const int t = t0 + lane;
      const int v = t < H ? __hip_atomic_load(a.ts_total + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      int64_t incl = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int64_t u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
      }
      if (t < H) {
        a.aux[2 + t] = carry + incl - v;
        __hip_atomic_store(a.ts_total + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int tl = (H - 1 - t0) < 63 ? (H - 1 - t0) : 63;  // this round's last valid lane
      if (t0 + 64 >= H) last = __shfl(v, tl, 64);
      carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) {
      const int64_t run = carry;
      a.aux[0] = run;
      if (a.cursor) {
        const int64_t M = a.capacity, c0 = a.cursor[0], c1 = a.cursor[1];
        a.aux[1] = c0;
        a.cursor[0] = (c0 + run) % M;
        a.cursor[1] = c1 + run < M ? c1 + run : M;
        a.cursor[2] += run;
        a.cursor[3] = last;  // windows of the horizon's last lockstep (the lockstep path's cursor[3])
      }
      __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ horizon emission
// Every window of the horizon, in the reference's order (lockstep major; env index within a
// lockstep: base.py:178-213), into the store rows after the cursor (FIFO wrap; windows older than
// the last `capacity` of this horizon are skipped as overwritten), in ONE launch: k_emit_cells, a
// workgroup per (lockstep, FUSED_EMIT_CW x 64-env block) cell. A cell's first store row is its exclusive window
// prefix: the lockstep's prefix (aux, formed at the end of the fused kernel from per-lockstep
// totals its waves summed with integer atomic adds: order-free) plus the wave counts of the cells
// before it in its lockstep (at most E / 64 counts, reduced by the workgroup). The fused kernel's
// last workgroup also advanced the store cursor. (A separate single-workgroup scan launch over the
// 5,120 cells took 8.6 us per horizon.)
// Within a cell: thread per (window, slot) record, consecutive slots of a window on consecutive
// lanes (consecutive ring records in, consecutive store rows out).

// 64 consecutive store rows [D] (one per lane, lane order) written through an LDS transpose as
// contiguous chunks: 16-byte stores when D % 4 == 0, else 4-byte, one contiguous run per
// instruction instead of D strided stores per lane. `stage` is the wave's 64 * D floats; its next
// writer is the same wave after these reads (a wave's LDS operations are in order).
// The emission's replay-store writes are non-temporal (`global_store … nt`): the store rows are
// read back only by the replay gather, 256 random windows per update, so caching them in L2 / the
// Infinity Cache only evicts what the update that follows reads (the networks, the batch, the
// ring). Bench 1.267-1.275 vs 1.253-1.262 B env-steps/s alternating on one box, the policy-free
// update 0.273-0.288 vs 0.282-0.298 ms (profiles/r06_emit_nt_ab.txt).
typedef float emit_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void emit_st(float* p, float v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void emit_st4(float* p, float4 v) {
  __builtin_nontemporal_store(__builtin_bit_cast(emit_f4, v), reinterpret_cast<emit_f4*>(p));
}

template <int D>
__device__ __forceinline__ void emit_rows_lds(float* dst, const float* row, float* stage, int lane) {
#pragma unroll
  for (int k = 0; k < D; ++k) stage[lane * D + k] = row[k];
  __builtin_amdgcn_wave_barrier();
  if constexpr (D % 4 == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(stage);
    float4* d4 = reinterpret_cast<float4*>(dst);
    float4 v[D / 4];
#pragma unroll
    for (int q = 0; q < D / 4; ++q) v[q] = s4[q * 64 + lane];
#pragma unroll
    for (int q = 0; q < D / 4; ++q) emit_st4(reinterpret_cast<float*>(d4 + q * 64 + lane), v[q]);
  } else {
    float v[D];
#pragma unroll
    for (int q = 0; q < D; ++q) v[q] = stage[q * 64 + lane];
#pragma unroll
    for (int q = 0; q < D; ++q) emit_st(dst + q * 64 + lane, v[q]);
  }
  __builtin_amdgcn_wave_barrier();
}

// Per-cell exclusive window prefixes of each lockstep (one 1024-thread workgroup per lockstep): the
// cells' window counts (four wave counts each), a block scan, the prefixes into cell_pre. Used
// only when a lockstep has more than FUSED_EMIT_SCAN_CELLS cells.
__global__ __launch_bounds__(1024) void k_emit_prefix(HorizonEmitArgs a) {
  constexpr int CW = FUSED_EMIT_CW;
  const int NW = (int)((a.E + 63) / 64);
  const int NBK = (NW + CW - 1) / CW;
  const int ts = blockIdx.x;
  const int32_t* cnt = a.emit_count + (int64_t)ts * NW;
  int32_t* out = a.cell_pre + (int64_t)ts * NBK;
  const int per = (NBK + 1023) / 1024;
  const int c0 = threadIdx.x * per, c1 = c0 + per < NBK ? c0 + per : NBK;
  int sum = 0;
  for (int c = c0; c < c1; ++c)
#pragma unroll
    for (int q = 0; q < CW; ++q) sum += CW * c + q < NW ? cnt[CW * c + q] : 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int u = __shfl_up(incl, off, 64);
    if (lane >= off) incl += u;
  }
  __shared__ int wsum[16];
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int before = 0;
  for (int v = 0; v < wave; ++v) before += wsum[v];
  int run = before + incl - sum;
  for (int c = c0; c < c1; ++c) {
    out[c] = run;
#pragma unroll
    for (int q = 0; q < CW; ++q) run += CW * c + q < NW ? cnt[CW * c + q] : 0;
  }
}

template <int D, int A>
__global__ __launch_bounds__(256) void k_emit_cells(HorizonEmitArgs a) {
  constexpr int F = rec_floats(D, A);
  constexpr int CW = FUSED_EMIT_CW;
  __shared__ float stage[4][64 * D];
  __shared__ int s_pre[4];
  const int NW = (int)((a.E + 63) / 64);
  const int NBK = (NW + CW - 1) / CW;
  const int64_t c = blockIdx.x;
  const int ts = (int)(c / NBK), b = (int)(c - (int64_t)ts * NBK);
  const int32_t* cnt = a.emit_count + (int64_t)ts * NW;
  // the cell's own wave counts, issued with the header and prefix loads (unconditional, clamped)
  int cv[CW];
#pragma unroll
  for (int q = 0; q < CW; ++q) cv[q] = cnt[CW * b + q < NW ? CW * b + q : NW - 1];
  __shared__ int64_t s_hdr[3];
  if (threadIdx.x == 0) {  // one lane reads the shared header (every workgroup reads the same line)
    s_hdr[0] = a.aux[0];
    s_hdr[1] = a.aux[1];
    s_hdr[2] = a.aux[2 + ts];
  }
  if (NBK > FUSED_EMIT_SCAN_CELLS) {  // k_emit_prefix formed the cell's prefix
    if (threadIdx.x < 4) s_pre[threadIdx.x] = threadIdx.x == 0 ? a.cell_pre[(int64_t)ts * NBK + b] : 0;
  } else {  // the wave counts of the lockstep's cells before b (at most CW * FUSED_EMIT_SCAN_CELLS)
    int part = 0;
    for (int i = threadIdx.x; i < CW * b; i += 256) part += cnt[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off, 64);
    if ((threadIdx.x & 63) == 0) s_pre[threadIdx.x >> 6] = part;
  }
  __syncthreads();
  const int64_t total = s_hdr[0], base = s_hdr[1], M = a.capacity;
  const int64_t g0 = s_hdr[2] + (int64_t)(s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3]);
  const int64_t start = total > M ? total - M : 0;  // older windows are overwritten this horizon
  int pre[CW + 1];
  pre[0] = 0;
#pragma unroll
  for (int q = 0; q < CW; ++q) pre[q + 1] = pre[q] + (CW * b + q < NW ? cv[q] : 0);
  const int nwin = pre[CW];
  const int n = a.n, R = a.R;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // wave-strided chunks of 64 records (every lane of a wave takes part in each chunk, so the
  // chunk's rows can be stored as one block when they are 64 consecutive store rows)
  for (int i0 = wave * 64; i0 < nwin * n; i0 += 256) {
    const int i = i0 + lane;
    bool valid = i < nwin * n;
    float rec[F];
    int64_t o = 0;
    if (valid) {
      const int w = i / n, j = i - w * n;
      const int64_t g = g0 + w;
      valid = g >= start;
      if (valid) {
        int q = 0, pq = 0;  // the wave holding window w and its first window (selects: no indexed registers)
#pragma unroll
        for (int k = 1; k < CW; ++k) {
          const bool past = w >= pre[k];
          q += past;
          pq = past ? pre[k] : pq;
        }
        const int gw = CW * b + q;
        const int packed = a.emit_list[(int64_t)ts * a.E + (int64_t)gw * 64 + (w - pq)];
        const int64_t e = (int64_t)gw * 64 + (packed & 63);
        int slot = (packed >> 6) + j;
        slot = slot >= R ? slot - R : slot;
        const float4* src = reinterpret_cast<const float4*>(a.ring + (e * R + slot) * (int64_t)F);
#pragma unroll
        for (int k = 0; k < F / 4; ++k) {
          const float4 v = src[k];
          rec[4 * k] = v.x;
          rec[4 * k + 1] = v.y;
          rec[4 * k + 2] = v.z;
          rec[4 * k + 3] = v.w;
        }
        o = ((base + g) % M) * n + j;
      }
    }
    // consecutive records are consecutive store rows except across the FIFO wrap and at the
    // chunk tail: the block store when all 64 are, the per-record stores otherwise
    const int64_t o0 = __shfl(o, 0, 64);
    const bool block = __ballot(valid && o == o0 + lane) == ~0ull;
    if (block) {
      emit_rows_lds<D>(a.obs + o0 * D, rec, stage[wave], lane);
      emit_rows_lds<D>(a.obs2 + o0 * D, rec + D + A, stage[wave], lane);
    } else if (valid) {
#pragma unroll
      for (int k = 0; k < D; ++k) emit_st(a.obs + o * D + k, rec[k]);
#pragma unroll
      for (int k = 0; k < D; ++k) emit_st(a.obs2 + o * D + k, rec[D + A + k]);
    }
    if (valid) {
      if constexpr (A == 4) {  // one 16-byte row per lane: consecutive lanes, consecutive rows
        emit_st4(a.act + o * A, make_float4(rec[D], rec[D + 1], rec[D + 2], rec[D + 3]));
      } else {
#pragma unroll
        for (int k = 0; k < A; ++k) emit_st(a.act + o * A + k, rec[D + k]);
      }
      emit_st(a.rew + o, rec[2 * D + A]);
      emit_st(a.cost + o, rec[2 * D + A + 1]);
      emit_st(a.done + o, rec[2 * D + A + 2]);
      emit_st(a.logp + o, rec[2 * D + A + 3]);
    }
  }
}

// ------------------------------------------------------------------ launchers
// the emission launch alone (the last horizon's windows again: it reads the ring, the per-wave
// lists and the fused kernel's header and writes the same store rows, so it is idempotent until
// the next horizon; bench.py times it this way at the trainer's own window count)
template <class Env>
static hipError_t launch_emit_t(const HorizonEmitArgs& ea, hipStream_t st) {
  if (fused_emit_cells_per_lockstep(ea.E) > FUSED_EMIT_SCAN_CELLS) {
    if (ea.cell_pre == nullptr) return hipErrorInvalidValue;
    k_emit_prefix<<<ea.H, 1024, 0, st>>>(ea);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  k_emit_cells<Env::D, Env::A><<<(unsigned)fused_emit_cells(ea.E, ea.H), 256, 0, st>>>(ea);
  return hipGetLastError();
}

template <class Env>
static hipError_t launch_fused_t(const FusedArgs& a, const HorizonEmitArgs& ea, hipStream_t st) {
  const int grid = (int)((a.E + FUSED_ENVS - 1) / FUSED_ENVS);
  k_sample_fused<Env><<<grid, FUSED_THREADS, 0, st>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ea.obs == nullptr) return e;
  return launch_emit_t<Env>(ea, st);
}

hipError_t launch_emit_horizon(int env_id, const HorizonEmitArgs& ea, hipStream_t st) {
  if (ea.obs == nullptr || ea.aux == nullptr) return hipErrorInvalidValue;
  switch (env_id) {
    case ENV_VANDERPOL: return launch_emit_t<VanderPol>(ea, st);
    case ENV_PENDULUM: return launch_emit_t<Pendulum>(ea, st);
    case ENV_DUCTEDFAN: return launch_emit_t<DuctedFan>(ea, st);
    case ENV_TWOLINK: return launch_emit_t<TwoLink>(ea, st);
    case ENV_SINGLETRACKCAR: return launch_emit_t<SingleTrackCar>(ea, st);
    case ENV_QUADTRACKING: return launch_emit_t<QuadTracking>(ea, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_sample_fused(int env_id, const FusedArgs& a, const HorizonEmitArgs& ea, hipStream_t st) {
  switch (env_id) {
    case ENV_VANDERPOL: return launch_fused_t<VanderPol>(a, ea, st);
    case ENV_PENDULUM: return launch_fused_t<Pendulum>(a, ea, st);
    case ENV_DUCTEDFAN: return launch_fused_t<DuctedFan>(a, ea, st);
    case ENV_TWOLINK: return launch_fused_t<TwoLink>(a, ea, st);
    case ENV_SINGLETRACKCAR: return launch_fused_t<SingleTrackCar>(a, ea, st);
    case ENV_QUADTRACKING: return launch_fused_t<QuadTracking>(a, ea, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace mh
