// rollout.h — argument blocks and launchers shared by rollout.hip and capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "env_math.h"
#include "philox.h"

namespace mh {

constexpr int BLK = 256;  // envs per step-kernel block (4 wavefronts)

// floats of one n-step ring record: obs[D] act[A] obs2[D] rew cost done logp, padded to 16 B
__host__ __device__ constexpr int rec_floats(int D, int A) { return ((2 * D + A + 4) + 3) / 4 * 4; }
// byte offset of the xstate part of a state trace (StepArgs::trace_state)
__host__ __device__ constexpr int64_t trace_xoff(int S, int64_t E) { return (S * E * 4 + 15) / 16 * 16; }

struct StepArgs {
  int64_t E;
  float* state;      // [S][E]
  double* xstate;    // [XS][E]
  int32_t* steps;    // [E]
  const double* tab; // QuadTracking desired-trajectory table (device) or null
  int64_t* meta;     // device int64[8]: emit base row, last emitted total, cursor snapshots
  uint32_t* ctr;     // [E] per-env Philox counter (lockstep steps + resets drawn so far)
  uint64_t seed;
  // io (AoS)
  float* obs;                 // [E][D] in: pre-step obs (ring), out: next obs
  const float* logits;        // [E][2A]
  const float* act_in;        // [E][A]
  const float* logp_in;       // [E]
  const float* reset_in;      // [E][RS]
  float* act_out;
  float* logp_out;
  float* real_next_obs;
  float* reward_out;
  uint8_t* term_out;
  uint8_t* trunc_out;
  // n-step ring
  float* ring;                // [E][n][F]
  int32_t* ring_len;
  int32_t* ring_pos;
  int32_t* emit_rank;         // [E]
  int32_t* block_count;       // [grid]
  int32_t* emit_list;         // [grid*BLK] block-compacted emitter env ids (rank order)
  const int64_t* cursor;      // store cursor, snapshotted into meta[1], meta[3], meta[4]
  int n;
  int ring_slots;             // R >= n ring slots per env (n unless mh_nstep_reserve grew it)
  float reward_scale, cost_scale;
  int raw_log_std;               // logits second half is log_std: std = exp(clamp(., lo, hi))
  float log_std_lo, log_std_hi;  // StochaPolicy min/max_log_std (mlp.py:125-136)
  float log_half_sum;            // sum_i log((high_i - low_i) / 2) of the action box (float32)
  const float* act_noise;        // device scalar added to every sampled action before the clip
                                 // (GaussNoise.sample, explore_noise.py:9; base.py:136-137) or null
  // on-policy trajectory store (OnSampler mb_* arrays, on_sampler.py:22-41): [E][H][.] rows,
  // this step writes column traj_t (null traj_obs: not recording)
  float *traj_obs, *traj_act, *traj_rew, *traj_cost, *traj_obs2, *traj_logp;
  uint8_t* traj_done;
  int traj_H, traj_t;
  // deferred emission (mh_rollout_step_deferred): each block has EMIT_WAVES extra waves that
  // copy the PREVIOUS step's full windows (prev_count / prev_list: its block counts and emitter
  // lists) into the window store while the env waves step; this step's counts / lists go to
  // block_count / emit_list (the other half of the double buffer)
  int defer;                  // 1: deferred mode (blockDim = BLK + 64 * EMIT_WAVES)
  int parity;                 // meta[META_ACC0 + parity] receives the windows emitted so far
  const int32_t* prev_count;  // null: nothing pending (first step of a horizon)
  const int32_t* prev_list;
  float *w_obs, *w_act, *w_rew, *w_cost, *w_obs2, *w_done, *w_logp;  // window store arrays
  int64_t capacity;
  // step trace of the post-step state of the envs that reset, BEFORE the autoreset overwrites it
  // (parity tests only; null: not traced): SoA [S][E] floats, then (from byte trace_xoff(S, E)) [XS][E] doubles —
  // one pointer, so the kernel's argument SGPRs do not grow
  void* trace_state;
};

constexpr int EMIT_WAVES = 4;  // emitter waves per block in deferred mode

// meta[] slots (device int64[8]); META_ACC0/1: windows emitted by the deferred steps of the
// current horizon before the pending step (double-buffered by step parity)
constexpr int META_BASE = 1, META_TOTAL = 2, META_SIZE = 3, META_GTOTAL = 4, META_ACC0 = 5;

struct EmitArgs {
  int64_t E;
  const float* ring;
  const int32_t* ring_pos;
  const int32_t* emit_rank;
  const int32_t* block_offset;
  const int64_t* meta;
  int64_t capacity;
  int n, F, D, A;
  int R;                      // ring slots per env (>= n)
  float *obs, *act, *rew, *cost, *obs2, *done, *logp;
  // fused scan + persistent emission (k_emit_fused)
  const int32_t* block_count;
  const int32_t* emit_list;
  int32_t nb;                 // step-kernel blocks
  int64_t* meta_rw;           // last emitted total, written by block 0
  int64_t* cursor;            // store cursor written by block 0
};

constexpr int EMIT_FUSED_MAX_NB = 4096;  // block prefix kept in LDS (16 KB) up to 1M envs

hipError_t launch_emit_fused(int env_id, const EmitArgs& a, hipStream_t st);

struct GatherArgs {
  const int64_t* idx;
  int64_t batch;
  int n, D, A;
  const float *s_obs, *s_act, *s_rew, *s_cost, *s_obs2, *s_done, *s_logp;
  float *o_obs, *o_act, *o_rew, *o_cost, *o_obs2, *o_done, *o_logp;
  // joint layouts the update consumes (null: not written): o_obs_act [batch][n][D + A] = [obs | act]
  // rows (the critics' input), o_v_in [batch + batch n][D] = obs(b, 0) rows then the obs2 rows (the
  // Lyapunov network's batch of the stability advantage)
  float *o_obs_act, *o_v_in;
  // in-kernel draw (draw != null: idx is ignored): idx[b] = the (seed, b, draw[0]) index into the
  // store's [0, cursor[1]) windows, written to idx_out (nullable); the last workgroup to finish
  // advances draw[0] (draw[1] is its arrival ticket, 0 between launches)
  const int64_t* cursor = nullptr;
  uint64_t seed = 0;
  int64_t* draw = nullptr;
  int64_t* idx_out = nullptr;
};

// The gather's flat grid (launch_gather): every output layout is a segment of `units` vectors of
// vw floats, cut into GATHER_CHUNK-vector chunks, one per workgroup from wg0 on. Vector q of a
// segment belongs to batch row q / rowlen; kind GATHER_PLAIN copies src[window * src_row + i],
// GATHER_OBS_ACT interleaves the window's obs and act rows (aux0/1/2 = (D + A)/vw, D/vw, A/vw;
// src_row = n store rows per window).
#ifndef MH_GATHER_K
#define MH_GATHER_K 4
#endif
constexpr int GATHER_K = MH_GATHER_K;  // vectors per thread
constexpr int GATHER_CHUNK = 256 * GATHER_K;
constexpr int GATHER_MAX_SEGS = 10;
enum { GATHER_PLAIN = 0, GATHER_OBS_ACT = 1 };
struct GatherSeg {
  const float* src;
  const float* src2;
  float* dst;
  uint32_t units, rowlen, src_row, vw, kind, aux0, aux1, aux2, wg0;
};
struct GatherPlan {
  GatherSeg seg[GATHER_MAX_SEGS];
  int nseg;
};

hipError_t launch_rollout(int env_id, const StepArgs& a, hipStream_t st);
hipError_t launch_gae(const float* val, const float* val2, const float* rew, const uint8_t* done, int64_t E,
                      int H, double gamma, double lam, float* adv, float* ret, hipStream_t st);
hipError_t launch_reset(int env_id, const StepArgs& a, hipStream_t st);
hipError_t launch_rng_draw(int env_id, int kind, uint64_t seed, const int64_t* env_idx, const uint32_t* ctr,
                           int64_t n, float* out, hipStream_t st);
int64_t policy_packed_floats(int D);
int act_grad_chunks(int64_t M);
hipError_t launch_gemm(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                       int64_t lda, int64_t ldb, int64_t ldc, int ta, int tb, int act, float* workspace,
                       hipStream_t st);
int64_t gemm_workspace_floats(int64_t M, int64_t N, int64_t K);
bool linear_backward_plan(int64_t rows, int64_t n_out, int64_t n_in, bool dx, bool dw, bool db, int64_t* ws);
hipError_t launch_linear_backward(const float* dy, const float* y, int act, const float* x, const float* W,
                                  int64_t rows, int64_t n_out, int64_t n_in, float* dx, float* dw, float* db,
                                  float* workspace, hipStream_t st);
hipError_t launch_stocha_head(const float* raw, int64_t M, int A, float lo, float hi, float* out, hipStream_t st);
hipError_t launch_stocha_head_bwd(const float* raw, const float* out, const float* dout, int64_t M, int A, float lo,
                                  float hi, float* draw, hipStream_t st);
hipError_t launch_tg_rsample(const float* logits, const float* eps, const float* high, const float* low, int64_t M,
                             int A, float* act, float* logp, hipStream_t st);
hipError_t launch_tg_rsample_bwd(const float* logits, const float* eps, const float* high, const float* low,
                                 const float* d_act, const float* d_logp, int64_t M, int A, float* d_logits,
                                 hipStream_t st);
hipError_t launch_tg_log_prob(const float* logits, const float* a, const float* high, const float* low, int64_t M,
                              int A, float* logp, hipStream_t st);
hipError_t launch_tg_log_prob_bwd(const float* logits, const float* a, const float* high, const float* low,
                                  const float* d_logp, int64_t M, int A, float* d_logits, hipStream_t st);
hipError_t launch_act_grad_colsum(const float* dy, const float* y, int64_t M, int N, int act, float* g, float* db,
                                  float* partial, uint32_t* tickets, hipStream_t st);
int act_grad_tickets(int N);
hipError_t launch_policy_head(const float* raw, const float* eps, const float* obs, const float* old_act,
                              const float* high, const float* low, int64_t M, int A, int D, float lo, float hi,
                              float* xq, float* new_logp, float* old_logp, hipStream_t st, uint64_t seed = 0,
                              unsigned long long* ctr = nullptr, float* eps_out = nullptr);
hipError_t launch_policy_head_bwd(const float* raw, const float* eps, const float* old_act, const float* high,
                                  const float* low, const float* d_xq, const float* d_new_logp,
                                  const float* d_old_logp, int64_t M, int A, int D, float lo, float hi, float* d_raw,
                                  hipStream_t st);
int64_t head_backward_workspace(int64_t M, int n_out, int n_in);
hipError_t launch_square_sum(const float* y, int64_t rows, int cols, float* out, hipStream_t st);
hipError_t launch_dx_narrow(const float* dy, const float* y, int act, const float* W, int64_t M, int n_out,
                            int n_in, float* dx, hipStream_t st);
hipError_t launch_square_sum_bwd(const float* y, const float* g, int64_t rows, int cols, float* dy, hipStream_t st);
hipError_t launch_head_backward(const float* dy, const float* x, const float* W, int64_t M, int n_out, int n_in,
                                float* dx, float* dw, float* db, float* workspace, hipStream_t st);
// dw = sum over blocks of pdw[b] (and db of pdb[b]) in block order, per group q at q x the strides
hipError_t launch_head_finish(const float* pdw, const float* pdb, int64_t nblk, int n_out, int n_in, int groups,
                              int64_t s_part, float* dw, int64_t s_dw, float* db, int64_t s_db, hipStream_t st);
hipError_t launch_head_backward_grouped(const float* dy, const float* x, const float* W, int64_t M, int n_out,
                                        int n_in, int64_t ldx, int64_t lddx, int groups, int64_t s_dy, int64_t s_x,
                                        int64_t s_W, int64_t s_dx, int64_t s_dw, int64_t s_db, float* dx, float* dw,
                                        float* db, float* workspace, hipStream_t st);
hipError_t launch_gemm_grouped(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N,
                               int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int ta, int tb, int act, int groups,
                               int64_t sA, int64_t sB, int64_t sBias, int64_t sC, hipStream_t st);
hipError_t launch_linear_backward_grouped(const float* dy, const float* y, int act, const float* x, const float* W,
                                          int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x,
                                          int64_t ld_dx, int groups, int64_t s_dy, int64_t s_x, int64_t s_W,
                                          int64_t s_dx, int64_t s_dw, int64_t s_db, float* dx, float* dw, float* db,
                                          float* workspace, hipStream_t st);
constexpr int ADAM_MAX_TENSORS = 32;
struct AdamList {  // one optimiser's tensors, passed by value in the kernel arguments
  float* p[ADAM_MAX_TENSORS];
  const float* g[ADAM_MAX_TENSORS];
  float* m[ADAM_MAX_TENSORS];
  float* v[ADAM_MAX_TENSORS];
  float* step[ADAM_MAX_TENSORS];
  int64_t start[ADAM_MAX_TENSORS + 1];  // prefix sums of the work units (4-element vectors or elements)
  double lr[ADAM_MAX_TENSORS];           // each tensor's learning rate (one launch may step several optimisers)
  int64_t numel[ADAM_MAX_TENSORS];
  int vec[ADAM_MAX_TENSORS];             // 1: the tensor is stepped as float4 units (aligned, numel % 4 == 0)
  int n;
};
struct PolyakList {
  float* t[ADAM_MAX_TENSORS];
  const float* s[ADAM_MAX_TENSORS];
  int64_t start[ADAM_MAX_TENSORS + 1];  // prefix sums of the work units, as in AdamList
  int64_t numel[ADAM_MAX_TENSORS];
  int vec[ADAM_MAX_TENSORS];
  int n;
};
// the fused 3-layer MLP forward (mlp_fused.hip)
struct Mlp3Args {
  const float* x;
  int64_t M, ldx;
  int K1, H, N3;
  int act1, act2, act3;  // 0 identity, 1 ReLU, 2 tanh
  const float *W1, *b1, *W2, *b2, *W3, *b3;
  float *h1, *h2, *y;    // h1 / h2 may be null (not kept)
  int64_t ldh, ldy;
  int64_t gs_x, gs_W1, gs_b1, gs_W2, gs_b2, gs_W3, gs_b3, gs_h, gs_y;
  // a second network set of the same shapes and group strides in the same launch (groups
  // [groups_a, groups_a + groups_b) of the grid: the twin target critics beside the twin critics),
  // its activations never kept; groups_b = 0: none
  const float *x_b, *W1_b, *b1_b, *W2_b, *b2_b, *W3_b, *b3_b;
  float* y_b;
  int groups_a, groups_b;
  // LyapunovValue's sum over the outputs of y^2 per row (N3 a multiple of 64), the square-sum
  // kernel's order; null: not formed
  float* sqsum;
};
// the fused 3-layer MLP input-gradient chain (mlp_fused.hip): g2 = (dy W3) * act2'(h2),
// g1 = (g2 W2) * act1'(h1), dx = sum over groups of g1 W1 (dy is the gradient of the identity-
// activated output)
struct Mlp3BwdArgs {
  const float* dy;
  int64_t ldy, gs_dy;
  const float *h1, *h2;
  int64_t ldh, gs_h;
  const float *W1, *W2, *W3;
  int64_t gs_W1, gs_W2, gs_W3;
  int64_t M;
  int K1, H, N3, act1, act2, groups;
  float *g2, *g1;  // optional
  int64_t ldg, gs_g;
  float* dx;       // optional [M][ldx]
  int64_t ldx;
  // LyapunovValue: dy = dv[row] (2 y) formed from the forward output y (ldy) and dv = dV instead
  // of read (square-sum backward's expression), written to g3 ([M][ldy]) for the weight gradient
  const float* sq_dv;
  float* g3;
  // N3 <= 16 (optional): the output layer's weight / bias gradient partials of every 16-row block
  // b, pdw3[b][N3][H] = sum over its rows (in order) of dy[r][o] h2[r][j] and pdb3[b][N3] = the
  // rows' dy sums, group q's at q s_part3 (k_head_backward's partials, bit for bit below 16,384
  // rows; summed by launch_head_finish)
  float *pdw3, *pdb3;
  int64_t s_part3;
};
hipError_t launch_mlp3_backward(const Mlp3BwdArgs& a, hipStream_t st);
void mlp3_set_row_tiles(int mode);
// several weight gradients dw = g^T x, db = column sums of g in two launches (gemm.hip)
struct WgradSpec {
  const float* g;
  int64_t ld_g;
  const float* x;
  int64_t ld_x;
  int64_t n_out, n_in;
  float* dw;
  float* db;
};
bool weight_grads_plan(const WgradSpec* ps, int n, int64_t rows, int64_t* ws_floats);
hipError_t launch_weight_grads(const WgradSpec* ps, int n, int64_t rows, float* ws, hipStream_t st);
bool mlp3_supported(int64_t M, int K1, int H, int N3);
hipError_t launch_mlp3_forward(const Mlp3Args& a, int groups, hipStream_t st);
hipError_t launch_polyak_multi(const PolyakList& L, double polyak, hipStream_t st);
hipError_t launch_adam_multi(const AdamList& L, double b1, double b2, double eps, uint32_t* ticket,
                             hipStream_t st);
hipError_t launch_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                              const float* b3, int D, int N3, float* P, hipStream_t st);
hipError_t launch_policy_forward(const float* P, const float* obs, int64_t E, int D, int N3, float* logits,
                                 hipStream_t st);
hipError_t launch_finalize(const int32_t* block_count, int32_t nb, int32_t* block_offset, int64_t* meta,
                           int64_t* cursor, int64_t capacity, hipStream_t st);
hipError_t launch_emit(const EmitArgs& a, hipStream_t st);
hipError_t launch_gather(const GatherArgs& a, hipStream_t st);
hipError_t launch_sample_idx(const int64_t* cursor, uint64_t seed, uint64_t counter, int64_t batch,
                             int64_t* idx, hipStream_t st);
hipError_t launch_sample_idx_dev(const int64_t* cursor, uint64_t seed, int64_t* draw, int64_t batch, int64_t* idx,
                                 hipStream_t st);
hipError_t launch_transpose_f32(const float* src, float* dst, int W, int64_t E, bool to_aos, hipStream_t st);
hipError_t launch_transpose_f64(const double* src, double* dst, int W, int64_t E, bool to_aos, hipStream_t st);

}  // namespace mh
