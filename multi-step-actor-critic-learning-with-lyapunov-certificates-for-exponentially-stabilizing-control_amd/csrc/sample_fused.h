// sample_fused.h — argument blocks of the fused horizon sampler (sample_fused.hip), shared with
// the C ABI (capi.hip: mh_sample_horizon).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mh {

struct FusedArgs {
  int64_t E;
  float* state;       // [S][E]
  double* xstate;     // [XS][E]
  int32_t* steps;     // [E]
  const double* tab;  // QuadTracking desired-trajectory table or null
  uint32_t* ctr;      // [E] per-env Philox counter
  uint64_t seed;
  float* obs;         // [E][D] in: current observation, out: the observation after the horizon
  const float* P;     // packed policy parameters (k_policy_pack_x3 layout)
  int K1, N3, H;
  float* ring;        // [E][R][F]
  int32_t* ring_len;
  int32_t* ring_pos;
  int n, R;
  float reward_scale, cost_scale;
  float log_std_lo, log_std_hi, log_half_sum;
  const float* act_noise;  // [H] GaussNoise scalars (one per lockstep) or null
  int32_t* emit_count;     // [H][NW] windows completed per (lockstep, 64-env wave)
  int32_t* emit_list;      // [H][E] per wave, rank-ordered (lane | oldest slot << 6)
  int32_t* ts_total;       // [H] windows completed per lockstep (atomic adds; zero on entry: the last
                           // workgroup to finish turns them into aux's prefixes and re-zeroes them)
  uint32_t* arrive;        // workgroup arrival count (0 between horizons)
  int64_t* aux;            // out: {total windows, store cursor before the horizon, prefix[0 .. H)}
  int64_t* cursor;         // the window store's {ptr, size, total, last} (advanced by the last
                           // workgroup), or null: no store
  int64_t capacity;
  float* act_out;          // [H][E][A] or null
  float* logp_out;         // [H][E] or null
  int64_t* err;            // device error word: policy-wave waits that timed out (0 when healthy)
  float* lgt_out;          // [H][E][2A] the logits each env sampled from, or null (diagnostics)
  float* obs_out;          // [H][E][D] the observation each env stepped from, or null (diagnostics)
  uint32_t spin_limit;     // polls of a policy-wave wait before it gives up and counts an error
};

// default bound of a policy-wave wait (~1e9 cycles; a healthy hand-off takes < 1e3)
constexpr uint32_t FUSED_SPIN_LIMIT = 1u << 26;

constexpr int FUSED_ENVS = 256;   // envs per workgroup (one workgroup per CU)
constexpr int FUSED_THREADS = 512;
// (lockstep, FUSED_EMIT_CW x 64-env block) cells of the horizon emission (one workgroup each)
// 16 waves (1,024 envs) per cell: 5 -> 1.25 k workgroups per 65,536-env horizon, one round of
// them on the chip; k_emit_cells alone 21.6 vs 24.3 us for 23,040 windows against 4 waves per cell
// (profiles/r05_emit_cell_width_ab.txt)
#ifndef MH_EMIT_CW
#define MH_EMIT_CW 16
#endif
constexpr int FUSED_EMIT_CW = MH_EMIT_CW;  // 64-env waves per emission cell
inline int64_t fused_emit_cells_per_lockstep(int64_t E) { return ((E + 63) / 64 + FUSED_EMIT_CW - 1) / FUSED_EMIT_CW; }
inline int64_t fused_emit_cells(int64_t E, int H) { return (int64_t)H * fused_emit_cells_per_lockstep(E); }
// Above this many 64-env waves per lockstep (E > 262,144) a cell no longer sums the wave counts
// of every earlier cell of its lockstep itself (O(cells^2) loads per lockstep): k_emit_prefix forms
// the per-cell prefixes first (one workgroup per lockstep), into HorizonEmitArgs::cell_pre.
constexpr int64_t FUSED_EMIT_SCAN_CELLS = 4096 / FUSED_EMIT_CW;

struct HorizonEmitArgs {
  int64_t E;
  int H, n, R;
  const float* ring;
  const int32_t* emit_count;  // [H][NW]
  const int32_t* emit_list;   // [H][E]
  float *obs, *act, *rew, *cost, *obs2, *done, *logp;
  int64_t capacity;
  const int64_t* aux;  // FusedArgs::aux
  int32_t* cell_pre;   // [H][cells] per-cell exclusive window prefixes within the lockstep (written by
                       // k_emit_prefix when cells > FUSED_EMIT_SCAN_CELLS, else unused; may be null then)
};


hipError_t launch_sample_fused(int env_id, const FusedArgs& a, const HorizonEmitArgs& ea, hipStream_t st);
hipError_t launch_emit_horizon(int env_id, const HorizonEmitArgs& ea, hipStream_t st);

}  // namespace mh
