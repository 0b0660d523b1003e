// rollout.hip — lockstep rollout kernels for the six MSACL envs on gfx950.
//
// One thread owns one env for a whole lockstep step: persistent state is float32 SoA
// ([dim][E], coalesced across the wavefront), caller-facing tensors are row-major AoS
// ([E][dim], what torch/numpy hold). The fused step kernel does, per env:
//   TanhGauss sample (or injected action) -> clip -> K Euler substeps -> reward ->
//   termination/truncation -> rew_plus_cost -> autoreset -> n-step deque push,
// and writes the block-local rank of every env whose deque became full. A single-block
// finalize kernel scans the per-block counts (env-index-order emission, base.py:178) and
// advances the store cursor; the emit kernel then copies each full deque into its window row,
// staging the env's ring record block through LDS so both sides are wide/coalesced.
#include <initializer_list>

#include "rollout.h"
#include "reset_draw.h"

namespace mh {

// reset distributions: reset_draw.h (shared with the host engine, host_engine.hip)

// --------------------------------------------------------------- SoA buffer access
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
// raw buffer resource over [p, p + bytes) (gfx9 dword3: 32-bit data format, no swizzle)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t soa_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Zero-sized resource for an absent optional input: buffer loads from it return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t opt_rsrc(const void* p, int64_t bytes) {
  return soa_rsrc(p, p ? (uint32_t)bytes : 0u);
}

// One env's row of a row-major [E][N] float tensor (byte offset off) as the widest aligned
// buffer loads (row offsets are multiples of N floats: 16-byte loads when N % 4 == 0, 8-byte
// loads when N is even; launch_rollout_t checks the base alignment).
template <int N>
__device__ __forceinline__ void load_row_buf(__amdgpu_buffer_rsrc_t r, int off, float* out) {
  // The whole load result is bit-cast to a float vector before any element is read: with this
  // toolchain (ROCm 7.2 clang, -O3) element extracts from an integer-vector b64/b128 buffer load
  // are miscompiled (the load shrinks to one dword and every element reads element 0).
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 16 * i, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) out[4 * i + j] = v[j];
    }
  } else if constexpr (N % 2 == 0) {
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const f32x2 v = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 8 * i, 0));
      out[2 * i] = v[0];
      out[2 * i + 1] = v[1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 4 * i, 0));
  }
}

template <int W>
__device__ __forceinline__ void store_vec(float* dst, const float* v);

// The wave's 64 rows [e0, e0 + 64) of a row-major [E][D] float tensor, each lane holding its own
// row: written through an LDS transpose as consecutive chunks (16-byte when D % 4 == 0, else
// 4-byte, one contiguous 256-byte run per instruction), not as D strided 4-byte stores per lane
// (for SingleTrackCar's D = 7 each of those touched 28 lines per instruction: 264 -> 229 us per
// 4 M-env step, DuctedFan 113 -> 101 us). Rows >= E fall
// outside the resource and are dropped. `so` is the wave's stage (>= 16 D float4); the next
// writer of the stage is the same wave, after these reads (LDS operations of a wave are in order).
template <int D>
__device__ __forceinline__ void wave_store_rows(float* dst, const float* row, int64_t e0, int64_t E, float4* so,
                                                int lane) {
  const int64_t nrow = e0 < E ? (E - e0 < 64 ? E - e0 : 64) : 0;
  const __amdgpu_buffer_rsrc_t ro = soa_rsrc(dst + e0 * D, (uint32_t)(nrow * D * 4));
  static_assert(D >= 4, "rows of <= 12 bytes are stored directly by their lanes");
  if constexpr (D % 4 == 0) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < D / 4; ++i) so[lane * (D / 4) + i] = make_float4(row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]);
    __builtin_amdgcn_wave_barrier();
    float4 v[D / 4];
#pragma unroll
    for (int j = 0; j < D / 4; ++j) v[j] = so[j * 64 + lane];
#pragma unroll
    for (int j = 0; j < D / 4; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v[j]), ro, (j * 64 + lane) * 16, 0, 0);
  } else {
    float* sf = reinterpret_cast<float*>(so);
#pragma unroll
    for (int i = 0; i < D; ++i) sf[lane * D + i] = row[i];
    __builtin_amdgcn_wave_barrier();
    float v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = sf[j * 64 + lane];
#pragma unroll
    for (int j = 0; j < D; ++j)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[j]), ro, (j * 64 + lane) * 4, 0, 0);
  }
  __builtin_amdgcn_wave_barrier();
}

// Deferred emission (emitter waves w = 0..EMIT_WAVES-1 of a block in mh_rollout_step_deferred):
// the previous step's full windows of THIS block's envs, in env-index order, into the window
// store rows after every earlier block's and every earlier deferred step's windows (the same
// rows and values as k_emit_fused would have written right after that step:
// RL/trainer/sampler/base.py:178-217, nstep_replay_buffer.py:122-125). The ring slots read
// here are overwritten by this launch's env waves only after the block barrier that follows.
template <int D, int A>
__device__ void deferred_emit(const StepArgs& a, int w, int lane) {
  constexpr int F = rec_floats(D, A);
  const int nb = gridDim.x, blk = blockIdx.x, n = a.n, R = a.ring_slots;
  int pre = 0, tot = 0;  // windows of the blocks before this one / of all blocks
  if (a.prev_count) {
    for (int i = lane; i < nb; i += 64) {
      const int c = a.prev_count[i];
      tot += c;
      pre += i < blk ? c : 0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      pre += __shfl_xor(pre, off, 64);
      tot += __shfl_xor(tot, off, 64);
    }
  }
  const int64_t M = a.capacity;
  const int64_t acc = a.prev_count ? a.meta[META_ACC0 + (a.parity ^ 1)] : 0;
  const int64_t c0 = a.cursor[0];
  if (a.prev_count) {
    const int mine = a.prev_count[blk];
    const int64_t base = (c0 + acc + pre) % M;  // store row of this block's first window
    for (int q = w * 64 + lane; q < mine * n; q += EMIT_WAVES * 64) {
      const int r = q / n, j = q - r * n;
      const int packed = a.prev_list[(int64_t)blk * BLK + r];
      const int64_t env = (int64_t)blk * BLK + (packed & (BLK - 1));
      int slot = (packed >> 8) + j;
      slot = slot >= R ? slot - R : slot;
      float rec[F];
      const float4* src = reinterpret_cast<const float4*>(a.ring + (env * R + slot) * (int64_t)F);
#pragma unroll
      for (int i = 0; i < F / 4; ++i) {
        const float4 v = src[i];
        rec[4 * i] = v.x;
        rec[4 * i + 1] = v.y;
        rec[4 * i + 2] = v.z;
        rec[4 * i + 3] = v.w;
      }
      int64_t row = base + r;
      if (row >= M) row %= M;
      const int64_t o = row * n + j;
      store_vec<D>(a.w_obs + o * D, rec);
      store_vec<A>(a.w_act + o * A, rec + D);
      store_vec<D>(a.w_obs2 + o * D, rec + D + A);
      a.w_rew[o] = rec[2 * D + A];
      a.w_cost[o] = rec[2 * D + A + 1];
      a.w_done[o] = rec[2 * D + A + 2];
      a.w_logp[o] = rec[2 * D + A + 3];
    }
  }
  if (blk == 0 && w == 0 && lane == 0) {
    // windows emitted by this horizon's deferred steps so far, and the cursor snapshot the
    // flush (k_emit_fused) starts from when this launch's own windows are the last pending ones
    const int64_t acc1 = acc + tot;
    a.meta[META_ACC0 + a.parity] = acc1;
    a.meta[META_BASE] = (c0 + acc1) % M;
    a.meta[META_SIZE] = a.cursor[1] + acc1;
    a.meta[META_GTOTAL] = a.cursor[2] + acc1;
  }
}

// --------------------------------------------------------------- fused lockstep step
// Occupancy floor per env (the launch bound's waves per SIMD, i.e. a VGPR budget of 512 / waves):
// 2 (<= 256 VGPRs) by default; the env-step bound kernels of the mid-weight envs run better with
// more waves resident to hide their dependent f32/f64 chains (MH_*_WAVES: A/B switches)
#ifndef MH_ROLLOUT_MIN_WAVES
#define MH_ROLLOUT_MIN_WAVES 2
#endif
#ifndef MH_CAR_WAVES
#define MH_CAR_WAVES MH_ROLLOUT_MIN_WAVES
#endif
#ifndef MH_TWOLINK_WAVES
#define MH_TWOLINK_WAVES MH_ROLLOUT_MIN_WAVES
#endif
template <class Env> struct RolloutWaves { static constexpr int v = MH_ROLLOUT_MIN_WAVES; };
template <> struct RolloutWaves<SingleTrackCar> { static constexpr int v = MH_CAR_WAVES; };
template <> struct RolloutWaves<TwoLink> { static constexpr int v = MH_TWOLINK_WAVES; };

// SAMPLE: actions drawn from the policy logits (the sampler); false: injected actions (a.act_in,
// the env.step / parity path), whose instantiation carries no sampling code at all.
template <class Env, bool SAMPLE>
__global__ __launch_bounds__(BLK + 64 * EMIT_WAVES, RolloutWaves<Env>::v) void k_rollout(StepArgs a) {
  constexpr int D = Env::D, A = Env::A, S = Env::S, XS = Env::XS, RS = Env::RS;
  constexpr int F = rec_floats(D, A);
  const int64_t E = a.E;
  const bool env_thread = threadIdx.x < BLK;  // waves 0-3; waves 4.. are emitter waves (deferred mode)
  const int64_t e = (int64_t)blockIdx.x * BLK + threadIdx.x;
  const bool live = env_thread && e < E;
  bool emit = false;
  int emit_pos = 0;  // ring slot of the window's oldest record (the position after this push)
  float rec[F];      // this step's ring record (stored transposed through LDS, below)
  float oout[D];     // next observation row (stored transposed through LDS, below)
  float nout[D];     // real next observation row (the same)
  // per-wave LDS stage: the observation rows' transposes, then the ring records'
  constexpr int RC = F / 4, RCP = RC + 1;  // ring record float4 chunks; padded LDS record stride
  __shared__ float4 wstage[BLK / 64][64 * RCP > 16 * D ? 64 * RCP : 16 * D];
  int wpos = 0;      // the ring slot it goes to
  // store-cursor snapshot for the emission kernel, loaded up front by one thread (the grid
  // finishes with its slowest wave: three dependent round trips at the end would be exposed)
  const bool snap = a.ring && a.cursor && !a.defer && blockIdx.x == 0 && threadIdx.x == 0;
  int64_t cur0 = 0, cur1 = 0, cur2 = 0;
  if (snap) {
    cur0 = a.cursor[0];
    cur1 = a.cursor[1];
    cur2 = a.cursor[2];
  }
  if (live) {
    // ---- every per-env input is issued up front, in dependency order: the step counter first
    // (the QuadTracking desired-trajectory row is addressed by it), then the sampler's inputs
    // (logits, Philox counter, exploration noise), the ring cursor, the pre-step observation and
    // the state. The sampling then starts while the state is still in flight, and no load waits
    // behind a store it cannot be proven disjoint from (one round trip per action component and
    // one for the ring cursor after the stores, before).
    // Every load is a raw buffer load, unconditional: an absent optional input is a zero-sized
    // resource (reads return 0), so there is no branch around a load and the compiler's vmcnt
    // bookkeeping stays exact (a join after an optional load made it wait for everything).
    const int vo4 = (int)(e * 4), vo8 = (int)(e * 8);
    const __amdgpu_buffer_rsrc_t rs_i32 = soa_rsrc(a.steps, (uint32_t)(E * 4));
    const int k = (int)__builtin_amdgcn_raw_buffer_load_b32(rs_i32, vo4, 0, 0);
    asm volatile("" ::: "memory");  // issue order pinned (compiler-only barriers: no instruction, no wait)
    const uint32_t ctr = __builtin_amdgcn_raw_buffer_load_b32(opt_rsrc(a.ctr, E * 4), vo4, 0, 0);
    float lgt[2 * A], inj[A];
    float logp_inj = 0.0f, noise = 0.0f;
    if constexpr (SAMPLE) {
      load_row_buf<2 * A>(opt_rsrc(a.logits, E * 2 * A * 4), (int)(e * 2 * A * 4), lgt);
      noise = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(opt_rsrc(a.act_noise, 4), 0, 0, 0));
    } else {
      load_row_buf<A>(opt_rsrc(a.act_in, E * A * 4), (int)(e * A * 4), inj);
      logp_inj = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(opt_rsrc(a.logp_in, E * 4), vo4, 0, 0));
    }
    float obs0[D];
    load_row_buf<D>(opt_rsrc((a.ring || a.traj_obs) ? a.obs : nullptr, E * D * 4), (int)(e * D * 4), obs0);
    float s[S];
    double xs[XS > 0 ? XS : 1];
    // SoA state through buffer resources: one VGPR byte offset per env plus a scalar offset per
    // component, instead of a 64-bit address pair per component held live from load to store
    // (mh_env_create bounds E so every byte offset fits in 31 bits)
    const __amdgpu_buffer_rsrc_t rs_state = soa_rsrc(a.state, (uint32_t)(S * E * 4));
    const __amdgpu_buffer_rsrc_t rs_xstate = soa_rsrc(a.xstate, (uint32_t)(XS * E * 8));
#pragma unroll
    for (int i = 0; i < S; ++i)
      s[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_state, vo4, (int)(i * E * 4), 0));
#pragma unroll
    for (int i = 0; i < XS; ++i)
      xs[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs_xstate, vo8, (int)(i * E * 8), 0));
    int len = (int)__builtin_amdgcn_raw_buffer_load_b32(opt_rsrc(a.ring_len, E * 4), vo4, 0, 0);
    int pos = (int)__builtin_amdgcn_raw_buffer_load_b32(opt_rsrc(a.ring_pos, E * 4), vo4, 0, 0);
    asm volatile("" ::: "memory");  // the table row, which waits for k, is issued after all of the above
    double rowv[Env::ROWN > 0 ? Env::ROWN : 1];
    if constexpr (Env::ROWN > 0) {  // Env::load_row as buffer loads (table rows 0..MAX_STEP)
      typedef double f64x2 __attribute__((ext_vector_type(2)));  // whole-vector cast: see load_row_buf
      const __amdgpu_buffer_rsrc_t rt = soa_rsrc(a.tab, (uint32_t)((MAX_STEP + 1) * Env::ROWN * 8));
      const int ro = (k + 1) * Env::ROWN * 8;
      static_assert(Env::ROWN % 2 == 0, "rows are read as 16-byte pairs from column 2");
#pragma unroll
      for (int i = 2; i < Env::ROWN; i += 2) {
        const f64x2 v = __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(rt, ro, 8 * i, 0));
        rowv[i] = v[0];
        rowv[i + 1] = v[1];
      }
    }
    // compiler-only barrier (no instruction, no wait): the loads above stay issued here instead
    // of being sunk, split per component, into the branches that consume them (the sampling
    // branch read one logit per round trip)
    asm volatile("" ::: "memory");
    const Rng rng = make_rng(a.seed, (uint64_t)e, ctr);

    // ---- action: TanhGaussDistribution.sample() + clip, or the injected action (selected
    // after the sampling, which runs either way: no branch merges pending loads into u)
    float u[A];
    float logp = 0.0f;
    if constexpr (SAMPLE) {
      float nz[4];
      rng.normal4f_fast(0, nz);
      // TanhGaussDistribution.sample (act_distribution_cls.py:45-57): z = mu + std * eps,
      // logp = Normal(mu, std).log_prob(z) - sum log(1 + 1e-6 - tanh(z)^2) - sum log((h-l)/2),
      // on the hardware transcendentals (v_exp/v_log/v_rcp_f32, ~1 ulp); the middle term through
      // squash_arg (philox.h: no float32 cancellation near |tanh z| = 1).
      float lg = -0.0f, lt = -0.0f;
#pragma unroll
      for (int i = 0; i < A; ++i) {
        const float mu = lgt[i];
        const float raw = lgt[A + i];
        float sd, log_sd;
        if (a.raw_log_std) {  // std = clamp(log_std, lo, hi).exp(): log(std) is the clamped value
          const float c = fminf(fmaxf(raw, a.log_std_lo), a.log_std_hi);
          sd = __builtin_amdgcn_exp2f(c * 1.44269504088896341f);
          log_sd = c;
        } else {
          sd = raw;
          log_sd = __builtin_amdgcn_logf(sd) * 0.693147180559945309f;
        }
        const float z = mu + sd * nz[i];
        const float df = z - mu;  // not sd * eps: keeps the reference's rounding for tiny std
        lg = lg + ((-(df * df) * __builtin_amdgcn_rcpf(2.0f * (sd * sd)) - log_sd) - 0.918938533204672742f);
        // tanh(z) = sign(z) (1 - t) / (1 + t), t = exp(-2|z|)
        const float t = __builtin_amdgcn_exp2f(-2.88539008177792682f * fabsf(z));
        const float rt = __builtin_amdgcn_rcpf(1.0f + t);
        const float th = copysignf((1.0f - t) * rt, z);
        lt = lt + __builtin_amdgcn_logf(squash_arg(t, rt)) * 0.693147180559945309f;
        const float lo = Env::act_lo(i), hi = Env::act_hi(i);
        const float half = (hi - lo) / 2.0f, mid = (hi + lo) / 2.0f;
        float act = half * th + mid;
        if (a.act_noise) act = act + noise;  // GaussNoise: one scalar per lockstep step
        act = fminf(fmaxf(act, lo), hi);  // actions.clip(low, high)
        u[i] = act;
      }
      const float ls = a.log_half_sum;
      logp = (lg - lt) - ls;
    }
    if constexpr (!SAMPLE) {  // injected action (and its log-prob when given)
#pragma unroll
      for (int i = 0; i < A; ++i) u[i] = inj[i];
      logp = a.logp_in ? logp_inj : 0.0f;
    }
    if (a.act_out) {
#pragma unroll
      for (int i = 0; i < A; ++i) a.act_out[e * A + i] = u[i];
    }
    if (a.logp_out) a.logp_out[e] = logp;

    // ---- env.step
    float obs2[D], r;
    if constexpr (Env::ROWN > 0)
      Env::step_row(s, xs, rowv, u, obs2, &r);
    else
      Env::step(s, xs, k, u, a.tab, obs2, &r);
    bool term = false;
#pragma unroll
    for (int i = 0; i < D; ++i) term = term || (obs2[i] < Env::obs_lo(i)) || (obs2[i] > Env::obs_hi(i));
    int k1 = k + 1;
    const bool trunc = k1 >= MAX_STEP;
    const bool done = term || trunc;
    // ---- rew_plus_cost (rew_plus_cost.py:18-21)
    float sq[D];
#pragma unroll
    for (int i = 0; i < D; ++i) sq[i] = obs2[i] * obs2[i];
    const float cost = np_sum<D>(sq) * a.cost_scale;
    const float rew = r * a.reward_scale;
    // ---- autoreset (gymnasium 0.28.1 SyncVectorEnv.step)
    float obsn[D];
    if (done) {
      if (a.trace_state) {  // parity trace: the post-step state the reset overwrites (uniform test)
        const __amdgpu_buffer_rsrc_t rt_s = soa_rsrc(a.trace_state, (uint32_t)(trace_xoff(S, E) + XS * E * 8));
        const int xo = (int)trace_xoff(S, E);
#pragma unroll
        for (int i = 0; i < S; ++i)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[i]), rt_s, vo4, (int)(i * E * 4), 0);
#pragma unroll
        for (int i = 0; i < XS; ++i)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, xs[i]), rt_s, vo8, xo + (int)(i * E * 8), 0);
      }
      float rs[RS];
      if (a.reset_in) {
#pragma unroll
        for (int i = 0; i < RS; ++i) rs[i] = a.reset_in[e * RS + i];
      } else {
        ResetDraw<Env>::draw(rng, rs);
      }
      Env::reset_from(rs, s, xs, a.tab, obsn);
      k1 = 0;
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) obsn[i] = obs2[i];
    }
#pragma unroll
    for (int i = 0; i < S; ++i)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[i]), rs_state, vo4, (int)(i * E * 4), 0);
#pragma unroll
    for (int i = 0; i < XS; ++i)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, xs[i]), rs_xstate, vo8, (int)(i * E * 8), 0);
    a.steps[e] = k1;
    a.ctr[e] = ctr + 1u;
    if constexpr (D >= 4) {
#pragma unroll
      for (int i = 0; i < D; ++i) {  // stored below, transposed through LDS with the wave's rows
        oout[i] = obsn[i];
        nout[i] = obs2[i];
      }
    } else {  // rows of <= 12 bytes: stored directly (the transpose measured slower there)
      if (a.obs) {
#pragma unroll
        for (int i = 0; i < D; ++i) a.obs[e * D + i] = obsn[i];
      }
      if (a.real_next_obs) {
#pragma unroll
        for (int i = 0; i < D; ++i) a.real_next_obs[e * D + i] = obs2[i];
      }
    }
    if (a.reward_out) a.reward_out[e] = r;
    if (a.term_out) a.term_out[e] = term ? 1 : 0;
    if (a.trunc_out) a.trunc_out[e] = trunc ? 1 : 0;

    // ---- on-policy trajectory column (on_sampler.py:131-141: mb_obs/act/rew/cost/obs2/done/logp)
    if (a.traj_obs) {
      const int64_t c = e * (int64_t)a.traj_H + a.traj_t;
#pragma unroll
      for (int i = 0; i < D; ++i) a.traj_obs[c * D + i] = obs0[i];
#pragma unroll
      for (int i = 0; i < A; ++i) a.traj_act[c * A + i] = u[i];
#pragma unroll
      for (int i = 0; i < D; ++i) a.traj_obs2[c * D + i] = obs2[i];
      a.traj_rew[c] = rew;
      a.traj_cost[c] = cost;
      a.traj_done[c] = done ? 1 : 0;
      a.traj_logp[c] = logp;
    }

    // ---- n-step deque push (base.py:180-217): the record is built here and stored below,
    // transposed through LDS with the rest of the wave's records
    if (a.ring) {
#pragma unroll
      for (int i = 0; i < D; ++i) rec[i] = obs0[i];
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
      const int n = a.n, R = a.ring_slots;
      wpos = pos;
      pos = pos + 1 == R ? 0 : pos + 1;
      len = len + 1 < n ? len + 1 : n;
      emit = (len == n);
      emit_pos = pos - n < 0 ? pos - n + R : pos - n;  // the window's oldest slot (pos when R == n)
      if (done) len = 0;  // deque.clear() when the newest item is done
      a.ring_len[e] = len;
      a.ring_pos[e] = pos;
    }
  }
  if constexpr (D >= 4) {
    if (env_thread && (a.obs || a.real_next_obs)) {
      // next observations and real next observations, [E][D] rows: the wave's 64 rows are one
      // contiguous 64 * D * 4-byte range each
      const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const int64_t e0 = (int64_t)blockIdx.x * BLK + wave * 64;
      if (a.real_next_obs) wave_store_rows<D>(a.real_next_obs, nout, e0, E, wstage[wave], lane);
      if (a.obs) wave_store_rows<D>(a.obs, oout, e0, E, wstage[wave], lane);
    }
  }
  if (a.ring) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // Ring records (F floats, one 128-byte line for QuadTracking) are written as the wave's
    // records transposed through LDS: in each store instruction 8 consecutive lanes write one
    // record's contiguous chunks, so an instruction touches 64 / (F / 4) records' lines instead
    // of 64 (one record per lane took 3.4 us of the 17.4 us QuadTracking step at E = 65,536:
    // a compiled-out variant, round 1). Staged here, stored after the block barrier.
    constexpr int C = RC, CP = RCP;
    __shared__ int spos[BLK / 64][64];
    if (env_thread) {
      float4* sw = wstage[wave];
#pragma unroll
      for (int i = 0; i < C; ++i) sw[lane * CP + i] = make_float4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
      spos[wave][lane] = wpos;
    } else {
      // emitter waves: the previous step's windows, while the env waves above compute
      deferred_emit<D, A>(a, wave - BLK / 64, lane);
    }
    // block-local exclusive rank of emitters (wave ballot + LDS), env-index order
    __shared__ int wcnt[BLK / 64];
    const unsigned long long m = __ballot(emit);
    if (lane == 0 && env_thread) wcnt[wave] = __popcll(m);
    // the barrier also orders the emitter waves' ring reads before the ring stores below, which
    // overwrite each emitted window's oldest slot
    __syncthreads();
    if (env_thread) {
      int base = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < BLK / 64; ++w) {
        base += (w < wave) ? wcnt[w] : 0;
        tot += wcnt[w];
      }
      const int rank = emit ? base + __popcll(m & ((1ull << lane) - 1ull)) : -1;
      if (a.emit_list) {
        // (block-local env index | oldest ring slot << 8): the emission needs no ring_pos load
        static_assert(BLK == 256, "emit_list packs the block-local env index into 8 bits");  // n <= 4096
        if (emit) a.emit_list[(int64_t)blockIdx.x * BLK + rank] = (int32_t)(e - (int64_t)blockIdx.x * BLK) | (emit_pos << 8);
      } else if (live) {
        a.emit_rank[e] = rank;
      }
      if (threadIdx.x == 0) a.block_count[blockIdx.x] = tot;
      if (snap) {
        // snapshot of the store cursor for the emission kernel (which rewrites the cursor)
        a.meta[META_BASE] = cur0;
        a.meta[META_SIZE] = cur1;
        a.meta[META_GTOTAL] = cur2;
      }
      const float4* sw = wstage[wave];
      const int64_t e0 = (int64_t)blockIdx.x * BLK + wave * 64;
      const int R = a.ring_slots;
      // the wave's slice of the ring as a buffer resource: records of envs >= E fall outside it
      // and are dropped by the hardware, so the loop has no branch and its LDS reads batch up
      const int64_t nrec = e0 < E ? (E - e0 < 64 ? E - e0 : 64) : 0;
      const __amdgpu_buffer_rsrc_t rr = soa_rsrc(a.ring + e0 * R * F, (uint32_t)(nrec * R * F * 4));
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      float4 v[C];
      int off[C];
#pragma unroll
      for (int j = 0; j < C; ++j) {  // every LDS read first (one wait), then the stores
        const int c = j * 64 + lane;
        const int r = c / C, q = c % C;
        v[j] = sw[r * CP + q];
        off[j] = ((r * R + spos[wave][r]) * F + 4 * q) * 4;
      }
#pragma unroll
      for (int j = 0; j < C; ++j) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v[j]), rr, off[j], 0, 0);
    }
  }
}

// --------------------------------------------------------------- reset kernel
template <class Env>
__device__ __forceinline__ void reset_one(const StepArgs& a, int64_t e) {
  constexpr int D = Env::D, S = Env::S, XS = Env::XS, RS = Env::RS;
  const int64_t E = a.E;
  float rs[RS], s[S], o[D];
  double xs[XS > 0 ? XS : 1];
  if (a.reset_in) {
#pragma unroll
    for (int i = 0; i < RS; ++i) rs[i] = a.reset_in[e * RS + i];
  } else {
    const uint32_t ctr = a.ctr[e];
    ResetDraw<Env>::draw(make_rng(a.seed, (uint64_t)e, ctr), rs);
    a.ctr[e] = ctr + 1u;
  }
  Env::reset_from(rs, s, xs, a.tab, o);
#pragma unroll
  for (int i = 0; i < S; ++i) a.state[(int64_t)i * E + e] = s[i];
#pragma unroll
  for (int i = 0; i < XS; ++i) a.xstate[(int64_t)i * E + e] = xs[i];
  a.steps[e] = 0;
  if (a.obs) {
#pragma unroll
    for (int i = 0; i < D; ++i) a.obs[e * D + i] = o[i];
  }
  if (a.ring) {
    a.ring_len[e] = 0;
    a.ring_pos[e] = 0;
  }
}

template <class Env>
__global__ __launch_bounds__(BLK) void k_reset(StepArgs a) {
  const int64_t e = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (e < a.E) reset_one<Env>(a, e);
}

// --------------------------------------------------------------- the kernels' Philox draws
// (mh_rng_draw): for unit i the key (seed, env_idx[i], ctr[i]) the rollout / fused kernels use for
// that env at that counter, and the SAME inline draws they make with it: kind 0 the four action
// normals (normal4f_fast, stream 0), kind 1 the env's reset draw (ResetDraw<Env>, streams 1..4).
template <class Env>
__global__ __launch_bounds__(BLK) void k_rng_draw(int kind, uint64_t seed, const int64_t* env_idx,
                                                  const uint32_t* ctr, int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (i >= n) return;
  const Rng r = make_rng(seed, (uint64_t)env_idx[i], ctr[i]);
  if (kind == 0) {
    float nz[4];
    r.normal4f_fast(0, nz);
#pragma unroll
    for (int j = 0; j < 4; ++j) out[i * 4 + j] = nz[j];
  } else {
    float rs[Env::RS];
    ResetDraw<Env>::draw(r, rs);
#pragma unroll
    for (int j = 0; j < Env::RS; ++j) out[i * Env::RS + j] = rs[j];
  }
}

template <class Env>
static hipError_t launch_rng_draw_t(int kind, uint64_t seed, const int64_t* env_idx, const uint32_t* ctr, int64_t n,
                                    float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  k_rng_draw<Env><<<(unsigned)((n + BLK - 1) / BLK), BLK, 0, st>>>(kind, seed, env_idx, ctr, n, out);
  return hipGetLastError();
}

hipError_t launch_rng_draw(int env_id, int kind, uint64_t seed, const int64_t* env_idx, const uint32_t* ctr,
                           int64_t n, float* out, hipStream_t st) {
  switch (env_id) {
    case ENV_VANDERPOL: return launch_rng_draw_t<VanderPol>(kind, seed, env_idx, ctr, n, out, st);
    case ENV_PENDULUM: return launch_rng_draw_t<Pendulum>(kind, seed, env_idx, ctr, n, out, st);
    case ENV_DUCTEDFAN: return launch_rng_draw_t<DuctedFan>(kind, seed, env_idx, ctr, n, out, st);
    case ENV_TWOLINK: return launch_rng_draw_t<TwoLink>(kind, seed, env_idx, ctr, n, out, st);
    case ENV_SINGLETRACKCAR: return launch_rng_draw_t<SingleTrackCar>(kind, seed, env_idx, ctr, n, out, st);
    case ENV_QUADTRACKING: return launch_rng_draw_t<QuadTracking>(kind, seed, env_idx, ctr, n, out, st);
  }
  return hipErrorInvalidValue;
}

// --------------------------------------------------------------- finalize (scan + cursor)
__global__ __launch_bounds__(1024) void k_finalize(const int32_t* block_count, int32_t nb,
                                                   int32_t* block_offset, int64_t* meta,
                                                   int64_t* cursor, int64_t capacity) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (nb + 1023) / 1024;
  const int lo = min(nb, t * per), hi = min(nb, lo + per);
  int64_t local = 0;
  for (int i = lo; i < hi; ++i) local += block_count[i];
  part[t] = local;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t > 0 ? part[t - 1] : 0;
  for (int i = lo; i < hi; ++i) {
    block_offset[i] = (int32_t)run;
    run += block_count[i];
  }
  if (t == 0) {
    const int64_t total = part[1023];
    meta[2] = total;
    if (cursor) {
      const int64_t base = cursor[0];
      meta[1] = base;
      int64_t keep = total < capacity ? total : capacity;
      (void)keep;
      cursor[0] = (base + total) % capacity;
      const int64_t sz = cursor[1] + total;
      cursor[1] = sz < capacity ? sz : capacity;
      cursor[2] += total;
      cursor[3] = total;
    }
  }
}

// --------------------------------------------------------------- window emission
__global__ __launch_bounds__(256) void k_emit(EmitArgs a) {
  extern __shared__ float lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t e = (int64_t)blockIdx.x * 4 + wave;
  if (e >= a.E) return;
  const int rank = a.emit_rank[e];
  if (rank < 0) return;
  const int64_t g = (int64_t)a.block_offset[e / BLK] + rank;
  const int64_t total = a.meta[2];
  const int64_t M = a.capacity;
  if (g < total - M) return;  // overwritten later in this same step (FIFO order)
  const int64_t row = (a.meta[1] + g) % M;
  const int n = a.n, F = a.F, D = a.D, A = a.A, R = a.R;
  float* buf = lds + wave * R * F;
  const float4* src = reinterpret_cast<const float4*>(a.ring + e * (int64_t)R * F);
  float4* b4 = reinterpret_cast<float4*>(buf);
  for (int i = lane; i < (R * F) / 4; i += 64) b4[i] = src[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int pos = a.ring_pos[e] - n < 0 ? a.ring_pos[e] - n + R : a.ring_pos[e] - n;  // oldest record
  struct Field {
    float* dst;
    int off, width;
  };
  const Field fields[7] = {{a.obs, 0, D},          {a.act, D, A},          {a.obs2, D + A, D},
                           {a.rew, 2 * D + A, 1},  {a.cost, 2 * D + A + 1, 1},
                           {a.done, 2 * D + A + 2, 1}, {a.logp, 2 * D + A + 3, 1}};
#pragma unroll
  for (int f = 0; f < 7; ++f) {
    const int W = fields[f].width, off = fields[f].off;
    float* dst = fields[f].dst + row * (int64_t)n * W;
    for (int idx = lane; idx < n * W; idx += 64) {
      const int j = idx / W, d = idx - j * W;
      int slot = pos + j;
      slot = slot >= R ? slot - R : slot;
      dst[idx] = buf[slot * F + off + d];
    }
  }
}

// Fused scan + emission, one thread per (window, slot) record. Every workgroup re-derives the
// env-order window offsets from the step kernel's per-block emitter counts (nb <= 4096 ints in
// LDS, wave-shuffle scan), so no separate scan launch is needed; workgroup 0 advances the store
// cursor. Thread q handles window g = q / n, slot j = q % n: it locates the emitting env with a
// binary search over the block offsets, reads ring record (pos + j) mod n of that env (F floats,
// 16-B loads; the n threads of a window read one contiguous ring block) and scatters the record's
// fields to row (base + g) mod M of the seven store arrays, where consecutive slots are adjacent
// (vector stores of D / A floats). All threads are independent: no per-window serial chain.
template <int W>
__device__ __forceinline__ void store_vec(float* dst, const float* v) {
  if constexpr (W % 4 == 0) {
#pragma unroll
    for (int i = 0; i < W; i += 4) *reinterpret_cast<float4*>(dst + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
  } else if constexpr (W % 2 == 0) {
#pragma unroll
    for (int i = 0; i < W; i += 2) *reinterpret_cast<float2*>(dst + i) = make_float2(v[i], v[i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < W; ++i) dst[i] = v[i];
  }
}

template <int D, int A>
__global__ __launch_bounds__(256) void k_emit_fused(EmitArgs a) {
  constexpr int F = rec_floats(D, A);
  extern __shared__ int offs[];  // [nb] block offsets, then [4] wave totals, then int64 total
  const int n = a.n, nb = a.nb;
  int* wtot = offs + ((nb + 3) & ~3);
  int64_t* s_total = reinterpret_cast<int64_t*>(wtot + 4);
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  // ---- exclusive scan of block_count: 256 contiguous chunks, wave shuffle scan + wave totals
  const int per = (nb + 255) / 256;
  const int lo = min(nb, t * per), hi = min(nb, lo + per);
  int local = 0;
  for (int i = lo; i < hi; ++i) local += a.block_count[i];
  int incl = local;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  if (lane == 63) wtot[wave] = incl;
  __syncthreads();
  int wbase = 0, all = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    wbase += (w < wave) ? wtot[w] : 0;
    all += wtot[w];
  }
  int run = wbase + incl - local;
  for (int i = lo; i < hi; ++i) {
    offs[i] = run;
    run += a.block_count[i];
  }
  if (t == 0) *s_total = all;
  __syncthreads();
  const int64_t total = *s_total;
  const int64_t M = a.capacity;
  const int64_t base = a.meta[META_BASE];
  if (blockIdx.x == 0 && t == 0) {
    a.meta_rw[META_TOTAL] = total;
    a.cursor[0] = (base + total) % M;
    const int64_t sz = a.meta[META_SIZE] + total;
    a.cursor[1] = sz < M ? sz : M;
    a.cursor[2] = a.meta[META_GTOTAL] + total;
    a.cursor[3] = total;
  }
  const int64_t start = total > M ? total - M : 0;  // older windows are overwritten this step
  const int64_t nrec = (total - start) * n;
  for (int64_t q = (int64_t)blockIdx.x * 256 + t; q < nrec; q += (int64_t)gridDim.x * 256) {
    const int64_t gl = q / n;
    const int j = (int)(q - gl * n);
    const int64_t g = start + gl;
    int bl = 0, bh = nb - 1;  // largest b with offs[b] <= g
    while (bl < bh) {
      const int mid = (bl + bh + 1) >> 1;
      if ((int64_t)offs[mid] <= g) bl = mid; else bh = mid - 1;
    }
    const int r = (int)(g - offs[bl]);
    const int packed = a.emit_list[(int64_t)bl * BLK + r];
    const int64_t e = (int64_t)bl * BLK + (packed & (BLK - 1));
    int slot = (packed >> 8) + j;
    slot = slot >= a.R ? slot - a.R : slot;
    float rec[F];
    const float4* src = reinterpret_cast<const float4*>(a.ring + (e * a.R + slot) * (int64_t)F);
#pragma unroll
    for (int i = 0; i < F / 4; ++i) {
      const float4 v = src[i];
      rec[4 * i] = v.x;
      rec[4 * i + 1] = v.y;
      rec[4 * i + 2] = v.z;
      rec[4 * i + 3] = v.w;
    }
    int64_t row = base + g;
    if (row >= M) row -= M;
    if (row >= M) row %= M;
    const int64_t o = row * n + j;
    store_vec<D>(a.obs + o * D, rec);
    store_vec<A>(a.act + o * A, rec + D);
    store_vec<D>(a.obs2 + o * D, rec + D + A);
    a.rew[o] = rec[2 * D + A];
    a.cost[o] = rec[2 * D + A + 1];
    a.done[o] = rec[2 * D + A + 2];
    a.logp[o] = rec[2 * D + A + 3];
  }
}

// --------------------------------------------------------------- replay gather / indices
// The replay draw (np.random.randint at nstep_replay_buffer.py:138): window b of draw `counter`
// is the (seed, b, counter) Philox draw modulo the store's window count.
__device__ __forceinline__ int64_t draw_index(uint64_t seed, int64_t b, uint64_t counter, int64_t size) {
  const Rng r = make_rng(seed, (uint64_t)b, counter);
  const u32x4 q = r.draw(7);
  const uint64_t v = ((uint64_t)q.x << 32) | q.y;
  return size > 0 ? (int64_t)(v % (uint64_t)size) : 0;
}

// Last-workgroup arrival of an in-kernel draw: advances the counter once every workgroup has
// READ it. Each thread's counter read was consumed (into the workgroup's drawn rows) before the
// barrier, and thread 0 arrives after the barrier; no data is handed between workgroups, so a
// relaxed arrival suffices (the same argument as k_adam_multi's step counter, optim.hip). The next
// launch reads the new counter across the kernel boundary.
__device__ __forceinline__ void draw_arrive_synced(int64_t* draw, uint64_t counter, unsigned int total) {
  if (threadIdx.x == 0) {
    unsigned int* ticket = reinterpret_cast<unsigned int*>(draw + 1);
    const unsigned int done = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == total - 1u) {
      draw[0] = (int64_t)(counter + 1);
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
__device__ __forceinline__ void draw_arrive(int64_t* draw, uint64_t counter, unsigned int total) {
  __syncthreads();
  draw_arrive_synced(draw, counter, total);
}

// Replay gather over a flat grid: launch_gather cuts every output layout into segments of
// GATHER_CHUNK vectors per workgroup (GatherPlan), so a workgroup copies one contiguous chunk of
// one output. The chunk spans a contiguous run of batch rows: the workgroup stages their window
// indices in LDS once (a coalesced read of the caller's idx, or one Philox draw per row), then
// every thread issues its GATHER_K vector loads before its first store. Sizing the grid by each
// output's bytes (instead of one fixed-width row of workgroups per output) keeps the number of
// workgroups — each of which draws its rows and, on the in-kernel draw, arrives on the draw
// counter's single ticket — near what the bytes need.
template <int VW>
struct GVec;
template <>
struct GVec<1> { using T = float; };
template <>
struct GVec<2> { using T = float2; };
template <>
struct GVec<4> { using T = float4; };

template <int VW>
__device__ __forceinline__ void gather_chunk(const GatherSeg& g, const int64_t* sidx, uint32_t b_lo, uint32_t q0,
                                             uint32_t q1) {
  using V = typename GVec<VW>::T;
  const V* s = reinterpret_cast<const V*>(g.src);
  const V* s2 = reinterpret_cast<const V*>(g.src2);
  V* d = reinterpret_cast<V*>(g.dst);
  V x[GATHER_K];
#pragma unroll
  for (int u = 0; u < GATHER_K; ++u) {
    const uint32_t q = q0 + u * 256 + threadIdx.x;
    const uint32_t qq = q < q1 ? q : q1 - 1;
    const uint32_t b = qq / g.rowlen, i = qq - b * g.rowlen;
    const int64_t w = sidx[b - b_lo];  // the window
    if (g.kind == GATHER_PLAIN) {
      x[u] = s[w * (int64_t)g.src_row + i];
    } else {  // [obs(t) | act(t)] rows of the window: aux0 = (D + A) / VW, aux1 = D / VW, aux2 = A / VW
      const uint32_t t = i / g.aux0, c = i - t * g.aux0;
      const int64_t wr = w * (int64_t)g.src_row + t;  // the store row (window w, step t)
      x[u] = c < g.aux1 ? s[wr * g.aux1 + c] : s2[wr * g.aux2 + (c - g.aux1)];
    }
  }
#pragma unroll
  for (int u = 0; u < GATHER_K; ++u) {
    const uint32_t q = q0 + u * 256 + threadIdx.x;
    if (q < q1) d[q] = x[u];
  }
}

__global__ __launch_bounds__(256) void k_gather(GatherArgs a, GatherPlan p) {
  __shared__ int64_t sidx[GATHER_CHUNK];
  const uint32_t wg = blockIdx.x;
  int y = 0;
#pragma unroll
  for (int k = 1; k < GATHER_MAX_SEGS; ++k) y += (k < p.nseg && wg >= p.seg[k].wg0) ? 1 : 0;
  const GatherSeg& g = p.seg[y];
  const uint32_t q0 = (wg - g.wg0) * GATHER_CHUNK;
  const uint32_t q1 = g.units - q0 < GATHER_CHUNK ? g.units : q0 + GATHER_CHUNK;
  const uint32_t b_lo = q0 / g.rowlen, b_hi = (q1 - 1) / g.rowlen;
  const uint64_t counter = a.draw ? (uint64_t)a.draw[0] : 0u;
  const int64_t size = a.draw ? a.cursor[1] : 0;
  for (uint32_t r = threadIdx.x; r <= b_hi - b_lo; r += 256) {
    const int64_t wv = a.draw ? draw_index(a.seed, b_lo + r, counter, size) : a.idx[b_lo + r];
    sidx[r] = wv;
    // the drawn indices, written once per row: by the workgroup holding the row's first vector
    if (y == 0 && a.idx_out && (uint64_t)(b_lo + r) * g.rowlen >= q0) a.idx_out[b_lo + r] = wv;
  }
  __syncthreads();
  // every thread's counter read was consumed by the draws above: arrive now, so the ticket's
  // round trip overlaps the copy instead of trailing it
  if (a.draw) draw_arrive_synced(a.draw, counter, gridDim.x);
  if (g.dst) {
    if (g.vw == 4)
      gather_chunk<4>(g, sidx, b_lo, q0, q1);
    else if (g.vw == 2)
      gather_chunk<2>(g, sidx, b_lo, q0, q1);
    else
      gather_chunk<1>(g, sidx, b_lo, q0, q1);
  }
}

__global__ __launch_bounds__(256) void k_sample_idx(const int64_t* cursor, uint64_t seed, uint64_t counter,
                                                   int64_t batch, int64_t* idx) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= batch) return;
  idx[b] = draw_index(seed, b, counter, cursor[1]);
}

// the same draw keyed by the device counter draw[0], advanced by the launch
__global__ __launch_bounds__(256) void k_sample_idx_dev(const int64_t* cursor, uint64_t seed, int64_t* draw,
                                                       int64_t batch, int64_t* idx) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t counter = (uint64_t)draw[0];
  if (b < batch) idx[b] = draw_index(seed, b, counter, cursor[1]);
  draw_arrive(draw, counter, gridDim.x);
}

// --------------------------------------------------------------- state transposes
template <typename T>
__global__ __launch_bounds__(256) void k_soa_to_aos(const T* src, T* dst, int W, int64_t E) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= E * W) return;
  const int64_t e = i / W;
  const int c = (int)(i - e * W);
  dst[i] = src[(int64_t)c * E + e];
}
template <typename T>
__global__ __launch_bounds__(256) void k_aos_to_soa(const T* src, T* dst, int W, int64_t E) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= E * W) return;
  const int64_t e = i / W;
  const int c = (int)(i - e * W);
  dst[(int64_t)c * E + e] = src[i];
}

// --------------------------------------------------------------- launchers

template <class Env>
hipError_t launch_rollout_t(const StepArgs& a, hipStream_t st) {
  // logits / obs rows are read as float4 / float2 vectors (load_row_f32): the tensors must be
  // aligned to their row vector width (torch allocations are 256-byte aligned)
  auto aligned = [](const void* p, int n) {
    const uintptr_t w = n % 4 == 0 ? 16 : (n % 2 == 0 ? 8 : 4);
    return p == nullptr || (reinterpret_cast<uintptr_t>(p) % w) == 0;
  };
  if (!aligned(a.act_in ? nullptr : a.logits, 2 * Env::A) || !aligned(a.act_in, Env::A) || !aligned(a.obs, Env::D))
    return hipErrorInvalidValue;
  const int grid = (int)((a.E + BLK - 1) / BLK);
  const int threads = a.defer ? BLK + 64 * EMIT_WAVES : BLK;
  if (a.act_in)
    k_rollout<Env, false><<<grid, threads, 0, st>>>(a);
  else
    k_rollout<Env, true><<<grid, threads, 0, st>>>(a);
  return hipGetLastError();
}
template <class Env>
hipError_t launch_reset_t(const StepArgs& a, hipStream_t st) {
  const int grid = (int)((a.E + BLK - 1) / BLK);
  k_reset<Env><<<grid, BLK, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_rollout(int env_id, const StepArgs& a, hipStream_t st) {
  switch (env_id) {
    case ENV_VANDERPOL: return launch_rollout_t<VanderPol>(a, st);
    case ENV_PENDULUM: return launch_rollout_t<Pendulum>(a, st);
    case ENV_DUCTEDFAN: return launch_rollout_t<DuctedFan>(a, st);
    case ENV_TWOLINK: return launch_rollout_t<TwoLink>(a, st);
    case ENV_SINGLETRACKCAR: return launch_rollout_t<SingleTrackCar>(a, st);
    case ENV_QUADTRACKING: return launch_rollout_t<QuadTracking>(a, st);
  }
  return hipErrorInvalidValue;
}
hipError_t launch_reset(int env_id, const StepArgs& a, hipStream_t st) {
  switch (env_id) {
    case ENV_VANDERPOL: return launch_reset_t<VanderPol>(a, st);
    case ENV_PENDULUM: return launch_reset_t<Pendulum>(a, st);
    case ENV_DUCTEDFAN: return launch_reset_t<DuctedFan>(a, st);
    case ENV_TWOLINK: return launch_reset_t<TwoLink>(a, st);
    case ENV_SINGLETRACKCAR: return launch_reset_t<SingleTrackCar>(a, st);
    case ENV_QUADTRACKING: return launch_reset_t<QuadTracking>(a, st);
  }
  return hipErrorInvalidValue;
}
hipError_t launch_finalize(const int32_t* block_count, int32_t nb, int32_t* block_offset, int64_t* meta,
                           int64_t* cursor, int64_t capacity, hipStream_t st) {
  k_finalize<<<1, 1024, 0, st>>>(block_count, nb, block_offset, meta, cursor, capacity);
  return hipGetLastError();
}
hipError_t launch_emit(const EmitArgs& a, hipStream_t st) {
  const int grid = (int)((a.E + 3) / 4);
  const size_t shm = (size_t)4 * a.R * a.F * sizeof(float);
  k_emit<<<grid, 256, shm, st>>>(a);
  return hipGetLastError();
}
template <int D, int A>
hipError_t launch_emit_fused_t(const EmitArgs& a, hipStream_t st) {
  // one thread per record of a full step (every env emitting); grid-stride beyond 2048 WGs
  const int64_t want = (a.E * a.n + 255) / 256;
  const int grid = (int)(want < 1 ? 1 : (want > 2048 ? 2048 : want));
  const size_t shm = (size_t)((a.nb + 3) & ~3) * sizeof(int) + 4 * sizeof(int) + sizeof(int64_t);
  k_emit_fused<D, A><<<grid, 256, shm, st>>>(a);
  return hipGetLastError();
}
hipError_t launch_emit_fused(int env_id, const EmitArgs& a, hipStream_t st) {
  switch (env_id) {
    case ENV_VANDERPOL: return launch_emit_fused_t<VanderPol::D, VanderPol::A>(a, st);
    case ENV_PENDULUM: return launch_emit_fused_t<Pendulum::D, Pendulum::A>(a, st);
    case ENV_DUCTEDFAN: return launch_emit_fused_t<DuctedFan::D, DuctedFan::A>(a, st);
    case ENV_TWOLINK: return launch_emit_fused_t<TwoLink::D, TwoLink::A>(a, st);
    case ENV_SINGLETRACKCAR: return launch_emit_fused_t<SingleTrackCar::D, SingleTrackCar::A>(a, st);
    case ENV_QUADTRACKING: return launch_emit_fused_t<QuadTracking::D, QuadTracking::A>(a, st);
  }
  return hipErrorInvalidValue;
}
hipError_t launch_gather(const GatherArgs& a, hipStream_t st) {
  if (a.batch <= 0) return hipSuccess;
  // the kernel's vector counts are 32-bit (the largest layouts: (batch + batch n) D, batch n (D + A))
  if (a.batch * ((int64_t)a.n + 1) * ((int64_t)a.D + a.A) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  const int64_t B = a.batch, n = a.n, D = a.D, A = a.A;
  auto fits = [](const void* ptr, int vw) { return ptr == nullptr || reinterpret_cast<uintptr_t>(ptr) % (4 * vw) == 0; };
  // the widest vector dividing every length in floats with every pointer aligned to it
  auto width = [&](std::initializer_list<int64_t> lens, std::initializer_list<const void*> ptrs) {
    for (int vw : {4, 2}) {
      bool ok = true;
      for (int64_t l : lens) ok = ok && l % vw == 0;
      for (const void* q : ptrs) ok = ok && fits(q, vw);
      if (ok) return vw;
    }
    return 1;
  };
  GatherPlan p{};
  uint32_t wg = 0;
  auto add = [&](GatherSeg g, int64_t floats) {
    g.units = (uint32_t)(floats / g.vw);
    g.wg0 = wg;
    p.seg[p.nseg++] = g;
    wg += (g.units + GATHER_CHUNK - 1) / GATHER_CHUNK;
  };
  // the per-row arrays [batch][n][w]: rows of n w floats; segment 0 also carries idx_out
  const float* srcs[7] = {a.s_obs, a.s_act, a.s_rew, a.s_cost, a.s_obs2, a.s_done, a.s_logp};
  float* dsts[7] = {a.o_obs, a.o_act, a.o_rew, a.o_cost, a.o_obs2, a.o_done, a.o_logp};
  const int64_t ws[7] = {D, A, 1, 1, D, 1, 1};
  for (int k = 0; k < 7; ++k) {
    if (!dsts[k] && !(k == 0 && a.idx_out)) continue;
    const int64_t len = n * ws[k];
    GatherSeg g{};
    g.vw = width({len}, {srcs[k], dsts[k]});
    g.src = srcs[k];
    g.dst = dsts[k];
    g.rowlen = g.src_row = (uint32_t)(len / g.vw);
    add(g, B * len);
  }
  if (a.o_obs_act) {  // [batch][n][D + A] = [obs | act] rows of the window
    GatherSeg g{};
    g.vw = width({D, A}, {a.s_obs, a.s_act, a.o_obs_act});
    g.kind = GATHER_OBS_ACT;
    g.src = a.s_obs;
    g.src2 = a.s_act;
    g.dst = a.o_obs_act;
    g.aux0 = (uint32_t)((D + A) / g.vw);
    g.aux1 = (uint32_t)(D / g.vw);
    g.aux2 = (uint32_t)(A / g.vw);
    g.rowlen = (uint32_t)(n * g.aux0);
    g.src_row = (uint32_t)n;  // store rows per window
    add(g, B * n * (D + A));
  }
  if (a.o_v_in) {  // [batch + batch n][D]: obs(b, 0) rows, then the obs2 windows
    const int vw = width({D}, {a.s_obs, a.s_obs2, a.o_v_in});
    GatherSeg h{};
    h.vw = vw;
    h.src = a.s_obs;
    h.dst = a.o_v_in;
    h.rowlen = (uint32_t)(D / vw);
    h.src_row = (uint32_t)(n * D / vw);
    add(h, B * D);
    GatherSeg t{};
    t.vw = vw;
    t.src = a.s_obs2;
    t.dst = a.o_v_in + B * D;
    t.rowlen = t.src_row = (uint32_t)(n * D / vw);
    add(t, B * n * D);
  }
  if (wg == 0) return hipSuccess;
  k_gather<<<wg, 256, 0, st>>>(a, p);
  return hipGetLastError();
}

hipError_t launch_sample_idx(const int64_t* cursor, uint64_t seed, uint64_t counter, int64_t batch,
                             int64_t* idx, hipStream_t st) {
  if (batch <= 0) return hipSuccess;
  k_sample_idx<<<(int)((batch + 255) / 256), 256, 0, st>>>(cursor, seed, counter, batch, idx);
  return hipGetLastError();
}
hipError_t launch_sample_idx_dev(const int64_t* cursor, uint64_t seed, int64_t* draw, int64_t batch, int64_t* idx,
                                 hipStream_t st) {
  if (batch <= 0) return hipSuccess;
  k_sample_idx_dev<<<(int)((batch + 255) / 256), 256, 0, st>>>(cursor, seed, draw, batch, idx);
  return hipGetLastError();
}
hipError_t launch_transpose_f32(const float* src, float* dst, int W, int64_t E, bool to_aos, hipStream_t st) {
  const int64_t n = E * W;
  if (n == 0) return hipSuccess;
  const int grid = (int)((n + 255) / 256);
  if (to_aos)
    k_soa_to_aos<float><<<grid, 256, 0, st>>>(src, dst, W, E);
  else
    k_aos_to_soa<float><<<grid, 256, 0, st>>>(src, dst, W, E);
  return hipGetLastError();
}
hipError_t launch_transpose_f64(const double* src, double* dst, int W, int64_t E, bool to_aos, hipStream_t st) {
  const int64_t n = E * W;
  if (n == 0) return hipSuccess;
  const int grid = (int)((n + 255) / 256);
  if (to_aos)
    k_soa_to_aos<double><<<grid, 256, 0, st>>>(src, dst, W, E);
  else
    k_aos_to_soa<double><<<grid, 256, 0, st>>>(src, dst, W, E);
  return hipGetLastError();
}

}  // namespace mh
