/*
 * msacl_hip.h — C ABI of the MI355X (gfx950) MSACL rollout + update engine.
 *
 * The reference (adamyindh/Multi-Step-Actor-Critic-...; Python only) has no FFI: its hot-path
 * boundary is the duck-typed plugin API behind create_envs / create_sampler / create_buffer.
 * Each entry point below states which reference interface it replaces (file:line relative to
 * the reference's repository root). The Python host layer binds these through ctypes
 *  and mirrors the reference's plugin API on top of them.
 *
 * Conventions
 *   - every data pointer is a DEVICE pointer owned by the caller (torch tensors in the Python
 *     layer); the library only allocates its own per-handle state;
 *   - all work is enqueued asynchronously on `stream` (a hipStream_t; NULL = default stream);
 *     no call synchronises, allocates or copies to the host on the hot path, so the calls
 *     can be captured into a hipGraph;
 *   - functions return 0 on success or a negative MH_E* code; mh_last_error() gives text.
 *     No C++ exception crosses the ABI. A handle is not thread-safe (one host thread/stream).
 *   - layouts: row-major AoS for every tensor exchanged with the caller ([E][obs_dim] etc.),
 *     exactly the shapes the reference's numpy arrays / torch tensors have.
 */
#ifndef MSACL_HIP_H
#define MSACL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_ABI_VERSION 1

/* error codes */
#define MH_OK 0
#define MH_EINVAL (-1)   /* bad argument (null handle, unknown env id, size mismatch)   */
#define MH_EHIP (-2)     /* a HIP runtime call failed                                   */
#define MH_ENOMEM (-3)   /* device allocation failed                                    */
#define MH_ESTATE (-4)   /* call order violated (e.g. rollout before mh_nstep_attach)   */

/* env ids — the six ids accepted by RL/env/make_env.py:16-29 */
#define MH_ENV_VANDERPOL 0
#define MH_ENV_PENDULUM 1
#define MH_ENV_DUCTEDFAN 2
#define MH_ENV_TWOLINK 3
#define MH_ENV_SINGLETRACKCAR 4
#define MH_ENV_QUADTRACKING 5

typedef struct mh_env_s* mh_env_t;

/* Static description of one env (what gymnasium's single_observation_space /
 * single_action_space expose to RL/utils/init_args.py:33-46). Host-only, needs no GPU. */
typedef struct {
  int32_t obs_dim, act_dim;
  int32_t state_dim;      /* float32 persistent state per env (Quad: x v R W = 18)      */
  int32_t xstate_dim;     /* float64 persistent state per env (Quad: Rd_last = 9)        */
  int32_t reset_dim;      /* floats of one injected reset state (= state_dim)           */
  int32_t control_step;   /* Euler substeps per env step                                */
  int32_t max_step;       /* truncation horizon (1000)                                  */
  int32_t record_floats;  /* floats of one n-step ring record (2*obs+act+4, padded to 4) */
  float obs_low[16], obs_high[16];
  float act_low[4], act_high[4];
} mh_env_info_t;

int mh_env_info(int32_t env_id, mh_env_info_t* out);

/* Replaces create_envs (RL/create_pkg/create_envs.py:9-35): a batch of `num_envs` envs of one
 * id, stepped in lockstep on the device. `seed` keys the in-kernel Philox stream used for
 * throughput-mode resets and action noise. */
/* num_envs is bounded so each persistent SoA array stays under 2 GiB (QuadTracking: ~29.8M envs). */
int mh_env_create(int32_t env_id, int64_t num_envs, uint64_t seed, mh_env_t* out);
int mh_env_destroy(mh_env_t h);

/* Replaces SyncVectorEnv.reset (called at RL/trainer/sampler/base.py:98): reset every env.
 * reset_states: [E][reset_dim] injected initial states (parity mode) or NULL (device draws
 * from the reset distribution of RL/env/<Env>.py reset()). obs: [E][obs_dim] output.
 * Also clears the n-step rings if attached. */
int mh_env_reset(mh_env_t h, const float* reset_states, float* obs, void* stream);

/* Replaces envs.step(actions_clip) (RL/trainer/sampler/base.py:148 -> gymnasium 0.28.1
 * SyncVectorEnv.step -> RL/env/<Env>.py step()), including the vector env's autoreset:
 *   act            [E][act_dim]  actions as passed to env.step (not clipped here)
 *   reset_states   [E][reset_dim] state used if env i finishes this step, or NULL (draws)
 *   next_obs       [E][obs_dim]  observation after autoreset (what step() returns)
 *   real_next_obs  [E][obs_dim]  pre-reset observation (infos["final_observation"] rows)
 *   reward         [E] float32 env reward (the vector env's float64 buffer holds exactly it)
 *   terminated/truncated [E] uint8
 * Any output pointer may be NULL. */
int mh_env_step(mh_env_t h, const float* act, const float* reset_states, float* next_obs,
                float* real_next_obs, float* reward, uint8_t* terminated, uint8_t* truncated,
                void* stream);

/* Persistent per-env state, for checkpoints and parity tests. state [E][state_dim],
 * xstate [E][xstate_dim] (may be NULL when xstate_dim == 0), steps [E] (steps since reset). */
int mh_env_get_state(mh_env_t h, float* state, double* xstate, int32_t* steps, void* stream);
int mh_env_set_state(mh_env_t h, const float* state, const double* xstate, const int32_t* steps,
                     void* stream);

/* Device window store = the storage of RL/trainer/buffer/nstep_replay_buffer.py:52-70 laid out
 * exactly as the reference's numpy arrays: obs/obs2 [capacity][n][obs_dim], act
 * [capacity][n][act_dim], rew/cost/done/logp [capacity][n]. cursor is a DEVICE int64[4]:
 * {ptr, size, total_emitted, last_emitted} with ptr/size following store() (:106-119). */
typedef struct {
  float* obs;
  float* act;
  float* rew;
  float* cost;
  float* obs2;
  float* done;
  float* logp;
  int64_t capacity;
  int64_t* cursor;
} mh_window_store_t;

/* Attach per-env n-step deques (RL/trainer/sampler/base.py:95: deque(maxlen=n) per env) and
 * the reward/cost scales of RL/utils/rew_plus_cost.py:18-21. */
int mh_nstep_attach(mh_env_t h, int32_t n_step, float reward_scale, float cost_scale);

/* One lockstep step of BaseSampler._n_step (RL/trainer/sampler/base.py:118-222) minus the
 * policy MLP: TanhGauss sample from `logits` (act_distribution_cls.py:45-57) with in-kernel
 * Philox noise, clip (base.py:140-143), env step + autoreset, rew_plus_cost, deque push, and
 * emission of every full window into `store` in env-index order (base.py:178-217,
 * nstep_replay_buffer.py:122-125).
 *   logits    [E][2*act_dim] StochaPolicy output (mean | std), or NULL when injecting
 *   act_in    [E][act_dim] already-clipped actions to use instead of sampling (parity mode)
 *   logp_in   [E] their log-probabilities (parity mode; NULL -> 0)
 *   reset_states [E][reset_dim] or NULL
 *   obs       [E][obs_dim] in: current observation (policy input); out: next observation
 *   store     window store receiving the emitted windows (NULL: deques only)
 *   act_out/logp_out  optional [E][act_dim] / [E] copies of the actions taken */
int mh_rollout_step(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                    const float* reset_states, float* obs, const mh_window_store_t* store,
                    float* act_out, float* logp_out, void* stream);

/* mh_rollout_step with the emission deferred by one step (same arguments; store required):
 * the windows that become full in this step are copied into `store` by the NEXT deferred step
 * of the same handle — by extra emitter waves of each block, while the env waves step — or by
 * mh_rollout_flush. A horizon of deferred steps followed by mh_rollout_flush leaves the store
 * rows, cursor and ring state identical to the same steps through mh_rollout_step. Every other
 * call that steps, resets or re-attaches the handle flushes a pending emission first. Falls
 * back to the immediate emission when num_envs > 1M or num_envs > store->capacity. */
int mh_rollout_step_deferred(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                             const float* reset_states, float* obs, const mh_window_store_t* store,
                             float* act_out, float* logp_out, void* stream);

/* Emit the pending windows of the last mh_rollout_step_deferred call (no-op when none). */
int mh_rollout_flush(mh_env_t h, void* stream);

/* rew_plus_cost scales (RL/utils/rew_plus_cost.py:18-21) used by every sampler step; also set
 * by mh_nstep_attach. Default 1, 1. */
int mh_env_set_reward_cost_scale(mh_env_t h, float reward_scale, float cost_scale);

/* Exploration noise of BaseSampler (base.py:136-137 -> GaussNoise.sample, explore_noise.py:9):
 * `noise` is a DEVICE float[1] holding the one scalar np.random.normal(mean, std) that is added
 * to every sampled action of a lockstep step, before the clip. The caller refreshes it per step
 * (a device RNG write, capturable). NULL disables. Ignored for injected actions. */
int mh_env_set_action_noise(mh_env_t h, const float* noise);

/* Grow each env's n-step ring to `ring_slots` (>= n_step) records, so that windows stay readable
 * for ring_slots - n_step further steps after they become full (the fused horizon sampler,
 * mh_sample_horizon, emits a whole horizon's windows after it: ring_slots >= n_step + H - 1).
 * Every deque restarts empty (call before sampling); a no-op when the size is unchanged.
 * Needs num_envs <= 1M when ring_slots > n_step. Reference: the per-env deque(maxlen=n) of
 * BaseSampler._n_step (base.py:180-188) — the extra slots only delay the reads. */
int mh_nstep_reserve(mh_env_t h, int32_t ring_slots);

/* A whole horizon of BaseSampler._n_step (RL/trainer/sampler/base.py:118-222, `horizon` lockstep
 * steps of policy -> TanhGauss sample -> clip -> env step -> autoreset -> rew_plus_cost -> deque
 * push) in ONE persistent kernel, followed by one emission launch that copies every window
 * completed in the horizon into `store` in the reference's order (lockstep major, env index
 * within a lockstep; base.py:178-213, nstep_replay_buffer.py:122-125) and advances its cursor.
 * The default StochaPolicy shape only (D -> 256 -> 256 -> 2A, ReLU; obs_dim <= 15): the policy
 * is `packed_policy` as built by mh_policy_pack, with the SAME split-f16 arithmetic as
 * mh_policy_forward, and the env step is mh_rollout_step's, so a horizon gives the same rows,
 * observations and env state bit for bit as `horizon` x (mh_policy_forward +
 * mh_rollout_step_deferred) + mh_rollout_flush with the same noise. Requires the rings reserved
 * for it: mh_nstep_reserve(h, n_step + horizon - 1).
 *   obs        [E][obs_dim] in: current observation; out: the observation after the horizon
 *   act_noise  DEVICE float[horizon] (GaussNoise, one scalar per lockstep) or NULL
 *   act_out / logp_out  optional [horizon][E][act_dim] / [horizon][E]: the sampled actions */
int mh_sample_horizon(mh_env_t h, const float* packed_policy, int32_t obs_dim, int32_t n_out, float* obs,
                      int32_t horizon, const mh_window_store_t* store, const float* act_noise, float* act_out,
                      float* logp_out, void* stream);

/* The emission launch of the last mh_sample_horizon alone, into `store` again: it reads the ring,
 * the per-wave window lists and the header the fused kernel formed, and writes the same store
 * rows (the cursor is not moved), so it is idempotent until the next horizon. A measurement
 * entry (bench.py times the emission at the trainer's own window count with it); windows_out:
 * optional DEVICE int64, the horizon's window count. `horizon` must equal the last
 * mh_sample_horizon's and `store` be the store it emitted into (same cursor), with no other
 * stepping / resetting call on the handle since: MH_EINVAL / MH_ESTATE otherwise. */
int mh_sample_horizon_emit(mh_env_t h, int32_t horizon, const mh_window_store_t* store, int64_t* windows_out,
                           void* stream);

/* The window count of the handle's last mh_sample_horizon (the fused kernel's header aux[0], the
 * windows the horizon completed, = the store cursor's advance of `total`), copied to int64 `out`
 * (DEVICE or pinned HOST) on `stream`; valid until the next mh_sample_horizon on the handle. Lets
 * the sampler report a horizon's window count lazily, without a cursor snapshot + subtraction
 * launched around every horizon. */
int mh_sample_horizon_windows(mh_env_t h, int64_t* out, void* stream);

/* Diagnostics of mh_sample_horizon: copies the handle's device error word (the number of bounded
 * intra-workgroup waits that timed out since mh_env_create; 0 when healthy) to int64 `out`, DEVICE
 * or pinned HOST memory (an async copy on `stream`). A timed-out wait means that horizon's logits,
 * and so its actions and windows, are not trustworthy: the HIP sampler reads the word every
 * log_save_interval iterations and at close() and raises when it is non-zero. */
int mh_sample_horizon_errors(mh_env_t h, int64_t* out, void* stream);

/* Polls of one policy-wave wait of mh_sample_horizon before it gives up (and counts an error);
 * 0 restores the default (2^26, ~1e9 cycles; a healthy hand-off takes < 1e3). Test hook: a tiny
 * limit forces the timeout path so the caller's error reporting can be exercised. */
int mh_sample_horizon_set_spin_limit(mh_env_t h, uint32_t limit);

/* The per-env Philox counters [E] (uint32, DEVICE or pinned HOST memory) that key the in-kernel
 * draws with the handle's seed: every lockstep step of env e draws its action normals and, if the
 * env finishes, its reset state from (seed, e, counter) and then advances the counter by one; a
 * drawn reset (mh_env_reset without states) also advances it by one. Part of the env batch's
 * persistent state (checkpoints) and the key the oracle (oracle/rng.py) replays the draws from.
 * Replaces the reference's RNG state: torch's / numpy's global generators (base.py:127-137,
 * RL/env/<Env>.py reset()). */
int mh_env_get_counters(mh_env_t h, uint32_t* out, void* stream);
int mh_env_set_counters(mh_env_t h, const uint32_t* in, void* stream);

/* The engine's in-kernel draws for n (env index, counter) keys under `seed` — the same inline
 * functions the rollout and fused sampler kernels call: kind 0 writes the four standard normals of
 * the TanhGauss action noise (out [n][4]; components 0..act_dim-1 are used), kind 1 the env's
 * reset draw (out [n][reset_dim], the state a finishing env restarts from). env_idx [n] int64 and
 * ctr [n] uint32 are DEVICE arrays. Used to pin the draws to oracle/rng.py. */
int mh_rng_draw(int32_t env_id, int32_t kind, uint64_t seed, const int64_t* env_idx, const uint32_t* ctr, int64_t n,
                float* out, void* stream);

/* Diagnostics of mh_sample_horizon: later horizons also write the logits every env sampled from
 * to DEVICE [horizon][E][2*act_dim] `logits_out` and the observation it stepped from to
 * [horizon][E][obs_dim] `obs_out` (both NULL: off). */
int mh_sample_horizon_debug_logits(mh_env_t h, float* logits_out, float* obs_out);

/* Per-env step trace of every later mh_rollout_step / mh_rollout_step_deferred of this handle,
 * in the SAME kernel instantiation the call would run anyway (the sampling one when logits are
 * given): the pre-reset observation [E][D] (SyncVectorEnv info["final_observation"], the
 * `real_next_obs` of base.py:156-160), the env's raw float32 reward [E] (before reward_scale),
 * and terminated / truncated [E] (u8) — the values gymnasium's step returns to
 * BaseSampler._n_step (base.py:148). DEVICE pointers owned by the caller; any may be NULL;
 * all NULL switches the trace off. Used by the parity tests of the benchmarked sampler path. */
int mh_rollout_set_trace(mh_env_t h, float* real_next_obs, float* reward, uint8_t* terminated,
                         uint8_t* truncated);

/* Step trace of the post-step env state BEFORE the autoreset overwrites it (the state
 * SyncVectorEnv's `final_observation` is the observation of: QuadTracking.py:205-250 computes it,
 * gymnasium resets after), for every later mh_rollout_step / mh_rollout_step_deferred of this handle:
 * the envs that reset in a step get their pre-reset state written to DEVICE SoA [state_dim][E]
 * floats and [xstate_dim][E] doubles (the mh_env_get_state layouts; xstate required when
 * xstate_dim > 0); the other envs' entries are left as they were (their post-step state is the
 * env state itself). state NULL switches it off. Parity tests only: it lets a terminal row's
 * observation be checked against the observation map of the kernel's own state. */
int mh_rollout_set_trace_state(mh_env_t h, float* state, double* xstate);

/* On-policy trajectory store = OnSampler's mini-batch arrays (RL/trainer/sampler/
 * on_sampler.py:22-41), env-major exactly as the reference's numpy arrays:
 * obs/obs2 [E][horizon][obs_dim], act [E][horizon][act_dim], rew/cost/logp [E][horizon] float32,
 * done [E][horizon] uint8 (np.bool_). */
typedef struct {
  float* obs;
  float* act;
  float* rew;
  float* cost;
  float* obs2;
  uint8_t* done;
  float* logp;
  int32_t horizon;
} mh_traj_store_t;

/* One lockstep step of OnSampler._sample (on_sampler.py:49-55 -> BaseSampler._step,
 * base.py:225-298) minus the policy/value MLPs: TanhGauss sample (or injected actions), clip,
 * env step + autoreset, rew_plus_cost, and column t of every trajectory array
 * (_process_experiences, on_sampler.py:131-141). Arguments as mh_rollout_step. */
int mh_rollout_traj_step(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                         const float* reset_states, float* obs, const mh_traj_store_t* traj, int32_t t,
                         float* act_out, float* logp_out, void* stream);

/* GAE + discounted returns over a whole trajectory block (OnSampler._process_experiences /
 * _finish_trajs, on_sampler.py:108-154). All arrays [num_envs][horizon]:
 *   val   V(obs_t)                 (mb_val)
 *   val2  V(real_next_obs_t)       (read only where a segment ends: done or t == horizon-1)
 *   rew, done                      (mb_rew, mb_done)
 *   adv, ret                       outputs (mb_adv, mb_ret)
 * Segments end at done or the horizon; bootstrap = val2 * (1 - done). */
int mh_gae(const float* val, const float* val2, const float* rew, const uint8_t* done, int64_t num_envs,
           int32_t horizon, double gamma, double gae_lambda, float* adv, float* ret, void* stream);

/* ---- sampler policy forward: StochaPolicy's MLP (RL/apprfunc/mlp.py:111-136, obs -> Linear ->
 * ReLU -> Linear -> ReLU -> Linear -> (mean | log_std)) as one fused MFMA kernel: split-f16
 * products (three per f32 product, f32 accumulation) for obs_dim <= 15 and out_dim <= 8 (every
 * env's policy head), f32-input MFMAs otherwise. Supported shape: hidden sizes 256 x 256 (every
 * reference script's default), obs_dim <= 16, out_dim (= 2 * act_dim) <= 32, W2 and W3 16-byte
 * aligned; other shapes return MH_EINVAL (the caller uses PyTorch). ---- */
/* floats of the packed parameter buffer for a given obs_dim */
int mh_policy_packed_size(int32_t obs_dim, int64_t* floats_out);
/* Pack nn.Linear parameters (row-major [out][in] weights, [out] biases, device pointers) into the
 * per-lane MFMA fragment order; run once per parameter update (inside a captured sample()). */
int mh_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                   const float* b3, int32_t obs_dim, int32_t hidden1, int32_t hidden2, int32_t out_dim,
                   float* packed, void* stream);
/* logits [num_envs][out_dim] = MLP(obs [num_envs][obs_dim]), the raw head output (the log_std
 * half is clamped/exponentiated by the rollout kernel, mh_nstep_set_log_std_clamp). */
int mh_policy_forward(const float* packed, const float* obs, int64_t num_envs, int32_t obs_dim, int32_t out_dim,
                      float* logits, void* stream);

/* ---- PyTorch MLP training helpers (the MLPs stay nn.Modules; these replace kernels inside their
 * autograd backward / optimiser step) ---- */
/* Rows of scratch `partial` needed by mh_act_grad_colsum for M rows: partial is [chunks][N]. */
int mh_act_grad_chunks(int64_t rows, int32_t* chunks_out);
/* g = dy * act'(y) (act: 0 identity, 1 ReLU via y > 0, 2 tanh via 1 - y^2) and db = column sums of
 * g, all [rows][cols] row-major; g may be NULL (identity activation: g is dy), db may be NULL.
 * Replaces threshold_backward / tanh_backward + the bias-gradient reduction of a Linear layer
 * (RL/apprfunc/mlp.py:18-30 layers under autograd). Deterministic (fixed summation order).
 * partial: mh_act_grad_chunks(rows) x cols floats of workspace. tickets: NULL (two launches) or a
 * DEVICE uint32 array of ceil(cols / 64) counters, zero on entry and left zero (one per stream):
 * the bias gradient is then finished inside the same launch. */
int mh_act_grad_colsum(const float* dy, const float* y, int64_t rows, int32_t cols, int32_t act, float* g,
                       float* db, float* partial, uint32_t* tickets, void* stream);
/* One torch.optim.Adam step (torch.optim.Adam(fused/capturable) math: betas, eps, no weight decay /
 * amsgrad / maximize) over a list of parameter tensors in one launch per 32 tensors, replacing
 * the optimiser.step() of every reference algorithm (RL/algorithm/{msacl,sac,lac,ppo,polyc}.py). Each entry: param,
 * grad, exp_avg, exp_avg_sq (numel floats each, contiguous, DEVICE) and step (DEVICE float32
 * scalar, the PyTorch capturable state; read, then advanced by one). ticket: DEVICE uint32, zero
 * on entry, left zero (one per stream). Capturable (no host sync); the list itself is host memory
 * passed by value in the kernel arguments. */
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;
  int64_t numel;
} mh_adam_tensor_t;
int mh_adam_multi(const mh_adam_tensor_t* tensors, int32_t n, double lr, double beta1, double beta2, double eps,
                  uint32_t* ticket, void* stream);
/* mh_adam_multi with one learning rate per tensor (lrs[n], host array): several optimisers' steps
 * in one launch (MSACL's policy and alpha optimisers, msacl.py:405-441). */
int mh_adam_multi_lr(const mh_adam_tensor_t* tensors, int32_t n, const double* lrs, double beta1, double beta2,
                     double eps, uint32_t* ticket, void* stream);

/* Polyak averaging of a target network, target = target * polyak + (1 - polyak) * source
 * (both scalars rounded to float32, two roundings as p_t.mul_(polyak); p_t.add_((1 - polyak) * p)
 * in RL/algorithm/sac.py:204-217 and msacl.py:445-460), over a tensor list in one launch per 32. */
typedef struct {
  float* target;
  const float* source;
  int64_t numel;
} mh_polyak_tensor_t;
int mh_polyak_multi(const mh_polyak_tensor_t* tensors, int32_t n, double polyak, void* stream);

/* f32 GEMM on the f32 MFMA (csrc/gemm.hip) for the update phase's nn.Linear layers
 * (RL/apprfunc/mlp.py:18-30 forward; autograd's input / weight gradients):
 *   C[M][N] = act(op(A)[M][K] . op(B)[K][N] + bias[N]),  act 0 identity, 1 ReLU, 2 tanh
 *   op(A)(m,k) = trans_a ? A[k*lda + m] : A[m*lda + k];  op(B)(k,n) = trans_b ? B[n*ldb + k] : B[k*ldb + n]
 * bias may be NULL; each operand must be smaller than 2 GiB. Shapes whose plan splits K across
 * workgroups need a `workspace` of the float count mh_gemm_workspace reports (0 = not needed); the split partials are summed in
 * split order by a second launch (deterministic). */
int mh_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t* workspace_floats);
int mh_gemm_f32(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a, int32_t trans_b, int32_t act,
                float* workspace, void* stream);

/* One nn.Linear + activation layer's backward (autograd of RL/apprfunc/mlp.py:18-30 layers) for
 * y = act(x W^T + b), W [n_out][n_in], over `rows` rows, with g = dy * act'(y) formed inside the
 * GEMMs (never written to memory):
 *   dx [rows][n_in] = g W;  dw [n_out][n_in] = g^T x;  db [n_out] = column sums of g
 * Each output may be NULL when not wanted (db needs dw). mh_linear_backward_plan says whether a
 * request is supported (tall dx: rows >= 2048, n_in % 64 == 0, n_out % 4 == 0, n_out >= 64; dw/db:
 * n_out and n_in multiples of 64, rows >= 1024) and the workspace floats it needs; matrices
 * contiguous and 16-byte aligned. Otherwise use mh_act_grad_colsum + mh_gemm_f32. */
/* The MSACL update's policy head on B*n rows of the StochaPolicy MLP's raw [mean | log_std]
 * (msacl.py:242-251, 270-273, 340-394; mlp.py:132-136; act_distribution_cls.py:39-62): std =
 * exp(clamp(log_std, lo, hi)); with eps: the TanhGauss reparameterised sample written into the
 * critic input rows xq = [obs | act] (D + A columns) and its log-prob new_logp; with old_act:
 * log_prob(old_act) into old_logp. Its backward gives d_raw from d_xq (the action columns),
 * d_new_logp and d_old_logp (each nullable), as autograd accumulates them. A <= 8. */
int mh_policy_head(const float* raw, const float* eps, const float* obs, const float* old_act, const float* high,
                   const float* low, int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, float* xq,
                   float* new_logp, float* old_logp, void* stream);
int mh_policy_head_backward(const float* raw, const float* eps, const float* old_act, const float* high,
                            const float* low, const float* d_xq, const float* d_new_logp, const float* d_old_logp,
                            int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, float* d_raw,
                            void* stream);
/* mh_policy_head with the rsample noise drawn in-kernel (TanhGaussDistribution.rsample's
 * torch.normal draw, act_distribution_cls.py:45-49, whose values are distribution-matched only):
 * eps_out[r][i] = standard normal from Philox4x32-10 keyed by (seed, row r, counter[0]), Box-Muller,
 * written for the backward (mh_policy_head_backward's eps). counter: device uint64[2], zeroed once;
 * every launch advances counter[0] by one on the device (counter[1] is its workgroup arrival
 * count), so a captured graph draws new noise on each replay. */
int mh_policy_head_sample(const float* raw, const float* obs, const float* old_act, const float* high, const float* low,
                          int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, uint64_t seed,
                          uint64_t* counter, float* eps_out, float* xq, float* new_logp, float* old_logp,
                          void* stream);
/* Input gradient of y = act(x W^T + b) for a narrow input (n_in <= 32, n_out <= 1024) when no
 * weight / bias gradient is wanted (a frozen critic's first layer): dx = (dy * act'(y)) W with the
 * activation derivative formed on the fly. Row-major contiguous dy, y [rows][n_out], W [n_out][n_in]. */
int mh_dx_narrow(const float* dy, const float* y, int32_t act, const float* W, int64_t rows, int32_t n_out,
                 int32_t n_in, float* dx, void* stream);
/* LyapunovValue's V = sum_j y[r][j]^2 per row (RL/apprfunc/mlp.py, torch.pow(y, 2).sum(-1)) and its
 * backward dy = g[r] * (2 y) (the pow backward's bits). Row-major contiguous y [rows][cols]. */
int mh_square_sum(const float* y, int64_t rows, int32_t cols, float* out, void* stream);
int mh_square_sum_backward(const float* y, const float* g, int64_t rows, int32_t cols, float* dy, void* stream);
/* Backward of a narrow identity output layer y = x W^T + b (W [n_out][n_in], n_out <= 16: the
 * critic / policy heads of RL/apprfunc/mlp.py:18-30 under autograd): dx = dy W, dW = dy^T x,
 * db = column sums of dy in one pass over x plus a block-ordered finish (deterministic). Any
 * output may be NULL (db needs dw); workspace: mh_head_backward_workspace floats when dw is wanted.
 * Row-major contiguous operands. */
int mh_head_backward_workspace(int64_t rows, int32_t n_out, int32_t n_in, int64_t* floats_out);
int mh_head_backward(const float* dy, const float* x, const float* W, int64_t rows, int32_t n_out, int32_t n_in,
                     float* dx, float* dw, float* db, float* workspace, void* stream);
int mh_linear_backward_plan(int64_t rows, int64_t n_out, int64_t n_in, int32_t need_dx, int32_t need_dw,
                            int32_t need_db, int32_t* supported, int64_t* workspace_floats);
int mh_linear_backward(const float* dy, const float* y, int32_t act, const float* x, const float* W, int64_t rows,
                       int64_t n_out, int64_t n_in, float* dx, float* dw, float* db, float* workspace, void* stream);

/* Grouped layers: `groups` products / layer backwards of ONE shape in one launch, group q's operands
 * at the group-0 pointers + q x the strides (floats). They replace the two critic networks q1, q2
 * of RL/algorithm/msacl.py:227-266 (critic update) and :383-391 (the policy step's frozen
 * critics), each evaluated by RL/apprfunc/mlp.py ActionValue.forward (mlp.py:18-30 layers) and
 * differentiated by autograd, with one launch per layer for both networks (the engine keeps the
 * two networks' layer parameters side by side, so their activations are the halves of one
 * [rows][2H] buffer: leading dimension 2H, group stride H). Each group's result is bit-identical
 * to the ungrouped entry point on that group's operands.
 *   mh_gemm_f32_grouped: mh_gemm_f32's tall path (rows >= 2048, N % 64 == 0, K % 4 == 0, K >= 1,
 *     16-byte aligned rows) and its one-output path (N == 1); MH_EINVAL for other shapes.
 *   mh_linear_backward_grouped: mh_linear_backward with leading dimensions (dy and y share ld_dy;
 *     x: ld_x; dx: ld_dx); workspace: groups x mh_linear_backward_plan's floats.
 *   mh_head_backward_grouped: mh_head_backward with x / dx leading dimensions; workspace: groups x
 *     mh_head_backward_workspace floats when dw is wanted. */
int mh_gemm_f32_grouped(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                        int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a, int32_t trans_b, int32_t act,
                        int32_t groups, int64_t stride_a, int64_t stride_b, int64_t stride_bias, int64_t stride_c,
                        void* stream);
int mh_linear_backward_grouped(const float* dy, const float* y, int32_t act, const float* x, const float* W,
                               int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x, int64_t ld_dx,
                               int32_t groups, int64_t stride_dy, int64_t stride_x, int64_t stride_w,
                               int64_t stride_dx, int64_t stride_dw, int64_t stride_db, float* dx, float* dw,
                               float* db, float* workspace, void* stream);
int mh_head_backward_grouped(const float* dy, const float* x, const float* W, int64_t rows, int32_t n_out,
                             int32_t n_in, int64_t ld_x, int64_t ld_dx, int32_t groups, int64_t stride_dy,
                             int64_t stride_x, int64_t stride_w, int64_t stride_dx, int64_t stride_dw,
                             int64_t stride_db, float* dx, float* dw, float* db, float* workspace, void* stream);

/* A whole 3-layer MLP forward (RL/apprfunc/mlp.py:18-30 mlp([k1, hidden, hidden, n_out]): Linear ->
 * act1 -> Linear -> act2 -> Linear -> act3, the policy / critic / Lyapunov networks of every
 * reference algorithm) in ONE launch instead of one per layer: h1 = act1(x W1^T + b1),
 * h2 = act2(h1 W2^T + b2), y = act3(h2 W3^T + b3), row-major operands (x [rows][ldx], W1 [hidden][k1],
 * W2 [hidden][hidden], W3 [n_out][hidden]); h1 / h2 [rows][ldh] are written when non-NULL (autograd
 * keeps them for the backward), y [rows][ldy]. Supported: k1 <= 32, hidden == 256, n_out <= 16 or a
 * multiple of 64 up to 256; act 0 identity, 1 ReLU, 2 tanh. f32 products (MFMA), f32 accumulation.
 * groups > 1 evaluates `groups` networks of one shape (the twin critics) in the same launch: group q
 * reads and writes each operand at its group-0 pointer + q x group_strides[i] floats, host array
 * {x, W1, b1, W2, b2, W3, b3, h (h1 and h2), y}. */
int mh_mlp3_forward(const float* x, int64_t rows, int32_t k1, int64_t ldx, const float* W1, const float* b1,
                    const float* W2, const float* b2, const float* W3, const float* b3, int32_t hidden, int32_t n_out,
                    int32_t act1, int32_t act2, int32_t act3, float* h1, float* h2, int64_t ldh, float* y, int64_t ldy,
                    int32_t groups, const int64_t* group_strides, void* stream);

/* Two network sets of one shape in ONE mh_mlp3_forward launch (the twin critics on [obs | act] and
 * the twin target critics on [obs2 | next act], RL/algorithm/msacl.py:240-247): set A = {x, params
 * = {W1, b1, W2, b2, W3, b3}, h1, h2, y} as in mh_mlp3_forward, set B = {x_b, params_b, y_b} run as
 * groups [groups, 2 groups) with the same group strides, its activations never kept. Each set's
 * results equal its own mh_mlp3_forward call bit for bit. */
int mh_mlp3_forward_pair(const float* x, const float* x_b, int64_t rows, int32_t k1, int64_t ldx,
                         const float* const* params, const float* const* params_b, int32_t hidden, int32_t n_out,
                         int32_t act1, int32_t act2, int32_t act3, float* h1, float* h2, int64_t ldh, float* y,
                         float* y_b, int64_t ldy, int32_t groups, const int64_t* group_strides, void* stream);

/* LyapunovValue (RL/apprfunc/mlp.py LyapunovValue: V(x) = sum_n MLP(x)_n^2, msacl.py:275-276) in the
 * MLP's launches: mh_mlp3_forward (set A only) that also writes v [rows] = sum over the n_out
 * outputs of y^2, in mh_square_sum's order (bit-identical); and its backward: mh_mlp3_backward's
 * chain with the output gradient dy = dv[row] (2 y) formed in-kernel from the forward output y
 * (mh_square_sum_backward's expression) and written to g3 [rows][ldy] for the weight gradients.
 * n_out a multiple of 64. */
int mh_mlp3_forward_sqsum(const float* x, int64_t rows, int32_t k1, int64_t ldx, const float* const* params,
                          int32_t hidden, int32_t n_out, int32_t act1, int32_t act2, int32_t act3, float* h1,
                          float* h2, int64_t ldh, float* y, int64_t ldy, float* v, void* stream);
int mh_mlp3_backward_sqsum(const float* y, int64_t ldy, const float* dv, const float* h1, const float* h2, int64_t ldh,
                           const float* W1, const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden,
                           int32_t n_out, int32_t act1, int32_t act2, float* g3, float* g2, float* g1, int64_t ldg,
                           float* dx, int64_t ldx, void* stream);

/* The input-gradient chain of mh_mlp3_forward's network (its autograd backward, identity output
 * activation) in ONE launch: with dy [rows][ldy] the gradient of y,
 *   g2 = (dy W3) * act2'(h2),  g1 = (g2 W2) * act1'(h1),  dx = g1 W1
 * (act' read from the kept activations h1 / h2 [rows][ldh], as autograd's threshold / tanh
 * backward). g2 / g1 [rows][ldg] (the weight gradients' left operands: dW2 = g2^T h1, db2 = column
 * sums of g2, ...) and dx [rows][ldx] are written when non-NULL. groups > 1: `groups` networks of
 * one shape (the twin critics), group q's operands at + q x group_strides[i] floats, host array
 * {dy, h (h1 and h2), W1, W2, W3, g (g1 and g2)}; dx is the SUM of the groups' input gradients (what
 * autograd accumulates for an input both critics read). Shapes as mh_mlp3_forward. */
int mh_mlp3_backward(const float* dy, int64_t ldy, const float* h1, const float* h2, int64_t ldh, const float* W1,
                     const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden, int32_t n_out,
                     int32_t act1, int32_t act2, float* g2, float* g1, int64_t ldg, float* dx, int64_t ldx,
                     int32_t groups, const int64_t* group_strides, void* stream);

/* The fused forward's rows per workgroup for the mh_mlp3_forward* launches that follow (host
 * state, read at launch, so also at graph capture): 0 = the default two 16-row tiles per wave;
 * -1 = the fewest tiles that still give one workgroup per CU (the fastest grid for a launch that
 * runs alone on the GPU, slower beside a concurrent branch: DESIGN 3.3); 1..4 fixed. The
 * environment variable MH_MLP_RT overrides it. Bits do not depend on it. */
int mh_mlp3_set_row_tiles(int32_t mode);

/* mh_mlp3_backward plus the output layer's gradients (n_out <= 16; the twin critics' q heads):
 * dw3 [n_out][hidden] = dy^T h2 and, when non-NULL, db3 [n_out] = the column sums of dy, group q's
 * at + q x gs_dw3 / gs_db3 floats. The chain launch forms each 16-row block's partials from the dy
 * rows and h2 columns it already holds; one more launch adds them in block order (deterministic;
 * the same bits as mh_head_backward's below 16,384 rows). workspace: the floats
 * mh_mlp3_backward_w3_workspace reports. Replaces mh_mlp3_backward + mh_head_backward_grouped for
 * TwinCritic.backward_weights (ActionValue's last nn.Linear, RL/apprfunc/mlp.py). */
int mh_mlp3_backward_w3_workspace(int64_t rows, int32_t hidden, int32_t n_out, int32_t groups, int64_t* floats_out);
int mh_mlp3_backward_w3(const float* dy, int64_t ldy, const float* h1, const float* h2, int64_t ldh, const float* W1,
                        const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden, int32_t n_out,
                        int32_t act1, int32_t act2, float* g2, float* g1, int64_t ldg, float* dx, int64_t ldx,
                        int32_t groups, const int64_t* group_strides, float* dw3, float* db3, int64_t gs_dw3,
                        int64_t gs_db3, float* workspace, void* stream);

/* Several weight gradients of one backward (the three layers of an MLP, both twin critics') in two
 * launches: for each product, dw [n_out][n_in] = g^T x over `rows` and, when db is non-NULL,
 * db [n_out] = the column sums of g, with g [rows][ld_g] the layer's pre-activation gradient (as
 * mh_mlp3_backward writes it) and x [rows][ld_x] the layer's input. Every product is split over the
 * rows into partials that one reduce launch adds in split order (deterministic). Supported: rows >=
 * 1024, 16-byte aligned g / x with ld_g, ld_x multiples of 4, and either n_out % 64 == 0 and
 * n_in % 4 == 0, or a narrow layer n_out < 64, n_out % 4 == 0, n_in % 64 == 0, ld_g == n_out; at most
 * 6 products. Replaces the per-layer weight-gradient GEMMs + bias reductions of autograd
 * (RL/apprfunc/mlp.py:18-30 layers). workspace: mh_weight_grads_workspace floats. */
typedef struct {
  const float* g;
  int64_t ld_g;
  const float* x;
  int64_t ld_x;
  int64_t n_out, n_in;
  float* dw;
  float* db;
} mh_wgrad_t;
int mh_weight_grads_workspace(const mh_wgrad_t* products, int32_t n, int64_t rows, int64_t* floats_out);
int mh_weight_grads(const mh_wgrad_t* products, int32_t n, int64_t rows, float* workspace, void* stream);

/* StochaPolicy's head (RL/apprfunc/mlp.py:132-136) on [rows][2 act_dim] rows:
 *   out = [mean | exp(clamp(log_std, min_log_std, max_log_std))] of raw = [mean | log_std]
 * and its backward d_raw = [d_mean | d_std * std * (min <= log_std <= max)], one launch each
 * (PyTorch: chunk + clamp + exp + cat forward, four kernels backward). */
int mh_stocha_head(const float* raw, int64_t rows, int32_t act_dim, float min_log_std, float max_log_std, float* out,
                   void* stream);
int mh_stocha_head_backward(const float* raw, const float* out, const float* d_out, int64_t rows, int32_t act_dim,
                            float min_log_std, float max_log_std, float* d_raw, void* stream);

/* TanhGaussDistribution (RL/utils/act_distribution_cls.py:15-85) on [rows][2A] logits (mean | std)
 * with DEVICE action bounds high/low [A] (A <= 8), forward and backward as single launches:
 *   rsample   (eps [rows][A] standard normals) -> act [rows][A], logp [rows]
 *   log_prob  (act [rows][A])                  -> logp [rows]
 * The backward entry points return d_logits [rows][2A]; d_act / d_logp may be NULL (zero). */
int mh_tanh_gauss_rsample(const float* logits, const float* eps, const float* high, const float* low, int64_t rows,
                          int32_t act_dim, float* act, float* logp, void* stream);
int mh_tanh_gauss_rsample_backward(const float* logits, const float* eps, const float* high, const float* low,
                                   const float* d_act, const float* d_logp, int64_t rows, int32_t act_dim,
                                   float* d_logits, void* stream);
int mh_tanh_gauss_log_prob(const float* logits, const float* act, const float* high, const float* low, int64_t rows,
                           int32_t act_dim, float* logp, void* stream);
int mh_tanh_gauss_log_prob_backward(const float* logits, const float* act, const float* high, const float* low,
                                    const float* d_logp, int64_t rows, int32_t act_dim, float* d_logits,
                                    void* stream);

/* Per-kernel HIP-event timing of mh_rollout_step (profiling aid; do not enable inside a
 * captured hipGraph). read_timing drains the pending events (host sync) and returns the summed
 * milliseconds of {step kernel, window scan, window emission} and the number of timed calls. */
int mh_env_set_timing(mh_env_t h, int32_t enable);
int mh_env_read_timing(mh_env_t h, double* ms_out, int64_t* launches_out, int32_t reset);

/* Let mh_rollout_step take the policy head's RAW output (mean | log_std) and apply
 * StochaPolicy's std = exp(clamp(log_std, lo, hi)) (RL/apprfunc/mlp.py:132-136) in-kernel,
 * saving the chunk/clamp/exp/cat launches of the PyTorch forward. */
int mh_nstep_set_log_std_clamp(mh_env_t h, int32_t enable, float lo, float hi);

/* NstepReplayBuffer.sample_batch gather (RL/trainer/buffer/nstep_replay_buffer.py:128-150):
 * out_X[b] = store.X[idx[b]] for the 7 arrays (any out pointer may be NULL). */
int mh_replay_gather(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim,
                     int32_t act_dim, const int64_t* idx, int64_t batch, float* out_obs,
                     float* out_act, float* out_rew, float* out_cost, float* out_obs2,
                     float* out_done, float* out_logp, void* stream);

/* mh_replay_gather plus the two joint layouts the MSACL update reads, so that it concatenates
 * nothing per update (RL/algorithm/msacl.py:236-238 q(obs, act) and :395-396 V(obs_0), V(obs2)):
 * out_obs_act [batch][n][obs_dim + act_dim] = [obs | act] rows; out_v_in [batch + batch n][obs_dim]
 * = obs[b][0] for every b, then obs2[b][t] rows in (b, t) order. Either may be NULL. */
int mh_replay_gather_joint(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim,
                           int32_t act_dim, const int64_t* idx, int64_t batch, float* out_obs,
                           float* out_act, float* out_rew, float* out_cost, float* out_obs2,
                           float* out_done, float* out_logp, float* out_obs_act, float* out_v_in,
                           void* stream);

/* Device uniform indices in [0, size) from the store cursor (np.random.randint at
 * nstep_replay_buffer.py:138), keyed by (seed, draw counter). */
int mh_replay_sample_indices(const mh_window_store_t* store, uint64_t seed, uint64_t counter,
                             int64_t batch, int64_t* idx_out, void* stream);

/* mh_replay_sample_indices keyed by a DEVICE draw counter: draw_state [2] int64 (0-initialised;
 * [0] the counter, [1] the launch's arrival ticket, 0 between launches). Draw k of a buffer uses
 * counter k and advances draw_state[0] by one inside the launch, so the call can be captured in a
 * HIP graph and replayed (each replay is the next draw); same indices as
 * mh_replay_sample_indices(..., counter = k, ...). */
int mh_replay_sample_indices_dev(const mh_window_store_t* store, uint64_t seed, int64_t* draw_state,
                                 int64_t batch, int64_t* idx_out, void* stream);

/* The replay draw and mh_replay_gather_joint in ONE launch (nstep_replay_buffer.py:136-148):
 * the indices are drawn inside the gather from (seed, draw_state[0]) exactly as
 * mh_replay_sample_indices_dev draws them, written to idx_out (nullable), and the counter is
 * advanced by the launch. Graph-capturable (the window count is read from store->cursor). */
int mh_replay_draw_gather(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim,
                          int32_t act_dim, uint64_t seed, int64_t* draw_state, int64_t batch,
                          int64_t* idx_out, float* out_obs, float* out_act, float* out_rew,
                          float* out_cost, float* out_obs2, float* out_done, float* out_logp,
                          float* out_obs_act, float* out_v_in, void* stream);

/* ---- MSACL target / certificate kernels (RL/algorithm/msacl.py), all [B][n] float32 ---- */

/* _q_update backup + twin MSE (msacl.py:242-257):
 *   backup = rew + (1-done) * gamma * (min(q1t, q2t) - alpha * next_logp)
 *   loss = mean((q1-backup)^2) + mean((q2-backup)^2)
 * Writes backup [B*n], dq1/dq2 = dloss/dq (gradients for autograd), loss_out [1], and
 * abs_td [B] = mean_k (|q1-backup| + |q2-backup|)/2 per window (PER priority source).
 * weight [B] (nullable): per-window importance weights (prioritized replay); with weights the
 * loss is mean_b,k w_b (q - backup)^2. NULL reproduces the reference loss exactly. */
int mh_msacl_q_target(const float* q1, const float* q2, const float* q1t, const float* q2t,
                      const float* next_logp, const float* rew, const float* done,
                      const float* log_alpha, const float* weight, float gamma, int32_t B,
                      int32_t n, float* backup, float* dq1, float* dq2, float* loss_out,
                      float* abs_td, void* stream);

/* mh_msacl_q_target plus the logged critic means (msacl.py:211-222, q1.mean() / q2.mean()):
 * q_means [2] (nullable) receives mean(q1), mean(q2) from the same pass and the same fixed-order
 * float64 reduction as the loss, in place of two separate mean reductions. */
int mh_msacl_q_target_stats(const float* q1, const float* q2, const float* q1t, const float* q2t,
                            const float* next_logp, const float* rew, const float* done,
                            const float* log_alpha, const float* weight, float gamma, int32_t B,
                            int32_t n, float* backup, float* dq1, float* dq2, float* loss_out,
                            float* abs_td, float* q_means, void* stream);

/* The seven logged scalars of model_update (msacl.py:211-222) packed in one launch:
 * out [7] = {entropy, exp(log_alpha), q_means[0], q_means[1], loss_q, loss_lya, loss_policy};
 * every input is a one-element device scalar (q_means: two). */
int mh_msacl_tb_pack(const float* entropy, const float* log_alpha, const float* q_means,
                     const float* loss_q, const float* loss_lya, const float* loss_policy, float* out,
                     void* stream);

/* mh_msacl_tb_pack into slot ctr[0] % slots of ring [slots][8] (element 7 = the low 32 bits of
 * ctr[0], as float bits: the reader checks that the slot still holds its update), then
 * ctr[0] += 1. Inside a replayed update graph this keeps each update's logged scalars readable for
 * `slots` further updates with no copy out of the graph's output. */
int mh_msacl_tb_pack_ring(const float* entropy, const float* log_alpha, const float* q_means,
                          const float* loss_q, const float* loss_lya, const float* loss_policy, float* ring,
                          int64_t* ctr, int32_t slots, void* stream);

/* _lyapunov_update certificate (msacl.py:279-332). Inputs: logp (policy log-prob of the
 * stored actions), old_logp, V(obs) lya_obs, V(obs2) lya_obs2, obs/obs2 [B][n][D].
 * Coefficients c (start_obs_norm_coef), w (lya_diff_coef), s (start_lya_coef) are [n].
 * Writes is_clip [B*n], esl [B*n], lya_diff [B], loss_out [1] (= bound*pos_scale +
 * mean(lya_diff)*diff_scale) and gradients d_lya_obs [B*n], d_lya_obs2 [B*n]. */
int mh_msacl_lyapunov(const float* logp, const float* old_logp, const float* lya_obs,
                      const float* lya_obs2, const float* obs, const float* obs2, const float* c,
                      const float* w, const float* s, float alpha1, float alpha2,
                      float pos_scale, float diff_scale, int32_t B, int32_t n, int32_t D,
                      float* is_clip, float* esl, float* lya_diff, float* loss_out,
                      float* d_lya_obs, float* d_lya_obs2, void* stream);

/* _policy_update stability advantage (msacl.py:383-400):
 *   adv_raw[b] = sum_k w_k (s_k V(obs_b0) - V(obs2_bk)); stats_out = {sum, sumsq} (float64)
 * Normalisation is a second call so the (sum, sumsq, count) triple can be all-reduced
 * across ranks in between. */
int mh_msacl_stability_adv(const float* lya_obs0, const float* lya_obs2, const float* w,
                           const float* s, int32_t B, int32_t n, float* adv_raw,
                           double* stats_out, void* stream);
/* PPO-clipped surrogate on the normalised advantage (msacl.py:400-405):
 *   adv = (adv_raw - mean) / (std + 1e-8) with mean/std from stats (count = n_total);
 *   loss = mean(min(r*adv, clip(r, 1-eps, 1+eps)*adv)); d_ratio = dloss/dr. */
int mh_msacl_ppo_clip(const float* ratio, const float* adv_raw, const double* stats,
                      double n_total, float clip_eps, int32_t B, float* adv, float* loss_out,
                      float* d_ratio, void* stream);
/* The policy loss of msacl.py:383-391 on B*n elements: loss = (min(q1, q2) - exp(log_alpha) logp).mean()
 * and entropy = -logp.mean() (one workgroup, fixed-order sums), and its autograd backward for a
 * DEVICE upstream gradient g_loss (min: the smaller input, ties half each). */
int mh_msacl_policy_loss(const float* q1, const float* q2, const float* logp, const float* log_alpha, int64_t N,
                         float* loss_out, float* entropy_out, void* stream);
int mh_msacl_policy_loss_backward(const float* q1, const float* q2, const float* log_alpha, const float* g_loss,
                                  int64_t N, float* dq1, float* dq2, float* dlogp, void* stream);
/* is_ratio = exp(logp_new - old_logp)[:, 0] on [B][n] (msacl.py:392-394) and its backward
 * (d_logp_new: g * ratio in step 0, zero elsewhere). */
int mh_msacl_ratio0(const float* logp_new, const float* old_logp, int32_t B, int32_t n, float* ratio_out,
                    void* stream);
int mh_msacl_ratio0_backward(const float* ratio, const float* g_ratio, int32_t B, int32_t n, float* d_logp_new,
                             void* stream);
/* A policy step's whole objective (msacl.py:379-405) in one single-workgroup launch: mh_msacl_policy_loss
 * (loss_q, entropy over B*n), mh_msacl_ratio0 (ratio [B] from lp_new = log_prob(old act) under the
 * current policy), mh_msacl_ppo_clip (adv, loss_ppo, d_ratio) and loss_policy = -loss_q - loss_ppo,
 * bit-identical to those launches; its backward for a device upstream g of loss_policy gives
 * dq1, dq2, dlogp [B*n] and dlp_new [B*n] (step 0 only). */
int mh_msacl_policy_objective(const float* q1, const float* q2, const float* logp, const float* log_alpha,
                              const float* lp_new, const float* old_logp, const float* adv_raw, const double* stats,
                              double n_total, float clip_eps, int32_t B, int32_t n, float* loss_q, float* entropy,
                              float* ratio, float* adv, float* loss_ppo, float* d_ratio, float* loss_policy,
                              void* stream);
/* The policy step's objective (mh_msacl_policy_objective's outputs) AND its backward for the seed
 * g_loss = 1 — the one MSACL.model_update uses (msacl.py:405, loss_policy.backward()) — into
 * dq1, dq2, dlogp, dlp_new, plus the alpha gradient d/dlog_alpha of exp(log_alpha)(entropy -
 * target_entropy) (msacl.py:429-437) into alpha_grad (nullable), in one launch: the three
 * entry points' expressions, so their bits. */
int mh_msacl_policy_objective_step(const float* q1, const float* q2, const float* logp, const float* log_alpha,
                                   const float* lp_new, const float* old_logp, const float* adv_raw,
                                   const double* stats, double n_total, float clip_eps, int32_t B, int32_t n,
                                   float* loss_q, float* entropy, float* ratio, float* adv, float* loss_ppo,
                                   float* d_ratio, float* loss_policy, float* dq1, float* dq2, float* dlogp,
                                   float* dlp_new, float target_entropy, float* alpha_grad, void* stream);
int mh_msacl_policy_objective_backward(const float* q1, const float* q2, const float* log_alpha, const float* ratio,
                                       const float* d_ratio, const float* g_loss, int32_t B, int32_t n, float* dq1,
                                       float* dq2, float* dlogp, float* dlp_new, void* stream);
/* loss_policy = -loss_q - loss_ppo (msacl.py:401-405, device scalars) and neg_d_ratio = -d_ratio
 * (the is_ratio backward seed of loss_policy) in one launch. */
int mh_msacl_policy_combine(const float* loss_q, const float* loss_ppo, const float* d_ratio, int32_t B,
                            float* loss_policy, float* neg_d_ratio, void* stream);
/* grad = (entropy - target_entropy) * exp(log_alpha): the log_alpha gradient of the alpha loss
 * (msacl.py:429-437, replaces its 6-kernel autograd chain; the Adam step follows). */
int mh_msacl_alpha_grad(const float* log_alpha, const float* entropy, float target_entropy, float* grad,
                        void* stream);

/* ---- prioritized replay (new: the reference trainer expects buffer.update_batch(idx, prio),
 * RL/trainer/nstep_off_serial_trainer.py:93-95, but ships no prioritized buffer) ---- */
/* sum-tree over `capacity` leaves (tree: float64 [2*pow2]); leaf i priority p_i. */
int mh_per_update(double* tree, int64_t pow2, const int64_t* idx, const float* prio,
                  int64_t count, float alpha, float eps, double* max_prio, void* stream);
int mh_per_set_new(double* tree, int64_t pow2, const int64_t* cursor_before, const int64_t* cursor_after,
                   int64_t capacity, const double* max_prio, void* stream);
int mh_per_sample(const double* tree, int64_t pow2, const int64_t* cursor, uint64_t seed,
                  uint64_t counter, int64_t batch, float beta, int64_t* idx_out,
                  float* weight_out, void* stream);

/* ---- HIP-graph capture hygiene (the engine's own update capture, utils/dist.py cuda_graph) ----
 * For a stream `origin` that is capturing, and n other streams: unjoined[i] = 1 when stream i
 * takes part in the same capture and some of its captured work is NOT an ancestor of origin's
 * current capture frontier (a fork that was never joined back: ending the capture then would leave
 * a dangling branch), else 0. Host-only graph inspection (hipStreamGetCaptureInfo_v2 +
 * hipGraphNodeGetDependencies); MH_ESTATE when origin is not capturing. */
int mh_capture_unjoined(void* origin, void* const* streams, int32_t n, int32_t* unjoined);

const char* mh_last_error(void);
int mh_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MSACL_HIP_H */
