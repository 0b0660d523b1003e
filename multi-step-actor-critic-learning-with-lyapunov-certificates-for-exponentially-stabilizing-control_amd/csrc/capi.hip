// capi.hip — C ABI (include/msacl_hip.h): env handles, lockstep rollout, window store, gather.
#include <string>
#include <cmath>
#include <cstring>
#include <unordered_set>
#include <vector>

#include "msacl_hip.h"
#include "rollout.h"
#include "sample_fused.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define MH_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(MH_EHIP, std::string(#call) + ": " + hipGetErrorString(_e));        \
  } while (0)

template <class Env>
void fill_info(mh_env_info_t* o) {
  std::memset(o, 0, sizeof(*o));
  o->obs_dim = Env::D;
  o->act_dim = Env::A;
  o->state_dim = Env::S;
  o->xstate_dim = Env::XS;
  o->reset_dim = Env::RS;
  o->control_step = Env::K;
  o->max_step = mh::MAX_STEP;
  o->record_floats = mh::rec_floats(Env::D, Env::A);
  for (int i = 0; i < Env::D; ++i) {
    o->obs_low[i] = Env::obs_lo(i);
    o->obs_high[i] = Env::obs_hi(i);
  }
  for (int i = 0; i < Env::A; ++i) {
    o->act_low[i] = Env::act_lo(i);
    o->act_high[i] = Env::act_hi(i);
  }
}

}  // namespace

struct mh_env_s {
  int env_id = -1;
  int64_t E = 0;
  uint64_t seed = 0;
  mh_env_info_t info{};
  float* state = nullptr;
  double* xstate = nullptr;
  int32_t* steps = nullptr;
  double* tab = nullptr;
  int64_t* meta = nullptr;
  uint32_t* ctr = nullptr;
  // n-step
  int n = 0;
  int R = 0;  // ring slots per env (n, or more after mh_nstep_reserve)
  float reward_scale = 1.0f, cost_scale = 1.0f;
  int raw_log_std = 0;
  float log_std_lo = -20.0f, log_std_hi = 1.0f;
  const float* act_noise = nullptr;
  float* ring = nullptr;
  int32_t* ring_len = nullptr;
  int32_t* ring_pos = nullptr;
  int32_t* emit_rank = nullptr;
  int32_t* block_count = nullptr;
  int32_t* block_offset = nullptr;
  int32_t* emit_list = nullptr;     // [2][grid * BLK]: halves alternate between deferred steps
  // fused horizon sampler (mh_sample_horizon): per-(lockstep, wave) window counts / lists for up
  // to hcap locksteps (sized by mh_nstep_reserve: hcap = ring slots - n + 1)
  int hcap = 0;
  int32_t* h_count = nullptr;       // [hcap][ceil(E / 64)]
  int32_t* h_list = nullptr;        // [hcap][E]
  int64_t* h_scan = nullptr;        // the emission's bookkeeping (mh_nstep_reserve): aux [hcap + 2], then
                                    // int32 lockstep totals [hcap] + arrival count
  int32_t* h_cpre = nullptr;        // [hcap][cells per lockstep]: per-cell window prefixes, only when a
                                    // lockstep has more than FUSED_EMIT_SCAN_CELLS cells (k_emit_prefix)
  float* dbg_logits = nullptr;      // mh_sample_horizon_debug_logits: [H][E][2A] logits trace
  float* dbg_obs = nullptr;         //   and [H][E][D] pre-step observations
  uint32_t spin_limit = 0;          // mh_sample_horizon_set_spin_limit (0: the kernel's default)
  // the last mh_sample_horizon that emitted into a store: its horizon and the store's cursor
  // (mh_sample_horizon_emit replays exactly that emission; 0 / null once anything else stepped,
  // reset or re-attached the handle: its rings and window lists no longer describe that horizon)
  int emit_H = 0;
  const int64_t* emit_cursor = nullptr;
  // deferred emission (mh_rollout_step_deferred): the last step's windows are not yet emitted
  bool pending = false;
  int parity = 0;                   // half of block_count / emit_list the next step writes
  mh_window_store_t pstore{};       // store the pending windows go to
  // optional step trace (mh_rollout_set_trace): caller-owned device outputs of every rollout step
  float* tr_real = nullptr;
  float* tr_reward = nullptr;
  uint8_t* tr_term = nullptr;
  uint8_t* tr_trunc = nullptr;
  float* tr_state = nullptr;        // mh_rollout_set_trace_state: the pre-reset post-step state
  double* tr_xstate = nullptr;      //   (caller's [S][E] / [XS][E]), copied out of tr_buf (the
  void* tr_buf = nullptr;           //   kernel's one-pointer layout, mh::trace_xoff) after each step

  // optional per-kernel HIP-event timing of mh_rollout_step (bench.py's live roofline)
  bool timing = false;
  std::vector<hipEvent_t> ev_free;
  std::vector<hipEvent_t> ev_pending;  // groups of 4: before rollout / finalize / emit / end
  double t_ms[3] = {0.0, 0.0, 0.0};
  int64_t t_launches = 0;

  hipEvent_t take_event() {
    if (!ev_free.empty()) {
      hipEvent_t e = ev_free.back();
      ev_free.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  int grid() const { return (int)((E + mh::BLK - 1) / mh::BLK); }
  mh::StepArgs base_args() const {
    mh::StepArgs a;
    std::memset(&a, 0, sizeof(a));
    a.E = E;
    a.state = state;
    a.xstate = xstate;
    a.steps = steps;
    a.tab = tab;
    a.meta = meta;
    a.ctr = ctr;
    a.seed = seed;
    a.n = n;
    a.ring_slots = R;
    a.reward_scale = reward_scale;
    a.cost_scale = cost_scale;
    a.raw_log_std = raw_log_std;
    a.log_std_lo = log_std_lo;
    a.log_std_hi = log_std_hi;
    a.act_noise = act_noise;
    // TanhGaussDistribution's constant log-Jacobian term, torch.log((high - low) / 2).sum(-1)
    // (act_distribution_cls.py:51-55), once on the host in float32
    float ls = 0.0f;
    for (int i = 0; i < info.act_dim; ++i) ls = ls + logf((info.act_high[i] - info.act_low[i]) / 2.0f);
    a.log_half_sum = ls;
    return a;
  }
};

static void free_handle(mh_env_s* h) {
  if (!h) return;
  for (hipEvent_t e : h->ev_free) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->ev_pending) (void)hipEventDestroy(e);
  void* ptrs[] = {h->state, h->xstate, h->steps, h->tab, h->meta, h->ctr, h->ring, h->ring_len,
                  h->ring_pos, h->emit_rank, h->block_count, h->block_offset, h->emit_list, h->h_count,
                  h->h_list, h->h_scan, h->h_cpre, h->tr_buf};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  delete h;
}

extern "C" {

static int flush_pending(mh_env_t h, void* stream);

int mh_abi_version(void) { return MH_ABI_VERSION; }

const char* mh_last_error(void) { return g_err.c_str(); }

int mh_env_info(int32_t env_id, mh_env_info_t* out) {
  if (!out) return fail(MH_EINVAL, "mh_env_info: null out");
  switch (env_id) {
    case MH_ENV_VANDERPOL: fill_info<mh::VanderPol>(out); return MH_OK;
    case MH_ENV_PENDULUM: fill_info<mh::Pendulum>(out); return MH_OK;
    case MH_ENV_DUCTEDFAN: fill_info<mh::DuctedFan>(out); return MH_OK;
    case MH_ENV_TWOLINK: fill_info<mh::TwoLink>(out); return MH_OK;
    case MH_ENV_SINGLETRACKCAR: fill_info<mh::SingleTrackCar>(out); return MH_OK;
    case MH_ENV_QUADTRACKING: fill_info<mh::QuadTracking>(out); return MH_OK;
  }
  return fail(MH_EINVAL, "mh_env_info: unknown env id " + std::to_string(env_id));
}

int mh_env_create(int32_t env_id, int64_t num_envs, uint64_t seed, mh_env_t* out) {
  if (!out) return fail(MH_EINVAL, "mh_env_create: null out");
  *out = nullptr;
  if (num_envs <= 0 || num_envs > (int64_t)1 << 31)
    return fail(MH_EINVAL, "mh_env_create: num_envs out of range");
  mh_env_s* h = new mh_env_s();
  int rc = mh_env_info(env_id, &h->info);
  if (rc != MH_OK) {
    delete h;
    return rc;
  }
  // the step kernel addresses the SoA state through 32-bit buffer offsets
  if (num_envs * h->info.state_dim * (int64_t)sizeof(float) > (int64_t)INT32_MAX ||
      num_envs * h->info.xstate_dim * (int64_t)sizeof(double) > (int64_t)INT32_MAX) {
    delete h;
    return fail(MH_EINVAL, "mh_env_create: num_envs too large for this env (state bytes must fit in 31 bits)");
  }
  h->env_id = env_id;
  h->E = num_envs;
  h->seed = seed;
  const int64_t E = num_envs;
  hipError_t e = hipSuccess;
  e = hipMalloc(&h->state, sizeof(float) * E * h->info.state_dim);
  if (e == hipSuccess && h->info.xstate_dim > 0) e = hipMalloc(&h->xstate, sizeof(double) * E * h->info.xstate_dim);
  if (e == hipSuccess) e = hipMalloc(&h->steps, sizeof(int32_t) * E);
  if (e == hipSuccess) e = hipMalloc(&h->meta, sizeof(int64_t) * 8);
  if (e == hipSuccess) e = hipMemset(h->meta, 0, sizeof(int64_t) * 8);
  if (e == hipSuccess) e = hipMemset(h->steps, 0, sizeof(int32_t) * E);
  if (e == hipSuccess) e = hipMalloc(&h->ctr, sizeof(uint32_t) * E);
  if (e == hipSuccess) e = hipMemset(h->ctr, 0, sizeof(uint32_t) * E);
  if (e == hipSuccess) e = hipMemset(h->state, 0, sizeof(float) * E * h->info.state_dim);
  if (e == hipSuccess && env_id == MH_ENV_QUADTRACKING) {
    const int rows = mh::MAX_STEP + 1;
    double* host = new double[(size_t)rows * mh::QT_ROW];
    mh::quad_fill_table(host, rows);
    if (!mh::quad_row0_matches(host)) {  // resets use the constant row 0 (QuadTracking::row0)
      delete[] host;
      free_handle(h);
      return fail(MH_EHIP, "mh_env_create: desired-trajectory row 0 differs from QuadTracking::row0");
    }
    e = hipMalloc(&h->tab, sizeof(double) * rows * mh::QT_ROW);
    if (e == hipSuccess) e = hipMemcpy(h->tab, host, sizeof(double) * rows * mh::QT_ROW, hipMemcpyHostToDevice);
    delete[] host;
  }
  if (e != hipSuccess) {
    free_handle(h);
    return fail(e == hipErrorOutOfMemory ? MH_ENOMEM : MH_EHIP,
                std::string("mh_env_create: ") + hipGetErrorString(e));
  }
  *out = h;
  return MH_OK;
}

int mh_capture_unjoined(void* origin, void* const* streams, int32_t n, int32_t* unjoined) {
  if (n < 0 || (n > 0 && (!streams || !unjoined))) return fail(MH_EINVAL, "mh_capture_unjoined: bad arguments");
  hipStreamCaptureStatus so = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* d = nullptr;
  size_t nd = 0;
  MH_HIP(hipStreamGetCaptureInfo_v2((hipStream_t)origin, &so, &id, &g, &d, &nd));
  if (so != hipStreamCaptureStatusActive) return fail(MH_ESTATE, "mh_capture_unjoined: origin stream is not capturing");
  // every node the origin's next captured node would depend on, transitively
  std::vector<hipGraphNode_t> todo(d, d + nd);
  std::unordered_set<hipGraphNode_t> anc(todo.begin(), todo.end());
  std::vector<hipGraphNode_t> deps;
  while (!todo.empty()) {
    hipGraphNode_t v = todo.back();
    todo.pop_back();
    size_t k = 0;
    MH_HIP(hipGraphNodeGetDependencies(v, nullptr, &k));
    deps.assign(k, nullptr);
    if (k) MH_HIP(hipGraphNodeGetDependencies(v, deps.data(), &k));
    for (size_t j = 0; j < k; ++j)
      if (deps[j] && anc.insert(deps[j]).second) todo.push_back(deps[j]);
  }
  for (int32_t i = 0; i < n; ++i) {
    hipStreamCaptureStatus si = hipStreamCaptureStatusNone;
    unsigned long long sid = 0;
    const hipGraphNode_t* sd = nullptr;
    size_t snd = 0;
    unjoined[i] = 0;
    if (streams[i] == origin) continue;
    MH_HIP(hipStreamGetCaptureInfo_v2((hipStream_t)streams[i], &si, &sid, nullptr, &sd, &snd));
    if (si != hipStreamCaptureStatusActive || sid != id) continue;  // not in this capture
    for (size_t j = 0; j < snd; ++j)
      if (sd[j] && !anc.count(sd[j])) unjoined[i] = 1;
  }
  return MH_OK;
}

int mh_env_destroy(mh_env_t h) {
  free_handle(h);
  return MH_OK;
}

int mh_nstep_attach(mh_env_t h, int32_t n_step, float reward_scale, float cost_scale) {
  if (!h) return fail(MH_EINVAL, "mh_nstep_attach: null handle");
  if (n_step <= 0 || n_step > 4096) return fail(MH_EINVAL, "mh_nstep_attach: n_step out of range");
  if (int rc = flush_pending(h, nullptr)) return rc;
  if (h->ring) {
    (void)hipFree(h->ring); (void)hipFree(h->ring_len); (void)hipFree(h->ring_pos);
    (void)hipFree(h->emit_rank); (void)hipFree(h->block_count); (void)hipFree(h->block_offset);
    (void)hipFree(h->emit_list);
    h->emit_list = nullptr;
    h->ring = nullptr;
  }
  h->n = n_step;
  h->R = n_step;
  h->reward_scale = reward_scale;
  h->cost_scale = cost_scale;
  const int64_t E = h->E;
  const int F = h->info.record_floats;
  MH_HIP(hipMalloc(&h->ring, sizeof(float) * E * n_step * F));
  MH_HIP(hipMalloc(&h->ring_len, sizeof(int32_t) * E));
  MH_HIP(hipMalloc(&h->ring_pos, sizeof(int32_t) * E));
  MH_HIP(hipMalloc(&h->emit_rank, sizeof(int32_t) * E));
  MH_HIP(hipMalloc(&h->block_count, sizeof(int32_t) * 2 * h->grid()));
  MH_HIP(hipMalloc(&h->block_offset, sizeof(int32_t) * h->grid()));
  MH_HIP(hipMalloc(&h->emit_list, sizeof(int32_t) * 2 * (size_t)h->grid() * mh::BLK));
  h->pending = false;
  h->parity = 0;
  MH_HIP(hipMemset(h->ring_len, 0, sizeof(int32_t) * E));
  MH_HIP(hipMemset(h->ring_pos, 0, sizeof(int32_t) * E));
  MH_HIP(hipMemset(h->ring, 0, sizeof(float) * E * n_step * F));
  return MH_OK;
}

int mh_nstep_reserve(mh_env_t h, int32_t ring_slots) {
  if (!h) return fail(MH_EINVAL, "mh_nstep_reserve: null handle");
  if (!h->ring) return fail(MH_ESTATE, "mh_nstep_reserve: call mh_nstep_attach first");
  if (ring_slots < h->n || ring_slots > 8192) return fail(MH_EINVAL, "mh_nstep_reserve: ring_slots outside [n_step, 8192]");
  // the legacy per-env emission stages a whole ring in LDS: only grids the fused emission covers
  if (ring_slots != h->n && h->grid() > mh::EMIT_FUSED_MAX_NB)
    return fail(MH_EINVAL, "mh_nstep_reserve: more ring slots than n_step need num_envs <= 1M");
  // the fused horizon's window lists cover horizons up to ring_slots - n + 1 locksteps; they are
  // sized even when the ring keeps its size (ring_slots == n: horizons of one lockstep)
  const int hcap = ring_slots - h->n + 1;
  const bool new_ring = ring_slots != h->R;
  if (!new_ring && h->hcap == hcap && h->h_count) return MH_OK;
  if (int rc = flush_pending(h, nullptr)) return rc;
  MH_HIP(hipDeviceSynchronize());
  const int64_t E = h->E;
  const int F = h->info.record_floats;
  // every buffer is allocated before anything is swapped: on failure the handle is unchanged
  float* ring = nullptr;
  int32_t *cnt = nullptr, *lst = nullptr, *cpre = nullptr;
  int64_t* scan = nullptr;
  const int64_t cells = mh::fused_emit_cells_per_lockstep(E);  // emission cells per lockstep
  hipError_t e = hipSuccess;
  if (new_ring) e = hipMalloc(&ring, sizeof(float) * E * ring_slots * F);
  if (e == hipSuccess) e = hipMalloc(&cnt, sizeof(int32_t) * hcap * ((E + 63) / 64));
  if (e == hipSuccess) e = hipMalloc(&lst, sizeof(int32_t) * hcap * E);
  // the horizon's emission bookkeeping: int64 aux [hcap + 2] ({total, start cursor, lockstep
  // prefixes}), then int32 per-lockstep window totals [hcap] and the arrival count, zero between
  // horizons
  if (e == hipSuccess) e = hipMalloc(&scan, sizeof(int64_t) * (hcap + 2) + sizeof(int32_t) * (hcap + 2));
  if (e == hipSuccess) e = hipMemset(scan, 0, sizeof(int64_t) * (hcap + 2) + sizeof(int32_t) * (hcap + 2));
  if (e == hipSuccess && cells > mh::FUSED_EMIT_SCAN_CELLS) e = hipMalloc(&cpre, sizeof(int32_t) * hcap * cells);
  if (e == hipSuccess && new_ring) e = hipMemset(ring, 0, sizeof(float) * E * ring_slots * F);
  if (e != hipSuccess) {
    for (void* p : {(void*)ring, (void*)cnt, (void*)lst, (void*)scan, (void*)cpre})
      if (p) (void)hipFree(p);
    (void)hipGetLastError();
    return fail(e == hipErrorOutOfMemory ? MH_ENOMEM : MH_EHIP, std::string("mh_nstep_reserve: ") + hipGetErrorString(e));
  }
  (void)hipFree(h->h_count);
  (void)hipFree(h->h_list);
  (void)hipFree(h->h_scan);
  (void)hipFree(h->h_cpre);
  h->h_count = cnt;
  h->h_list = lst;
  h->h_scan = scan;
  h->h_cpre = cpre;
  h->hcap = hcap;
  if (new_ring) {  // every deque restarts empty over the new ring
    (void)hipFree(h->ring);
    h->ring = ring;
    h->R = ring_slots;
    MH_HIP(hipMemset(h->ring_len, 0, sizeof(int32_t) * E));
    MH_HIP(hipMemset(h->ring_pos, 0, sizeof(int32_t) * E));
  }
  return MH_OK;
}

int mh_sample_horizon(mh_env_t h, const float* packed_policy, int32_t obs_dim, int32_t n_out, float* obs,
                      int32_t horizon, const mh_window_store_t* store, const float* act_noise, float* act_out,
                      float* logp_out, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_sample_horizon: null handle");
  if (!h->ring) return fail(MH_ESTATE, "mh_sample_horizon: call mh_nstep_attach first");
  if (!packed_policy || !obs) return fail(MH_EINVAL, "mh_sample_horizon: null policy / obs");
  if (obs_dim != h->info.obs_dim || n_out != 2 * h->info.act_dim || obs_dim > 15)
    return fail(MH_EINVAL, "mh_sample_horizon: policy shape does not match the env (or obs_dim > 15)");
  if (horizon <= 0 || horizon > h->hcap || h->R < h->n + horizon - 1)
    return fail(MH_ESTATE, "mh_sample_horizon: horizon exceeds the reserved ring (mh_nstep_reserve(n + H - 1))");
  if (store && (store->capacity <= 0 || !store->cursor || !store->obs || !store->act || !store->rew ||
                !store->cost || !store->obs2 || !store->done || !store->logp))
    return fail(MH_EINVAL, "mh_sample_horizon: incomplete window store");
  if (int rc = flush_pending(h, stream)) return rc;
  mh::FusedArgs a;
  std::memset(&a, 0, sizeof(a));
  const mh::StepArgs b = h->base_args();
  a.E = h->E;
  a.state = h->state;
  a.xstate = h->xstate;
  a.steps = h->steps;
  a.tab = h->tab;
  a.ctr = h->ctr;
  a.seed = h->seed;
  a.obs = obs;
  a.P = packed_policy;
  a.K1 = obs_dim / 2 + 1;
  a.N3 = n_out;
  a.H = horizon;
  a.ring = h->ring;
  a.ring_len = h->ring_len;
  a.ring_pos = h->ring_pos;
  a.n = h->n;
  a.R = h->R;
  a.reward_scale = h->reward_scale;
  a.cost_scale = h->cost_scale;
  a.log_std_lo = h->log_std_lo;
  a.log_std_hi = h->log_std_hi;
  a.log_half_sum = b.log_half_sum;
  a.act_noise = act_noise;
  a.emit_count = h->h_count;
  a.emit_list = h->h_list;
  a.aux = h->h_scan;
  a.ts_total = reinterpret_cast<int32_t*>(h->h_scan + h->hcap + 2);
  a.arrive = reinterpret_cast<uint32_t*>(a.ts_total + h->hcap);
  a.cursor = store ? store->cursor : nullptr;
  a.capacity = store ? store->capacity : 0;
  a.act_out = act_out;
  a.logp_out = logp_out;
  a.err = h->meta + 7;  // meta[7]: the fused kernel's error word
  a.spin_limit = h->spin_limit ? h->spin_limit : mh::FUSED_SPIN_LIMIT;
  a.lgt_out = h->dbg_logits;
  a.obs_out = h->dbg_obs;
  mh::HorizonEmitArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.E = h->E;
  ea.H = horizon;
  ea.n = h->n;
  ea.R = h->R;
  ea.ring = h->ring;
  ea.emit_count = h->h_count;
  ea.emit_list = h->h_list;
  if (store) {
    ea.obs = store->obs;
    ea.act = store->act;
    ea.rew = store->rew;
    ea.cost = store->cost;
    ea.obs2 = store->obs2;
    ea.done = store->done;
    ea.logp = store->logp;
    ea.capacity = store->capacity;
    ea.aux = h->h_scan;
    ea.cell_pre = h->h_cpre;
  }
  MH_HIP(mh::launch_sample_fused(h->env_id, a, ea, (hipStream_t)stream));
  h->emit_H = store ? horizon : 0;
  h->emit_cursor = store ? store->cursor : nullptr;
  return MH_OK;
}

int mh_sample_horizon_emit(mh_env_t h, int32_t horizon, const mh_window_store_t* store, int64_t* windows_out,
                           void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_sample_horizon_emit: null handle");
  if (!h->ring || !h->h_scan) return fail(MH_ESTATE, "mh_sample_horizon_emit: no horizon has been sampled");
  if (horizon <= 0 || horizon > h->hcap) return fail(MH_EINVAL, "mh_sample_horizon_emit: bad horizon");
  if (!store || store->capacity <= 0 || !store->cursor || !store->obs || !store->act || !store->rew ||
      !store->cost || !store->obs2 || !store->done || !store->logp)
    return fail(MH_EINVAL, "mh_sample_horizon_emit: incomplete window store");
  // the aux prefixes and window lists describe exactly the last horizon sampled into a store
  if (h->emit_H == 0 || store->cursor != h->emit_cursor)
    return fail(MH_ESTATE, "mh_sample_horizon_emit: no horizon was sampled into this store since the handle last "
                           "stepped");
  if (horizon != h->emit_H)
    return fail(MH_EINVAL, "mh_sample_horizon_emit: horizon differs from the last sampled horizon");
  mh::HorizonEmitArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.E = h->E;
  ea.H = horizon;
  ea.n = h->n;
  ea.R = h->R;
  ea.ring = h->ring;
  ea.emit_count = h->h_count;
  ea.emit_list = h->h_list;
  ea.obs = store->obs;
  ea.act = store->act;
  ea.rew = store->rew;
  ea.cost = store->cost;
  ea.obs2 = store->obs2;
  ea.done = store->done;
  ea.logp = store->logp;
  ea.capacity = store->capacity;
  ea.aux = h->h_scan;
  ea.cell_pre = h->h_cpre;
  MH_HIP(mh::launch_emit_horizon(h->env_id, ea, (hipStream_t)stream));
  if (windows_out)  // the horizon's window count (header word 0, formed by the fused kernel)
    MH_HIP(hipMemcpyAsync(windows_out, h->h_scan, sizeof(int64_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MH_OK;
}

int mh_sample_horizon_debug_logits(mh_env_t h, float* logits_out, float* obs_out) {
  if (!h) return fail(MH_EINVAL, "mh_sample_horizon_debug_logits: null handle");
  if ((logits_out == nullptr) != (obs_out == nullptr)) return fail(MH_EINVAL, "mh_sample_horizon_debug_logits: both or neither");
  h->dbg_logits = logits_out;
  h->dbg_obs = obs_out;
  return MH_OK;
}

int mh_sample_horizon_windows(mh_env_t h, int64_t* out, void* stream) {
  if (!h || !out) return fail(MH_EINVAL, "mh_sample_horizon_windows: null handle / out");
  if (!h->h_scan) return fail(MH_ESTATE, "mh_sample_horizon_windows: no horizon has been sampled");
  MH_HIP(hipMemcpyAsync(out, h->h_scan, sizeof(int64_t), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MH_OK;
}

int mh_sample_horizon_errors(mh_env_t h, int64_t* out, void* stream) {
  if (!h || !out) return fail(MH_EINVAL, "mh_sample_horizon_errors: null argument");
  // hipMemcpyDefault: `out` may be device memory or pinned host memory (the sampler's capturable
  // per-horizon copy of the word, read without a device sync)
  MH_HIP(hipMemcpyAsync(out, h->meta + 7, sizeof(int64_t), hipMemcpyDefault, (hipStream_t)stream));
  return MH_OK;
}

int mh_sample_horizon_set_spin_limit(mh_env_t h, uint32_t limit) {
  if (!h) return fail(MH_EINVAL, "mh_sample_horizon_set_spin_limit: null handle");
  h->spin_limit = limit;
  return MH_OK;
}

int mh_env_get_counters(mh_env_t h, uint32_t* out, void* stream) {
  if (!h || !out) return fail(MH_EINVAL, "mh_env_get_counters: null argument");
  MH_HIP(hipMemcpyAsync(out, h->ctr, sizeof(uint32_t) * h->E, hipMemcpyDefault, (hipStream_t)stream));
  return MH_OK;
}

int mh_env_set_counters(mh_env_t h, const uint32_t* in, void* stream) {
  if (!h || !in) return fail(MH_EINVAL, "mh_env_set_counters: null argument");
  if (int rc = flush_pending(h, stream)) return rc;
  MH_HIP(hipMemcpyAsync(h->ctr, in, sizeof(uint32_t) * h->E, hipMemcpyDefault, (hipStream_t)stream));
  return MH_OK;
}

int mh_rng_draw(int32_t env_id, int32_t kind, uint64_t seed, const int64_t* env_idx, const uint32_t* ctr, int64_t n,
                float* out, void* stream) {
  if (kind != 0 && kind != 1) return fail(MH_EINVAL, "mh_rng_draw: kind must be 0 (action normals) or 1 (reset draw)");
  if (n < 0 || (n > 0 && (!env_idx || !ctr || !out))) return fail(MH_EINVAL, "mh_rng_draw: bad arguments");
  mh_env_info_t info;
  if (int rc = mh_env_info(env_id, &info)) return rc;
  MH_HIP(mh::launch_rng_draw(env_id, kind, seed, env_idx, ctr, n, out, (hipStream_t)stream));
  return MH_OK;
}

int mh_env_reset(mh_env_t h, const float* reset_states, float* obs, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_env_reset: null handle");
  if (int rc = flush_pending(h, stream)) return rc;
  hipStream_t st = (hipStream_t)stream;
  mh::StepArgs a = h->base_args();
  a.reset_in = reset_states;
  a.obs = obs;
  a.ring = h->ring;
  a.ring_len = h->ring_len;
  a.ring_pos = h->ring_pos;
  MH_HIP(mh::launch_reset(h->env_id, a, st));
  return MH_OK;
}

int mh_env_step(mh_env_t h, const float* act, const float* reset_states, float* next_obs,
                float* real_next_obs, float* reward, uint8_t* terminated, uint8_t* truncated,
                void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_env_step: null handle");
  if (int rc = flush_pending(h, stream)) return rc;
  if (!act) return fail(MH_EINVAL, "mh_env_step: null actions");
  hipStream_t st = (hipStream_t)stream;
  mh::StepArgs a = h->base_args();
  a.act_in = act;
  a.reset_in = reset_states;
  a.obs = next_obs;
  a.real_next_obs = real_next_obs;
  a.reward_out = reward;
  a.term_out = terminated;
  a.trunc_out = truncated;
  a.reward_scale = 1.0f;
  a.cost_scale = 1.0f;
  MH_HIP(mh::launch_rollout(h->env_id, a, st));
  return MH_OK;
}

int mh_env_get_state(mh_env_t h, float* state, double* xstate, int32_t* steps, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_env_get_state: null handle");
  hipStream_t st = (hipStream_t)stream;
  if (state) MH_HIP(mh::launch_transpose_f32(h->state, state, h->info.state_dim, h->E, true, st));
  if (xstate && h->info.xstate_dim > 0)
    MH_HIP(mh::launch_transpose_f64(h->xstate, xstate, h->info.xstate_dim, h->E, true, st));
  if (steps) MH_HIP(hipMemcpyAsync(steps, h->steps, sizeof(int32_t) * h->E, hipMemcpyDeviceToDevice, st));
  return MH_OK;
}

int mh_env_set_state(mh_env_t h, const float* state, const double* xstate, const int32_t* steps,
                     void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_env_set_state: null handle");
  if (int rc = flush_pending(h, stream)) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (state) MH_HIP(mh::launch_transpose_f32(state, h->state, h->info.state_dim, h->E, false, st));
  if (xstate && h->info.xstate_dim > 0)
    MH_HIP(mh::launch_transpose_f64(xstate, h->xstate, h->info.xstate_dim, h->E, false, st));
  if (steps) MH_HIP(hipMemcpyAsync(h->steps, steps, sizeof(int32_t) * h->E, hipMemcpyDeviceToDevice, st));
  return MH_OK;
}

static int rollout_impl(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                        const float* reset_states, float* obs, const mh_window_store_t* store,
                        float* act_out, float* logp_out, void* stream, bool defer) {
  if (!h->ring) return fail(MH_ESTATE, "mh_rollout_step: call mh_nstep_attach first");
  if (!obs) return fail(MH_EINVAL, "mh_rollout_step: null obs");
  if (!logits && !act_in) return fail(MH_EINVAL, "mh_rollout_step: need logits or act_in");
  if (store && (store->capacity <= 0 || !store->cursor || !store->obs || !store->act || !store->rew ||
                !store->cost || !store->obs2 || !store->done || !store->logp))
    return fail(MH_EINVAL, "mh_rollout_step: incomplete window store");
  hipStream_t st = (hipStream_t)stream;
  mh::StepArgs a = h->base_args();
  a.logits = logits;
  a.act_in = act_in;
  a.logp_in = logp_in;
  a.reset_in = reset_states;
  a.obs = obs;
  a.act_out = act_out;
  a.logp_out = logp_out;
  a.real_next_obs = h->tr_real;
  a.reward_out = h->tr_reward;
  a.term_out = h->tr_term;
  a.trunc_out = h->tr_trunc;
  a.trace_state = h->tr_state ? h->tr_buf : nullptr;
  a.ring = h->ring;
  a.ring_len = h->ring_len;
  a.ring_pos = h->ring_pos;
  a.emit_rank = h->emit_rank;
  a.block_count = h->block_count;
  // fused scan+emission when the per-block emitter prefix fits in LDS (E <= 1M envs)
  const bool fused = store && h->grid() <= mh::EMIT_FUSED_MAX_NB;
  if (fused) {
    a.emit_list = h->emit_list;
    a.cursor = store->cursor;
  }
  if (defer) {  // this step's counts / lists go to half `parity`; the pending ones are in the other
    const int p = h->parity;
    const size_t nb = (size_t)h->grid();
    a.defer = 1;
    a.parity = p;
    a.block_count = h->block_count + p * nb;
    a.emit_list = h->emit_list + p * nb * mh::BLK;
    if (h->pending) {
      a.prev_count = h->block_count + (1 - p) * nb;
      a.prev_list = h->emit_list + (1 - p) * nb * mh::BLK;
    }
    a.w_obs = store->obs;
    a.w_act = store->act;
    a.w_rew = store->rew;
    a.w_cost = store->cost;
    a.w_obs2 = store->obs2;
    a.w_done = store->done;
    a.w_logp = store->logp;
    a.capacity = store->capacity;
    a.cursor = store->cursor;
  }
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  if (h->timing)
    for (int i = 0; i < 4; ++i) ev[i] = h->take_event();
  if (ev[0]) MH_HIP(hipEventRecord(ev[0], st));
  MH_HIP(mh::launch_rollout(h->env_id, a, st));
  if (a.trace_state) {
    const int S = h->info.state_dim, XS = h->info.xstate_dim;
    MH_HIP(hipMemcpyAsync(h->tr_state, h->tr_buf, (size_t)S * h->E * 4, hipMemcpyDeviceToDevice, st));
    if (XS > 0)
      MH_HIP(hipMemcpyAsync(h->tr_xstate, (const char*)h->tr_buf + mh::trace_xoff(S, h->E), (size_t)XS * h->E * 8,
                            hipMemcpyDeviceToDevice, st));
  }
  if (ev[1]) MH_HIP(hipEventRecord(ev[1], st));
  if (defer) {  // the emission of this step's windows is left to the next step or the flush
    h->pending = true;
    h->pstore = *store;
    h->parity = 1 - h->parity;
    if (ev[3]) {
      MH_HIP(hipEventRecord(ev[2], st));
      MH_HIP(hipEventRecord(ev[3], st));
      for (int i = 0; i < 4; ++i) h->ev_pending.push_back(ev[i]);
    }
    return MH_OK;
  }
  if (store && !fused)
    MH_HIP(mh::launch_finalize(h->block_count, store ? h->grid() : 0, h->block_offset, h->meta,
                               store ? store->cursor : nullptr, store ? store->capacity : 1, st));
  if (ev[2]) MH_HIP(hipEventRecord(ev[2], st));
  if (fused) {
    mh::EmitArgs ea;
    std::memset(&ea, 0, sizeof(ea));
    ea.E = h->E;
    ea.ring = h->ring;
    ea.ring_pos = h->ring_pos;
    ea.meta = h->meta;
    ea.meta_rw = h->meta;
    ea.capacity = store->capacity;
    ea.n = h->n;
    ea.R = h->R;
    ea.F = h->info.record_floats;
    ea.D = h->info.obs_dim;
    ea.A = h->info.act_dim;
    ea.obs = store->obs;
    ea.act = store->act;
    ea.rew = store->rew;
    ea.cost = store->cost;
    ea.obs2 = store->obs2;
    ea.done = store->done;
    ea.logp = store->logp;
    ea.block_count = h->block_count;
    ea.emit_list = h->emit_list;
    ea.nb = h->grid();
    ea.cursor = store->cursor;
    MH_HIP(mh::launch_emit_fused(h->env_id, ea, st));
  } else if (store) {
    mh::EmitArgs ea;
    ea.E = h->E;
    ea.ring = h->ring;
    ea.ring_pos = h->ring_pos;
    ea.emit_rank = h->emit_rank;
    ea.block_offset = h->block_offset;
    ea.meta = h->meta;
    ea.capacity = store->capacity;
    ea.n = h->n;
    ea.R = h->R;
    ea.F = h->info.record_floats;
    ea.D = h->info.obs_dim;
    ea.A = h->info.act_dim;
    ea.obs = store->obs;
    ea.act = store->act;
    ea.rew = store->rew;
    ea.cost = store->cost;
    ea.obs2 = store->obs2;
    ea.done = store->done;
    ea.logp = store->logp;
    MH_HIP(mh::launch_emit(ea, st));
  }
  if (ev[3]) {
    MH_HIP(hipEventRecord(ev[3], st));
    for (int i = 0; i < 4; ++i) h->ev_pending.push_back(ev[i]);
  }
  return MH_OK;
}


// Emission of the pending deferred step's windows (k_emit_fused on the half of the double
// buffer that step wrote; the cursor snapshot in meta was written by its emitter waves).
static int flush_pending(mh_env_t h, void* stream) {
  h->emit_H = 0;  // every stepping / resetting entry point passes here: the last horizon is stale
  h->emit_cursor = nullptr;
  if (!h->pending) return MH_OK;
  h->pending = false;
  const int pp = 1 - h->parity;  // half written by the pending step
  const size_t nb = (size_t)h->grid();
  const mh_window_store_t* store = &h->pstore;
  mh::EmitArgs ea;
  std::memset(&ea, 0, sizeof(ea));
  ea.E = h->E;
  ea.ring = h->ring;
  ea.ring_pos = h->ring_pos;
  ea.meta = h->meta;
  ea.meta_rw = h->meta;
  ea.capacity = store->capacity;
  ea.n = h->n;
  ea.R = h->R;
  ea.F = h->info.record_floats;
  ea.D = h->info.obs_dim;
  ea.A = h->info.act_dim;
  ea.obs = store->obs;
  ea.act = store->act;
  ea.rew = store->rew;
  ea.cost = store->cost;
  ea.obs2 = store->obs2;
  ea.done = store->done;
  ea.logp = store->logp;
  ea.block_count = h->block_count + pp * nb;
  ea.emit_list = h->emit_list + pp * nb * mh::BLK;
  ea.nb = (int32_t)nb;
  ea.cursor = store->cursor;
  MH_HIP(mh::launch_emit_fused(h->env_id, ea, (hipStream_t)stream));
  return MH_OK;
}

int mh_rollout_step(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                    const float* reset_states, float* obs, const mh_window_store_t* store,
                    float* act_out, float* logp_out, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_step: null handle");
  if (int rc = flush_pending(h, stream)) return rc;
  return rollout_impl(h, logits, act_in, logp_in, reset_states, obs, store, act_out, logp_out, stream, false);
}

int mh_rollout_step_deferred(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                             const float* reset_states, float* obs, const mh_window_store_t* store,
                             float* act_out, float* logp_out, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_step_deferred: null handle");
  if (!store) return fail(MH_EINVAL, "mh_rollout_step_deferred: null store (use mh_rollout_step)");
  h->emit_H = 0;
  h->emit_cursor = nullptr;
  // deferral needs the fused emission (E <= 1M envs) and at most `capacity` windows per step
  const bool ok = h->grid() <= mh::EMIT_FUSED_MAX_NB && h->E <= store->capacity;
  const bool same = h->pending && std::memcmp(&h->pstore, store, sizeof(*store)) == 0;
  if (h->pending && (!ok || !same))
    if (int rc = flush_pending(h, stream)) return rc;
  return rollout_impl(h, logits, act_in, logp_in, reset_states, obs, store, act_out, logp_out, stream, ok);
}

int mh_rollout_flush(mh_env_t h, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_flush: null handle");
  return flush_pending(h, stream);
}

int mh_env_set_reward_cost_scale(mh_env_t h, float reward_scale, float cost_scale) {
  if (!h) return fail(MH_EINVAL, "mh_env_set_reward_cost_scale: null handle");
  h->reward_scale = reward_scale;
  h->cost_scale = cost_scale;
  return MH_OK;
}

int mh_env_set_action_noise(mh_env_t h, const float* noise) {
  if (!h) return fail(MH_EINVAL, "mh_env_set_action_noise: null handle");
  h->act_noise = noise;
  return MH_OK;
}

int mh_rollout_set_trace(mh_env_t h, float* real_next_obs, float* reward, uint8_t* terminated,
                         uint8_t* truncated) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_set_trace: null handle");
  h->tr_real = real_next_obs;
  h->tr_reward = reward;
  h->tr_term = terminated;
  h->tr_trunc = truncated;
  return MH_OK;
}

int mh_rollout_set_trace_state(mh_env_t h, float* state, double* xstate) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_set_trace_state: null handle");
  if (state && h->info.xstate_dim > 0 && !xstate) return fail(MH_EINVAL, "mh_rollout_set_trace_state: this env needs xstate");
  if (state && !h->tr_buf) {
    const int S = h->info.state_dim, XS = h->info.xstate_dim;
    MH_HIP(hipMalloc(&h->tr_buf, (size_t)mh::trace_xoff(S, h->E) + (size_t)XS * h->E * 8 + 16));
  }
  h->tr_state = state;
  h->tr_xstate = state ? xstate : nullptr;
  return MH_OK;
}

int mh_rollout_traj_step(mh_env_t h, const float* logits, const float* act_in, const float* logp_in,
                         const float* reset_states, float* obs, const mh_traj_store_t* traj, int32_t t,
                         float* act_out, float* logp_out, void* stream) {
  if (!h) return fail(MH_EINVAL, "mh_rollout_traj_step: null handle");
  if (int rc = flush_pending(h, stream)) return rc;
  if (!obs) return fail(MH_EINVAL, "mh_rollout_traj_step: null obs");
  if (!logits && !act_in) return fail(MH_EINVAL, "mh_rollout_traj_step: need logits or act_in");
  if (!traj || !traj->obs || !traj->act || !traj->rew || !traj->cost || !traj->obs2 || !traj->done ||
      !traj->logp)
    return fail(MH_EINVAL, "mh_rollout_traj_step: incomplete trajectory store");
  if (traj->horizon <= 0 || t < 0 || t >= traj->horizon)
    return fail(MH_EINVAL, "mh_rollout_traj_step: column t outside [0, horizon)");
  mh::StepArgs a = h->base_args();
  a.logits = logits;
  a.act_in = act_in;
  a.logp_in = logp_in;
  a.reset_in = reset_states;
  a.obs = obs;
  a.act_out = act_out;
  a.logp_out = logp_out;
  a.traj_obs = traj->obs;
  a.traj_act = traj->act;
  a.traj_rew = traj->rew;
  a.traj_cost = traj->cost;
  a.traj_obs2 = traj->obs2;
  a.traj_done = traj->done;
  a.traj_logp = traj->logp;
  a.traj_H = traj->horizon;
  a.traj_t = t;
  MH_HIP(mh::launch_rollout(h->env_id, a, (hipStream_t)stream));
  return MH_OK;
}

int mh_gae(const float* val, const float* val2, const float* rew, const uint8_t* done, int64_t num_envs,
           int32_t horizon, double gamma, double gae_lambda, float* adv, float* ret, void* stream) {
  if (!val || !val2 || !rew || !done || !adv || !ret) return fail(MH_EINVAL, "mh_gae: null array");
  if (num_envs < 0 || horizon < 0) return fail(MH_EINVAL, "mh_gae: negative size");
  MH_HIP(mh::launch_gae(val, val2, rew, done, num_envs, horizon, gamma, gae_lambda, adv, ret, (hipStream_t)stream));
  return MH_OK;
}

int mh_policy_packed_size(int32_t obs_dim, int64_t* floats_out) {
  if (!floats_out) return fail(MH_EINVAL, "mh_policy_packed_size: null out");
  if (obs_dim <= 0 || obs_dim > 16) return fail(MH_EINVAL, "mh_policy_packed_size: obs_dim must be in [1, 16]");
  *floats_out = mh::policy_packed_floats(obs_dim);
  return MH_OK;
}

int mh_policy_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                   const float* b3, int32_t obs_dim, int32_t hidden1, int32_t hidden2, int32_t out_dim,
                   float* packed, void* stream) {
  if (!W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !packed) return fail(MH_EINVAL, "mh_policy_pack: null pointer");
  if (hidden1 != 256 || hidden2 != 256) return fail(MH_EINVAL, "mh_policy_pack: hidden sizes must be 256 x 256");
  if (obs_dim <= 0 || obs_dim > 16) return fail(MH_EINVAL, "mh_policy_pack: obs_dim must be in [1, 16]");
  if (out_dim <= 0 || out_dim > 32) return fail(MH_EINVAL, "mh_policy_pack: out_dim must be in [1, 32]");
  if ((reinterpret_cast<uintptr_t>(W2) | reinterpret_cast<uintptr_t>(W3)) & 15)
    return fail(MH_EINVAL, "mh_policy_pack: W2 and W3 must be 16-byte aligned");
  MH_HIP(mh::launch_policy_pack(W1, b1, W2, b2, W3, b3, obs_dim, out_dim, packed, (hipStream_t)stream));
  return MH_OK;
}

int mh_policy_forward(const float* packed, const float* obs, int64_t num_envs, int32_t obs_dim, int32_t out_dim,
                      float* logits, void* stream) {
  if (!packed || !obs || !logits) return fail(MH_EINVAL, "mh_policy_forward: null pointer");
  if (obs_dim <= 0 || obs_dim > 16 || out_dim <= 0 || out_dim > 32 || num_envs < 0)
    return fail(MH_EINVAL, "mh_policy_forward: shape out of range");
  MH_HIP(mh::launch_policy_forward(packed, obs, num_envs, obs_dim, out_dim, logits, (hipStream_t)stream));
  return MH_OK;
}

int mh_act_grad_chunks(int64_t rows, int32_t* chunks_out) {
  if (!chunks_out || rows < 0) return fail(MH_EINVAL, "mh_act_grad_chunks: bad argument");
  *chunks_out = mh::act_grad_chunks(rows);
  return MH_OK;
}

int mh_act_grad_colsum(const float* dy, const float* y, int64_t rows, int32_t cols, int32_t act, float* g,
                       float* db, float* partial, uint32_t* tickets, void* stream) {
  if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_act_grad_colsum: act must be 0, 1 or 2");
  if (rows < 0 || cols <= 0) return fail(MH_EINVAL, "mh_act_grad_colsum: bad shape");
  if (rows > 0 && (!dy || (act != 0 && (!y || !g)) || !partial))
    return fail(MH_EINVAL, "mh_act_grad_colsum: null pointer");
  MH_HIP(mh::launch_act_grad_colsum(dy, y, rows, cols, act, act == 0 ? nullptr : g, db, partial, tickets,
                                    (hipStream_t)stream));
  return MH_OK;
}

int mh_policy_head(const float* raw, const float* eps, const float* obs, const float* old_act, const float* high,
                   const float* low, int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, float* xq,
                   float* new_logp, float* old_logp, void* stream) {
  if (rows < 0 || A <= 0 || A > 8 || D < 0) return fail(MH_EINVAL, "mh_policy_head: bad shape");
  if (!raw || ((eps || old_act) && (!high || !low)) || (eps && !xq && !new_logp) || (xq && !obs && D > 0))
    return fail(MH_EINVAL, "mh_policy_head: null pointer");
  MH_HIP(mh::launch_policy_head(raw, eps, obs, old_act, high, low, rows, A, D, log_std_lo, log_std_hi, xq, new_logp,
                                old_logp, (hipStream_t)stream));
  return MH_OK;
}

int mh_policy_head_sample(const float* raw, const float* obs, const float* old_act, const float* high, const float* low,
                          int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, uint64_t seed,
                          uint64_t* counter, float* eps_out, float* xq, float* new_logp, float* old_logp,
                          void* stream) {
  if (rows < 0 || A <= 0 || A > 8 || D < 0) return fail(MH_EINVAL, "mh_policy_head_sample: bad shape");
  if (!raw || !high || !low || !counter || !eps_out || (!xq && !new_logp) || (xq && !obs && D > 0))
    return fail(MH_EINVAL, "mh_policy_head_sample: null pointer");
  MH_HIP(mh::launch_policy_head(raw, nullptr, obs, old_act, high, low, rows, A, D, log_std_lo, log_std_hi, xq,
                                new_logp, old_logp, (hipStream_t)stream, seed,
                                reinterpret_cast<unsigned long long*>(counter), eps_out));
  return MH_OK;
}

int mh_policy_head_backward(const float* raw, const float* eps, const float* old_act, const float* high,
                            const float* low, const float* d_xq, const float* d_new_logp, const float* d_old_logp,
                            int64_t rows, int32_t A, int32_t D, float log_std_lo, float log_std_hi, float* d_raw,
                            void* stream) {
  if (rows < 0 || A <= 0 || A > 8 || D < 0) return fail(MH_EINVAL, "mh_policy_head_backward: bad shape");
  if (!raw || !d_raw || !high || !low || ((d_xq || d_new_logp) && !eps) || (d_old_logp && !old_act))
    return fail(MH_EINVAL, "mh_policy_head_backward: null pointer");
  MH_HIP(mh::launch_policy_head_bwd(raw, eps, old_act, high, low, d_xq, d_new_logp, d_old_logp, rows, A, D,
                                    log_std_lo, log_std_hi, d_raw, (hipStream_t)stream));
  return MH_OK;
}

int mh_dx_narrow(const float* dy, const float* y, int32_t act, const float* W, int64_t rows, int32_t n_out,
                 int32_t n_in, float* dx, void* stream) {
  if (act < 0 || act > 2 || rows < 0 || n_out <= 0 || n_out > 1024 || n_in <= 0 || n_in > 32)
    return fail(MH_EINVAL, "mh_dx_narrow: bad shape");
  if (rows > 0 && (!dy || !W || !dx || (act != 0 && !y))) return fail(MH_EINVAL, "mh_dx_narrow: null pointer");
  MH_HIP(mh::launch_dx_narrow(dy, y, act, W, rows, n_out, n_in, dx, (hipStream_t)stream));
  return MH_OK;
}

int mh_square_sum(const float* y, int64_t rows, int32_t cols, float* out, void* stream) {
  if (rows < 0 || cols <= 0 || (rows > 0 && (!y || !out))) return fail(MH_EINVAL, "mh_square_sum: bad argument");
  MH_HIP(mh::launch_square_sum(y, rows, cols, out, (hipStream_t)stream));
  return MH_OK;
}

int mh_square_sum_backward(const float* y, const float* g, int64_t rows, int32_t cols, float* dy, void* stream) {
  if (rows < 0 || cols <= 0 || (rows > 0 && (!y || !g || !dy)))
    return fail(MH_EINVAL, "mh_square_sum_backward: bad argument");
  MH_HIP(mh::launch_square_sum_bwd(y, g, rows, cols, dy, (hipStream_t)stream));
  return MH_OK;
}

int mh_head_backward_workspace(int64_t rows, int32_t n_out, int32_t n_in, int64_t* floats_out) {
  if (!floats_out || rows < 0 || n_out <= 0 || n_out > 16 || n_in <= 0)
    return fail(MH_EINVAL, "mh_head_backward_workspace: bad argument");
  *floats_out = mh::head_backward_workspace(rows, n_out, n_in);
  return MH_OK;
}

int mh_head_backward(const float* dy, const float* x, const float* W, int64_t rows, int32_t n_out, int32_t n_in,
                     float* dx, float* dw, float* db, float* workspace, void* stream) {
  if (rows <= 0 || n_out <= 0 || n_out > 16 || n_in <= 0) return fail(MH_EINVAL, "mh_head_backward: bad shape");
  // the kernel reads x on every path (dx-only calls included), so x is always required
  if (!dy || !x || (dx && !W) || ((dw || db) && !workspace) || (db && !dw))
    return fail(MH_EINVAL, "mh_head_backward: null pointer");
  MH_HIP(mh::launch_head_backward(dy, x, W, rows, n_out, n_in, dx, dw, db, workspace, (hipStream_t)stream));
  return MH_OK;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static int adam_multi_impl(const mh_adam_tensor_t* tensors, int32_t n, double lr, const double* lrs, double beta1,
                           double beta2, double eps, uint32_t* ticket, void* stream) {
  if (n < 0 || (n > 0 && (!tensors || !ticket))) return fail(MH_EINVAL, "mh_adam_multi: bad argument");
  for (int32_t base = 0; base < n; base += mh::ADAM_MAX_TENSORS) {
    mh::AdamList L{};
    L.n = n - base < mh::ADAM_MAX_TENSORS ? n - base : mh::ADAM_MAX_TENSORS;
    L.start[0] = 0;
    for (int k = 0; k < L.n; ++k) {
      const mh_adam_tensor_t& t = tensors[base + k];
      if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || !t.step || t.numel < 0)
        return fail(MH_EINVAL, "mh_adam_multi: null pointer or negative size in the tensor list");
      L.p[k] = t.param;
      L.g[k] = t.grad;
      L.m[k] = t.exp_avg;
      L.v[k] = t.exp_avg_sq;
      L.step[k] = t.step;
      // float4 units when every array of the tensor allows them, single elements otherwise
      const bool vec = t.numel % 4 == 0 && aligned16(t.param) && aligned16(t.grad) && aligned16(t.exp_avg) &&
                       aligned16(t.exp_avg_sq);
      L.vec[k] = vec ? 1 : 0;
      L.numel[k] = t.numel;
      L.start[k + 1] = L.start[k] + (vec ? t.numel / 4 : t.numel);
      L.lr[k] = lrs ? lrs[base + k] : lr;
    }
    MH_HIP(mh::launch_adam_multi(L, beta1, beta2, eps, ticket, (hipStream_t)stream));
  }
  return MH_OK;
}

int mh_adam_multi(const mh_adam_tensor_t* tensors, int32_t n, double lr, double beta1, double beta2, double eps,
                  uint32_t* ticket, void* stream) {
  return adam_multi_impl(tensors, n, lr, nullptr, beta1, beta2, eps, ticket, stream);
}

int mh_adam_multi_lr(const mh_adam_tensor_t* tensors, int32_t n, const double* lrs, double beta1, double beta2,
                     double eps, uint32_t* ticket, void* stream) {
  if (n > 0 && !lrs) return fail(MH_EINVAL, "mh_adam_multi_lr: null learning-rate list");
  return adam_multi_impl(tensors, n, 0.0, lrs, beta1, beta2, eps, ticket, stream);
}

int mh_polyak_multi(const mh_polyak_tensor_t* tensors, int32_t n, double polyak, void* stream) {
  if (n < 0 || (n > 0 && !tensors)) return fail(MH_EINVAL, "mh_polyak_multi: bad argument");
  for (int32_t base = 0; base < n; base += mh::ADAM_MAX_TENSORS) {
    mh::PolyakList L{};
    L.n = n - base < mh::ADAM_MAX_TENSORS ? n - base : mh::ADAM_MAX_TENSORS;
    for (int k = 0; k < L.n; ++k) {
      const mh_polyak_tensor_t& t = tensors[base + k];
      if (!t.target || !t.source || t.numel < 0)
        return fail(MH_EINVAL, "mh_polyak_multi: null pointer or negative size in the tensor list");
      L.t[k] = t.target;
      L.s[k] = t.source;
      const bool vec = t.numel % 4 == 0 && aligned16(t.target) && aligned16(t.source);
      L.vec[k] = vec ? 1 : 0;
      L.numel[k] = t.numel;
      L.start[k + 1] = L.start[k] + (vec ? t.numel / 4 : t.numel);
    }
    MH_HIP(mh::launch_polyak_multi(L, polyak, (hipStream_t)stream));
  }
  return MH_OK;
}

int mh_gemm_workspace(int64_t M, int64_t N, int64_t K, int64_t* workspace_floats) {
  if (!workspace_floats) return fail(MH_EINVAL, "mh_gemm_workspace: null out");
  if (M < 0 || N < 0 || K < 0) return fail(MH_EINVAL, "mh_gemm_workspace: negative size");
  *workspace_floats = (M > 0 && N > 0) ? mh::gemm_workspace_floats(M, N, K > 0 ? K : 1) : 0;
  return MH_OK;
}

int mh_gemm_f32(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a, int32_t trans_b, int32_t act,
                float* workspace, void* stream) {
  if (M < 0 || N < 0 || K < 0) return fail(MH_EINVAL, "mh_gemm_f32: negative size");
  if (M == 0 || N == 0) return MH_OK;
  if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_gemm_f32: act must be 0 (identity), 1 (relu) or 2 (tanh)");
  if (!C || (K > 0 && (!A || !B))) return fail(MH_EINVAL, "mh_gemm_f32: null operand");
  if (ldc < N || (K > 0 && (lda < (trans_a ? M : K) || ldb < (trans_b ? K : N))))
    return fail(MH_EINVAL, "mh_gemm_f32: leading dimension smaller than the matrix");
  if ((trans_a ? K : M) * lda * 4 >= ((int64_t)1 << 31) - 64 || (trans_b ? N : K) * ldb * 4 >= ((int64_t)1 << 31) - 64)
    return fail(MH_EINVAL, "mh_gemm_f32: each operand must be smaller than 2 GiB");
  if (mh::gemm_workspace_floats(M, N, K > 0 ? K : 1) > 0 && !workspace)
    return fail(MH_EINVAL, "mh_gemm_f32: this shape needs the workspace of mh_gemm_workspace");
  MH_HIP(mh::launch_gemm(A, B, bias, C, M, N, K, lda, ldb, ldc, trans_a != 0, trans_b != 0, act, workspace,
                         (hipStream_t)stream));
  return MH_OK;
}

int mh_linear_backward_plan(int64_t rows, int64_t n_out, int64_t n_in, int32_t need_dx, int32_t need_dw,
                            int32_t need_db, int32_t* supported, int64_t* workspace_floats) {
  if (!supported || !workspace_floats) return fail(MH_EINVAL, "mh_linear_backward_plan: null out");
  if (rows < 0 || n_out <= 0 || n_in <= 0) return fail(MH_EINVAL, "mh_linear_backward_plan: bad shape");
  int64_t ws = 0;
  *supported = mh::linear_backward_plan(rows, n_out, n_in, need_dx != 0, need_dw != 0, need_db != 0, &ws) ? 1 : 0;
  *workspace_floats = ws;
  return MH_OK;
}

int mh_linear_backward(const float* dy, const float* y, int32_t act, const float* x, const float* W, int64_t rows,
                       int64_t n_out, int64_t n_in, float* dx, float* dw, float* db, float* workspace, void* stream) {
  if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_linear_backward: act must be 0, 1 or 2");
  int64_t ws = 0;
  if (rows < 0 || n_out <= 0 || n_in <= 0 ||
      !mh::linear_backward_plan(rows, n_out, n_in, dx != nullptr, dw != nullptr, db != nullptr, &ws))
    return fail(MH_EINVAL, "mh_linear_backward: shape or request not supported (see mh_linear_backward_plan)");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!dy || (act != 0 && !y) || (dx && !W) || (dw && !x) || (ws > 0 && !workspace))
    return fail(MH_EINVAL, "mh_linear_backward: null pointer");
  if (!al16(dy) || !al16(y) || !al16(x) || !al16(W) || !al16(dx) || !al16(dw) || !al16(workspace))
    return fail(MH_EINVAL, "mh_linear_backward: every matrix must be 16-byte aligned");
  MH_HIP(mh::launch_linear_backward(dy, act != 0 ? y : nullptr, act, x, W, rows, n_out, n_in, dx, dw, db, workspace,
                                    (hipStream_t)stream));
  return MH_OK;
}

// ------------------------------------------------------------------ grouped layers (twin critics)
int mh_gemm_f32_grouped(const float* A, const float* B, const float* bias, float* C, int64_t M, int64_t N, int64_t K,
                        int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a, int32_t trans_b, int32_t act,
                        int32_t groups, int64_t stride_a, int64_t stride_b, int64_t stride_bias, int64_t stride_c,
                        void* stream) {
  if (M < 0 || N < 0 || K <= 0 || groups < 0) return fail(MH_EINVAL, "mh_gemm_f32_grouped: bad size");
  if (M == 0 || N == 0 || groups == 0) return MH_OK;
  if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_gemm_f32_grouped: act must be 0, 1 or 2");
  if (!A || !B || !C) return fail(MH_EINVAL, "mh_gemm_f32_grouped: null operand");
  if (stride_a < 0 || stride_b < 0 || stride_bias < 0 || stride_c < 0)
    return fail(MH_EINVAL, "mh_gemm_f32_grouped: negative group stride");
  if (ldc < N || lda < (trans_a ? M : K) || ldb < (trans_b ? K : N))
    return fail(MH_EINVAL, "mh_gemm_f32_grouped: leading dimension smaller than the matrix");
  const hipError_t e = mh::launch_gemm_grouped(A, B, bias, C, M, N, K, lda, ldb, ldc, trans_a != 0, trans_b != 0, act,
                                               groups, stride_a, stride_b, stride_bias, stride_c, (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(MH_EINVAL, "mh_gemm_f32_grouped: shape not supported (tall products and one-output products only)");
  MH_HIP(e);
  return MH_OK;
}

// mh_mlp3_forward's body; `second`: {x, W1, b1, W2, b2, W3, b3, y} of a second network set run
// as groups [groups, 2 groups) of the same launch (mh_mlp3_forward_pair), or null
static int mlp3_forward_impl(const float* x, int64_t rows, int32_t k1, int64_t ldx, const float* W1, const float* b1,
                             const float* W2, const float* b2, const float* W3, const float* b3, int32_t hidden,
                             int32_t n_out, int32_t act1, int32_t act2, int32_t act3, float* h1, float* h2,
                             int64_t ldh, float* y, int64_t ldy, int32_t groups, const int64_t* group_strides,
                             const void* const* second, void* stream) {
  if (rows < 0 || groups < 0) return fail(MH_EINVAL, "mh_mlp3_forward: bad size");
  if (rows == 0 || groups == 0) return MH_OK;
  if (!mh::mlp3_supported(rows, k1, hidden, n_out))
    return fail(MH_EINVAL, "mh_mlp3_forward: shape not supported (k1 <= 32, hidden 256, n_out <= 16 or a multiple of 64 <= 256)");
  for (int act : {act1, act2, act3})
    if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_mlp3_forward: act must be 0, 1 or 2");
  if (!x || !W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !y) return fail(MH_EINVAL, "mh_mlp3_forward: null operand");
  if (ldx < k1 || ldy < n_out || ((h1 || h2) && ldh < hidden))
    return fail(MH_EINVAL, "mh_mlp3_forward: leading dimension smaller than the matrix");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al16(W2) || !al16(W3) || !al16(h1) || !al16(h2) || (ldh & 3))
    return fail(MH_EINVAL, "mh_mlp3_forward: W2, W3, h1, h2 must be 16-byte aligned (ldh a multiple of 4)");
  if (groups > 1 && !group_strides) return fail(MH_EINVAL, "mh_mlp3_forward: grouped launch needs group_strides");
  mh::Mlp3Args a;
  std::memset(&a, 0, sizeof(a));
  a.x = x; a.M = rows; a.ldx = ldx; a.K1 = k1; a.H = hidden; a.N3 = n_out;
  a.act1 = act1; a.act2 = act2; a.act3 = act3;
  a.W1 = W1; a.b1 = b1; a.W2 = W2; a.b2 = b2; a.W3 = W3; a.b3 = b3;
  a.h1 = h1; a.h2 = h2; a.y = y; a.ldh = ldh; a.ldy = ldy;
  if (groups > 1) {
    const int64_t* g = group_strides;
    for (int i = 0; i < 9; ++i)
      if (g[i] < 0) return fail(MH_EINVAL, "mh_mlp3_forward: negative group stride");
    if ((g[3] & 3) || (g[5] & 3) || (g[7] & 3))
      return fail(MH_EINVAL, "mh_mlp3_forward: W2 / W3 / h group strides must keep 16-byte alignment");
    a.gs_x = g[0]; a.gs_W1 = g[1]; a.gs_b1 = g[2]; a.gs_W2 = g[3]; a.gs_b2 = g[4]; a.gs_W3 = g[5]; a.gs_b3 = g[6];
    a.gs_h = g[7]; a.gs_y = g[8];
  }
  if (second) {
    a.x_b = static_cast<const float*>(second[0]);
    a.W1_b = static_cast<const float*>(second[1]);
    a.b1_b = static_cast<const float*>(second[2]);
    a.W2_b = static_cast<const float*>(second[3]);
    a.b2_b = static_cast<const float*>(second[4]);
    a.W3_b = static_cast<const float*>(second[5]);
    a.b3_b = static_cast<const float*>(second[6]);
    a.y_b = static_cast<float*>(const_cast<void*>(second[7]));
    a.groups_b = groups;
  }
  MH_HIP(mh::launch_mlp3_forward(a, groups, (hipStream_t)stream));
  return MH_OK;
}

int mh_mlp3_forward(const float* x, int64_t rows, int32_t k1, int64_t ldx, const float* W1, const float* b1,
                    const float* W2, const float* b2, const float* W3, const float* b3, int32_t hidden, int32_t n_out,
                    int32_t act1, int32_t act2, int32_t act3, float* h1, float* h2, int64_t ldh, float* y, int64_t ldy,
                    int32_t groups, const int64_t* group_strides, void* stream) {
  return mlp3_forward_impl(x, rows, k1, ldx, W1, b1, W2, b2, W3, b3, hidden, n_out, act1, act2, act3, h1, h2, ldh,
                           y, ldy, groups, group_strides, nullptr, stream);
}

int mh_mlp3_forward_pair(const float* x, const float* x_b, int64_t rows, int32_t k1, int64_t ldx,
                         const float* const* params, const float* const* params_b, int32_t hidden, int32_t n_out,
                         int32_t act1, int32_t act2, int32_t act3, float* h1, float* h2, int64_t ldh, float* y,
                         float* y_b, int64_t ldy, int32_t groups, const int64_t* group_strides, void* stream) {
  if (!params || !params_b || !x_b || !y_b) return fail(MH_EINVAL, "mh_mlp3_forward_pair: null operand");
  for (int i = 0; i < 6; ++i)
    if (!params[i] || !params_b[i]) return fail(MH_EINVAL, "mh_mlp3_forward_pair: null operand");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al16(params_b[2]) || !al16(params_b[4]))
    return fail(MH_EINVAL, "mh_mlp3_forward_pair: W2, W3 must be 16-byte aligned");
  const void* second[8] = {x_b, params_b[0], params_b[1], params_b[2], params_b[3], params_b[4], params_b[5], y_b};
  return mlp3_forward_impl(x, rows, k1, ldx, params[0], params[1], params[2], params[3], params[4], params[5], hidden,
                           n_out, act1, act2, act3, h1, h2, ldh, y, ldy, groups, group_strides, second, stream);
}

// mh_mlp3_backward, and with dw3 set (n_out <= 16) the output layer's weight / bias gradients from
// the same launch's partials (Mlp3BwdArgs::pdw3) plus one k_head_finish launch
static int mlp3_backward_impl(const float* dy, int64_t ldy, const float* h1, const float* h2, int64_t ldh,
                              const float* W1, const float* W2, const float* W3, int64_t rows, int32_t k1,
                              int32_t hidden, int32_t n_out, int32_t act1, int32_t act2, float* g2, float* g1,
                              int64_t ldg, float* dx, int64_t ldx, int32_t groups, const int64_t* group_strides,
                              float* dw3, float* db3, int64_t gs_dw3, int64_t gs_db3, float* workspace,
                              void* stream) {
  if (rows < 0 || groups < 0) return fail(MH_EINVAL, "mh_mlp3_backward: bad size");
  if (rows == 0 || groups == 0) return MH_OK;
  if (!mh::mlp3_supported(rows, k1, hidden, n_out))
    return fail(MH_EINVAL, "mh_mlp3_backward: shape not supported (k1 <= 32, hidden 256, n_out <= 16 or a multiple of 64 <= 256)");
  if (act1 < 0 || act1 > 2 || act2 < 0 || act2 > 2) return fail(MH_EINVAL, "mh_mlp3_backward: act must be 0, 1 or 2");
  if (!dy || !h1 || !h2 || !W1 || !W2 || !W3) return fail(MH_EINVAL, "mh_mlp3_backward: null operand");
  if (ldy < n_out || ldh < hidden || ((g1 || g2) && ldg < hidden) || (dx && ldx < k1))
    return fail(MH_EINVAL, "mh_mlp3_backward: leading dimension smaller than the matrix");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al16(g1) || !al16(g2) || ((g1 || g2) && (ldg & 3)))
    return fail(MH_EINVAL, "mh_mlp3_backward: g1 / g2 must be 16-byte aligned (ldg a multiple of 4)");
  if (groups > 1 && !group_strides) return fail(MH_EINVAL, "mh_mlp3_backward: grouped launch needs group_strides");
  mh::Mlp3BwdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.dy = dy; a.ldy = ldy; a.h1 = h1; a.h2 = h2; a.ldh = ldh;
  a.W1 = W1; a.W2 = W2; a.W3 = W3; a.M = rows; a.K1 = k1; a.H = hidden; a.N3 = n_out;
  a.act1 = act1; a.act2 = act2; a.groups = groups;
  a.g2 = g2; a.g1 = g1; a.ldg = ldg; a.dx = dx; a.ldx = ldx;
  if (groups > 1) {
    const int64_t* g = group_strides;
    for (int i = 0; i < 6; ++i)
      if (g[i] < 0) return fail(MH_EINVAL, "mh_mlp3_backward: negative group stride");
    if (g[5] & 3) return fail(MH_EINVAL, "mh_mlp3_backward: the g group stride must keep 16-byte alignment");
    a.gs_dy = g[0]; a.gs_h = g[1]; a.gs_W1 = g[2]; a.gs_W2 = g[3]; a.gs_W3 = g[4]; a.gs_g = g[5];
  }
  const int64_t nblk = (rows + 15) / 16;
  if (dw3) {
    if (n_out > 16) return fail(MH_EINVAL, "mh_mlp3_backward_w3: the output-layer gradients need n_out <= 16");
    if (!workspace) return fail(MH_EINVAL, "mh_mlp3_backward_w3: null workspace");
    if (groups > 1 && (gs_dw3 < 0 || gs_db3 < 0)) return fail(MH_EINVAL, "mh_mlp3_backward_w3: negative group stride");
    a.pdw3 = workspace;
    a.pdb3 = db3 ? workspace + nblk * n_out * (int64_t)hidden : nullptr;
    a.s_part3 = nblk * n_out * (int64_t)(hidden + 1);
  } else if (db3) {
    return fail(MH_EINVAL, "mh_mlp3_backward_w3: db3 without dw3");
  }
  MH_HIP(mh::launch_mlp3_backward(a, (hipStream_t)stream));
  if (dw3)
    MH_HIP(mh::launch_head_finish(a.pdw3, a.pdb3, nblk, n_out, hidden, groups, a.s_part3, dw3, gs_dw3, db3, gs_db3,
                                  (hipStream_t)stream));
  return MH_OK;
}

int mh_mlp3_backward(const float* dy, int64_t ldy, const float* h1, const float* h2, int64_t ldh, const float* W1,
                     const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden, int32_t n_out,
                     int32_t act1, int32_t act2, float* g2, float* g1, int64_t ldg, float* dx, int64_t ldx,
                     int32_t groups, const int64_t* group_strides, void* stream) {
  return mlp3_backward_impl(dy, ldy, h1, h2, ldh, W1, W2, W3, rows, k1, hidden, n_out, act1, act2, g2, g1, ldg, dx,
                            ldx, groups, group_strides, nullptr, nullptr, 0, 0, nullptr, stream);
}

int mh_mlp3_set_row_tiles(int32_t mode) {
  if (mode < -1 || mode > 4) return fail(MH_EINVAL, "mh_mlp3_set_row_tiles: mode must be -1, 0 or 1..4");
  mh::mlp3_set_row_tiles(mode);
  return MH_OK;
}

int mh_mlp3_backward_w3_workspace(int64_t rows, int32_t hidden, int32_t n_out, int32_t groups, int64_t* floats_out) {
  if (rows < 0 || hidden <= 0 || n_out <= 0 || n_out > 16 || groups < 1 || !floats_out)
    return fail(MH_EINVAL, "mh_mlp3_backward_w3_workspace: bad argument");
  *floats_out = (rows + 15) / 16 * n_out * (int64_t)(hidden + 1) * groups;
  return MH_OK;
}

int mh_mlp3_backward_w3(const float* dy, int64_t ldy, const float* h1, const float* h2, int64_t ldh, const float* W1,
                        const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden, int32_t n_out,
                        int32_t act1, int32_t act2, float* g2, float* g1, int64_t ldg, float* dx, int64_t ldx,
                        int32_t groups, const int64_t* group_strides, float* dw3, float* db3, int64_t gs_dw3,
                        int64_t gs_db3, float* workspace, void* stream) {
  if (!dw3) return fail(MH_EINVAL, "mh_mlp3_backward_w3: null dw3");
  return mlp3_backward_impl(dy, ldy, h1, h2, ldh, W1, W2, W3, rows, k1, hidden, n_out, act1, act2, g2, g1, ldg, dx,
                            ldx, groups, group_strides, dw3, db3, gs_dw3, gs_db3, workspace, stream);
}

int mh_mlp3_forward_sqsum(const float* x, int64_t rows, int32_t k1, int64_t ldx, const float* const* params,
                          int32_t hidden, int32_t n_out, int32_t act1, int32_t act2, int32_t act3, float* h1,
                          float* h2, int64_t ldh, float* y, int64_t ldy, float* v, void* stream) {
  if (!params || !v) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: null operand");
  if (n_out % 64 != 0) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: n_out must be a multiple of 64");
  if (rows < 0) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: bad size");
  if (rows == 0) return MH_OK;
  if (!mh::mlp3_supported(rows, k1, hidden, n_out)) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: shape not supported");
  for (int act : {act1, act2, act3})
    if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: act must be 0, 1 or 2");
  for (int i = 0; i < 6; ++i)
    if (!params[i]) return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: null operand");
  if (!x || !y || ldx < k1 || ldy < n_out || ((h1 || h2) && ldh < hidden))
    return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: null operand or leading dimension too small");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al16(params[2]) || !al16(params[4]) || !al16(h1) || !al16(h2) || (ldh & 3))
    return fail(MH_EINVAL, "mh_mlp3_forward_sqsum: W2, W3, h1, h2 must be 16-byte aligned");
  mh::Mlp3Args a;
  std::memset(&a, 0, sizeof(a));
  a.x = x; a.M = rows; a.ldx = ldx; a.K1 = k1; a.H = hidden; a.N3 = n_out;
  a.act1 = act1; a.act2 = act2; a.act3 = act3;
  a.W1 = params[0]; a.b1 = params[1]; a.W2 = params[2]; a.b2 = params[3]; a.W3 = params[4]; a.b3 = params[5];
  a.h1 = h1; a.h2 = h2; a.y = y; a.ldh = ldh; a.ldy = ldy;
  a.sqsum = v;
  MH_HIP(mh::launch_mlp3_forward(a, 1, (hipStream_t)stream));
  return MH_OK;
}

int mh_mlp3_backward_sqsum(const float* y, int64_t ldy, const float* dv, const float* h1, const float* h2, int64_t ldh,
                           const float* W1, const float* W2, const float* W3, int64_t rows, int32_t k1, int32_t hidden,
                           int32_t n_out, int32_t act1, int32_t act2, float* g3, float* g2, float* g1, int64_t ldg,
                           float* dx, int64_t ldx, void* stream) {
  if (!dv || !g3) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: null operand");
  if (n_out % 64 != 0) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: n_out must be a multiple of 64");
  if (rows < 0) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: bad size");
  if (rows == 0) return MH_OK;
  if (!mh::mlp3_supported(rows, k1, hidden, n_out)) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: shape not supported");
  if (act1 < 0 || act1 > 2 || act2 < 0 || act2 > 2) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: act must be 0, 1 or 2");
  if (!y || !h1 || !h2 || !W1 || !W2 || !W3) return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: null operand");
  if (ldy < n_out || ldh < hidden || ((g1 || g2) && ldg < hidden) || (dx && ldx < k1))
    return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: leading dimension smaller than the matrix");
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!al16(g1) || !al16(g2) || ((g1 || g2) && (ldg & 3)))
    return fail(MH_EINVAL, "mh_mlp3_backward_sqsum: g1 / g2 must be 16-byte aligned (ldg a multiple of 4)");
  mh::Mlp3BwdArgs a;
  std::memset(&a, 0, sizeof(a));
  a.dy = y; a.ldy = ldy; a.h1 = h1; a.h2 = h2; a.ldh = ldh;
  a.W1 = W1; a.W2 = W2; a.W3 = W3; a.M = rows; a.K1 = k1; a.H = hidden; a.N3 = n_out;
  a.act1 = act1; a.act2 = act2; a.groups = 1;
  a.g2 = g2; a.g1 = g1; a.ldg = ldg; a.dx = dx; a.ldx = ldx;
  a.sq_dv = dv; a.g3 = g3;
  MH_HIP(mh::launch_mlp3_backward(a, (hipStream_t)stream));
  return MH_OK;
}

static bool wgrad_specs(const mh_wgrad_t* products, int32_t n, std::vector<mh::WgradSpec>& v) {
  if (!products || n < 1 || n > 6) return false;
  v.resize(n);
  for (int i = 0; i < n; ++i) {
    const mh_wgrad_t& p = products[i];
    if (!p.g || !p.x || !p.dw || p.n_out <= 0 || p.n_in <= 0 || p.ld_g < p.n_out || p.ld_x < p.n_in) return false;
    v[i] = mh::WgradSpec{p.g, p.ld_g, p.x, p.ld_x, p.n_out, p.n_in, p.dw, p.db};
  }
  return true;
}

int mh_weight_grads_workspace(const mh_wgrad_t* products, int32_t n, int64_t rows, int64_t* floats_out) {
  if (!floats_out) return fail(MH_EINVAL, "mh_weight_grads_workspace: null out");
  std::vector<mh::WgradSpec> v;
  if (!wgrad_specs(products, n, v) || !mh::weight_grads_plan(v.data(), n, rows, floats_out))
    return fail(MH_EINVAL, "mh_weight_grads_workspace: products not supported (see msacl_hip.h)");
  return MH_OK;
}

int mh_weight_grads(const mh_wgrad_t* products, int32_t n, int64_t rows, float* workspace, void* stream) {
  std::vector<mh::WgradSpec> v;
  int64_t need = 0;
  if (!wgrad_specs(products, n, v) || !mh::weight_grads_plan(v.data(), n, rows, &need))
    return fail(MH_EINVAL, "mh_weight_grads: products not supported (see msacl_hip.h)");
  if (need > 0 && !workspace) return fail(MH_EINVAL, "mh_weight_grads: workspace required");
  MH_HIP(mh::launch_weight_grads(v.data(), n, rows, workspace, (hipStream_t)stream));
  return MH_OK;
}

int mh_linear_backward_grouped(const float* dy, const float* y, int32_t act, const float* x, const float* W,
                               int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x, int64_t ld_dx,
                               int32_t groups, int64_t stride_dy, int64_t stride_x, int64_t stride_w,
                               int64_t stride_dx, int64_t stride_dw, int64_t stride_db, float* dx, float* dw,
                               float* db, float* workspace, void* stream) {
  if (act < 0 || act > 2) return fail(MH_EINVAL, "mh_linear_backward_grouped: act must be 0, 1 or 2");
  int64_t ws = 0;
  if (rows < 0 || n_out <= 0 || n_in <= 0 || groups < 0 ||
      !mh::linear_backward_plan(rows, n_out, n_in, dx != nullptr, dw != nullptr, db != nullptr, &ws))
    return fail(MH_EINVAL, "mh_linear_backward_grouped: shape or request not supported (see mh_linear_backward_plan)");
  if (groups == 0) return MH_OK;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!dy || (act != 0 && !y) || (dx && !W) || (dw && !x) || (ws > 0 && !workspace))
    return fail(MH_EINVAL, "mh_linear_backward_grouped: null pointer");
  if (!al16(dy) || !al16(y) || !al16(x) || !al16(W) || !al16(dx) || !al16(dw) || !al16(workspace))
    return fail(MH_EINVAL, "mh_linear_backward_grouped: every matrix must be 16-byte aligned");
  if (ld_dy < n_out || (dw && ld_x < n_in) || (dx && ld_dx < n_in))
    return fail(MH_EINVAL, "mh_linear_backward_grouped: leading dimension smaller than the matrix");
  const hipError_t e = mh::launch_linear_backward_grouped(
      dy, act != 0 ? y : nullptr, act, x, W, rows, n_out, n_in, ld_dy, ld_x, ld_dx, groups, stride_dy, stride_x,
      stride_w, stride_dx, stride_dw, stride_db, dx, dw, db, workspace, (hipStream_t)stream);
  if (e == hipErrorInvalidValue)
    return fail(MH_EINVAL, "mh_linear_backward_grouped: strides / leading dimensions must keep 16-byte alignment");
  MH_HIP(e);
  return MH_OK;
}

int mh_head_backward_grouped(const float* dy, const float* x, const float* W, int64_t rows, int32_t n_out,
                             int32_t n_in, int64_t ld_x, int64_t ld_dx, int32_t groups, int64_t stride_dy,
                             int64_t stride_x, int64_t stride_w, int64_t stride_dx, int64_t stride_dw,
                             int64_t stride_db, float* dx, float* dw, float* db, float* workspace, void* stream) {
  if (rows <= 0 || n_out <= 0 || n_out > 16 || n_in <= 0 || groups < 0 || ld_x < n_in || (dx && ld_dx < n_in))
    return fail(MH_EINVAL, "mh_head_backward_grouped: bad shape");
  if (groups == 0) return MH_OK;
  if (!dy || !x || (dx && !W) || ((dw || db) && !workspace) || (db && !dw))
    return fail(MH_EINVAL, "mh_head_backward_grouped: null pointer");
  MH_HIP(mh::launch_head_backward_grouped(dy, x, W, rows, n_out, n_in, ld_x, ld_dx, groups, stride_dy, stride_x,
                                          stride_w, stride_dx, stride_dw, stride_db, dx, dw, db, workspace,
                                          (hipStream_t)stream));
  return MH_OK;
}

int mh_stocha_head(const float* raw, int64_t rows, int32_t act_dim, float min_log_std, float max_log_std, float* out,
                   void* stream) {
  if (rows < 0 || act_dim <= 0) return fail(MH_EINVAL, "mh_stocha_head: bad shape");
  if (rows > 0 && (!raw || !out)) return fail(MH_EINVAL, "mh_stocha_head: null pointer");
  MH_HIP(mh::launch_stocha_head(raw, rows, act_dim, min_log_std, max_log_std, out, (hipStream_t)stream));
  return MH_OK;
}

int mh_stocha_head_backward(const float* raw, const float* out, const float* d_out, int64_t rows, int32_t act_dim,
                            float min_log_std, float max_log_std, float* d_raw, void* stream) {
  if (rows < 0 || act_dim <= 0) return fail(MH_EINVAL, "mh_stocha_head_backward: bad shape");
  if (rows > 0 && (!raw || !out || !d_out || !d_raw)) return fail(MH_EINVAL, "mh_stocha_head_backward: null pointer");
  MH_HIP(mh::launch_stocha_head_bwd(raw, out, d_out, rows, act_dim, min_log_std, max_log_std, d_raw,
                                    (hipStream_t)stream));
  return MH_OK;
}

#define MH_TG_CHECK(name)                                                                           \
  if (rows < 0 || act_dim <= 0 || act_dim > 8) return fail(MH_EINVAL, name ": act_dim must be in [1, 8]"); \
  if (rows == 0) return MH_OK;                                                                     \
  if (!logits || !high || !low) return fail(MH_EINVAL, name ": null pointer")

int mh_tanh_gauss_rsample(const float* logits, const float* eps, const float* high, const float* low, int64_t rows,
                          int32_t act_dim, float* act, float* logp, void* stream) {
  MH_TG_CHECK("mh_tanh_gauss_rsample");
  if (!eps || !act || !logp) return fail(MH_EINVAL, "mh_tanh_gauss_rsample: null pointer");
  MH_HIP(mh::launch_tg_rsample(logits, eps, high, low, rows, act_dim, act, logp, (hipStream_t)stream));
  return MH_OK;
}

int mh_tanh_gauss_rsample_backward(const float* logits, const float* eps, const float* high, const float* low,
                                   const float* d_act, const float* d_logp, int64_t rows, int32_t act_dim,
                                   float* d_logits, void* stream) {
  MH_TG_CHECK("mh_tanh_gauss_rsample_backward");
  if (!eps || !d_logits) return fail(MH_EINVAL, "mh_tanh_gauss_rsample_backward: null pointer");
  MH_HIP(mh::launch_tg_rsample_bwd(logits, eps, high, low, d_act, d_logp, rows, act_dim, d_logits,
                                   (hipStream_t)stream));
  return MH_OK;
}

int mh_tanh_gauss_log_prob(const float* logits, const float* act, const float* high, const float* low, int64_t rows,
                           int32_t act_dim, float* logp, void* stream) {
  MH_TG_CHECK("mh_tanh_gauss_log_prob");
  if (!act || !logp) return fail(MH_EINVAL, "mh_tanh_gauss_log_prob: null pointer");
  MH_HIP(mh::launch_tg_log_prob(logits, act, high, low, rows, act_dim, logp, (hipStream_t)stream));
  return MH_OK;
}

int mh_tanh_gauss_log_prob_backward(const float* logits, const float* act, const float* high, const float* low,
                                    const float* d_logp, int64_t rows, int32_t act_dim, float* d_logits,
                                    void* stream) {
  MH_TG_CHECK("mh_tanh_gauss_log_prob_backward");
  if (!act || !d_logp || !d_logits) return fail(MH_EINVAL, "mh_tanh_gauss_log_prob_backward: null pointer");
  MH_HIP(mh::launch_tg_log_prob_bwd(logits, act, high, low, d_logp, rows, act_dim, d_logits, (hipStream_t)stream));
  return MH_OK;
}

int mh_nstep_set_log_std_clamp(mh_env_t h, int32_t enable, float lo, float hi) {
  if (!h) return fail(MH_EINVAL, "mh_nstep_set_log_std_clamp: null handle");
  if (enable && !(lo <= hi)) return fail(MH_EINVAL, "mh_nstep_set_log_std_clamp: lo > hi");
  h->raw_log_std = enable != 0;
  h->log_std_lo = lo;
  h->log_std_hi = hi;
  return MH_OK;
}

int mh_env_set_timing(mh_env_t h, int32_t enable) {
  if (!h) return fail(MH_EINVAL, "mh_env_set_timing: null handle");
  h->timing = enable != 0;
  return MH_OK;
}

int mh_env_read_timing(mh_env_t h, double* ms_out, int64_t* launches_out, int32_t reset) {
  if (!h || !ms_out || !launches_out) return fail(MH_EINVAL, "mh_env_read_timing: null arg");
  for (size_t g = 0; g + 3 < h->ev_pending.size(); g += 4) {
    hipEvent_t* e = &h->ev_pending[g];
    MH_HIP(hipEventSynchronize(e[3]));
    for (int k = 0; k < 3; ++k) {
      float ms = 0.0f;
      MH_HIP(hipEventElapsedTime(&ms, e[k], e[k + 1]));
      h->t_ms[k] += ms;
    }
    h->t_launches += 1;
    for (int k = 0; k < 4; ++k) h->ev_free.push_back(e[k]);
  }
  h->ev_pending.clear();
  for (int k = 0; k < 3; ++k) ms_out[k] = h->t_ms[k];
  *launches_out = h->t_launches;
  if (reset) {
    h->t_ms[0] = h->t_ms[1] = h->t_ms[2] = 0.0;
    h->t_launches = 0;
  }
  return MH_OK;
}

int mh_replay_gather(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim, int32_t act_dim,
                     const int64_t* idx, int64_t batch, float* out_obs, float* out_act, float* out_rew,
                     float* out_cost, float* out_obs2, float* out_done, float* out_logp, void* stream) {
  if (!store || !idx) return fail(MH_EINVAL, "mh_replay_gather: null store/idx");
  mh::GatherArgs g;
  g.idx = idx;
  g.batch = batch;
  g.n = n_step;
  g.D = obs_dim;
  g.A = act_dim;
  g.s_obs = store->obs; g.s_act = store->act; g.s_rew = store->rew; g.s_cost = store->cost;
  g.s_obs2 = store->obs2; g.s_done = store->done; g.s_logp = store->logp;
  g.o_obs = out_obs; g.o_act = out_act; g.o_rew = out_rew; g.o_cost = out_cost;
  g.o_obs2 = out_obs2; g.o_done = out_done; g.o_logp = out_logp;
  g.o_obs_act = nullptr; g.o_v_in = nullptr;
  MH_HIP(mh::launch_gather(g, (hipStream_t)stream));
  return MH_OK;
}

int mh_replay_gather_joint(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim, int32_t act_dim,
                           const int64_t* idx, int64_t batch, float* out_obs, float* out_act, float* out_rew,
                           float* out_cost, float* out_obs2, float* out_done, float* out_logp, float* out_obs_act,
                           float* out_v_in, void* stream) {
  if (!store || !idx) return fail(MH_EINVAL, "mh_replay_gather_joint: null store/idx");
  mh::GatherArgs g;
  g.idx = idx;
  g.batch = batch;
  g.n = n_step;
  g.D = obs_dim;
  g.A = act_dim;
  g.s_obs = store->obs; g.s_act = store->act; g.s_rew = store->rew; g.s_cost = store->cost;
  g.s_obs2 = store->obs2; g.s_done = store->done; g.s_logp = store->logp;
  g.o_obs = out_obs; g.o_act = out_act; g.o_rew = out_rew; g.o_cost = out_cost;
  g.o_obs2 = out_obs2; g.o_done = out_done; g.o_logp = out_logp;
  g.o_obs_act = out_obs_act; g.o_v_in = out_v_in;
  MH_HIP(mh::launch_gather(g, (hipStream_t)stream));
  return MH_OK;
}

int mh_replay_sample_indices(const mh_window_store_t* store, uint64_t seed, uint64_t counter,
                             int64_t batch, int64_t* idx_out, void* stream) {
  if (!store || !store->cursor || !idx_out) return fail(MH_EINVAL, "mh_replay_sample_indices: null arg");
  MH_HIP(mh::launch_sample_idx(store->cursor, seed, counter, batch, idx_out, (hipStream_t)stream));
  return MH_OK;
}

int mh_replay_sample_indices_dev(const mh_window_store_t* store, uint64_t seed, int64_t* draw_state, int64_t batch,
                                 int64_t* idx_out, void* stream) {
  if (!store || !store->cursor || !draw_state || !idx_out)
    return fail(MH_EINVAL, "mh_replay_sample_indices_dev: null arg");
  MH_HIP(mh::launch_sample_idx_dev(store->cursor, seed, draw_state, batch, idx_out, (hipStream_t)stream));
  return MH_OK;
}

int mh_replay_draw_gather(const mh_window_store_t* store, int32_t n_step, int32_t obs_dim, int32_t act_dim,
                          uint64_t seed, int64_t* draw_state, int64_t batch, int64_t* idx_out, float* out_obs,
                          float* out_act, float* out_rew, float* out_cost, float* out_obs2, float* out_done,
                          float* out_logp, float* out_obs_act, float* out_v_in, void* stream) {
  if (!store || !store->cursor || !draw_state) return fail(MH_EINVAL, "mh_replay_draw_gather: null store/state");
  if (batch <= 0) return fail(MH_EINVAL, "mh_replay_draw_gather: batch must be positive");
  mh::GatherArgs g;
  g.idx = nullptr;
  g.batch = batch;
  g.n = n_step;
  g.D = obs_dim;
  g.A = act_dim;
  g.s_obs = store->obs; g.s_act = store->act; g.s_rew = store->rew; g.s_cost = store->cost;
  g.s_obs2 = store->obs2; g.s_done = store->done; g.s_logp = store->logp;
  g.o_obs = out_obs; g.o_act = out_act; g.o_rew = out_rew; g.o_cost = out_cost;
  g.o_obs2 = out_obs2; g.o_done = out_done; g.o_logp = out_logp;
  g.o_obs_act = out_obs_act; g.o_v_in = out_v_in;
  g.cursor = store->cursor;
  g.seed = seed;
  g.draw = draw_state;
  g.idx_out = idx_out;
  MH_HIP(mh::launch_gather(g, (hipStream_t)stream));
  return MH_OK;
}

}  // extern "C"
