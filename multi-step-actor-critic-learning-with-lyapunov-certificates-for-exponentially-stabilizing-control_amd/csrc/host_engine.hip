// host_engine.hip — the engine's CPU build (libmsacl_host.so): BASELINE.json config 1, "VanderPol,
// 1 env, MSACL off_serial_trainer on CPU reference sampler (plumbing, no GPU)".
//
// The same env math as the gfx950 kernels (env_math.h, compiled here for the host) and the same
// reset distributions and Philox streams (reset_draw.h), behind a C ABI that mirrors the device
// library's (include/msacl_host.h): a batch of envs stepped one after another on the calling CPU
// thread with the SyncVectorEnv contract (step, termination at the observation box, truncation at
// step 1000, autoreset with final_observation), and the MSACL target / certificate math of
// msacl_kernels.hip as host loops (batch sums in float64, in row order). It is an explicit CPU
// deployment of the engine (selected with device="cpu"), never a fallback of the GPU path: the HIP
// library raises when it is missing on a GPU box.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "msacl_host.h"
#include "reset_draw.h"

#pragma clang fp contract(off)

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct HostEnv {
  int env_id = 0;
  int64_t E = 0;
  uint64_t seed = 0;
  int S = 0, XS = 0, D = 0, A = 0, RS = 0;
  std::vector<float> state;      // [E][S]
  std::vector<double> xstate;    // [E][XS]
  std::vector<int32_t> steps;    // [E]
  std::vector<uint32_t> ctr;     // [E] Philox counters (as the device's per-env counters)
  std::vector<double> tab;       // QuadTracking desired-trajectory table
};

template <class Env>
void dims(HostEnv& h) {
  h.S = Env::S;
  h.XS = Env::XS;
  h.D = Env::D;
  h.A = Env::A;
  h.RS = Env::RS;
}

template <class Env>
void reset_one(HostEnv& h, int64_t e, const float* rs_in, float* obs) {
  float rs[Env::RS];
  if (rs_in) {
    for (int i = 0; i < Env::RS; ++i) rs[i] = rs_in[i];
  } else {
    mh::ResetDraw<Env>::draw(mh::make_rng(h.seed, (uint64_t)e, h.ctr[e]), rs);
    h.ctr[e] += 1u;
  }
  double xs[Env::XS > 0 ? Env::XS : 1];
  Env::reset_from(rs, &h.state[e * Env::S], xs, h.tab.empty() ? nullptr : h.tab.data(), obs);
  for (int i = 0; i < Env::XS; ++i) h.xstate[e * Env::XS + i] = xs[i];
  h.steps[e] = 0;
}

// gymnasium 0.28.1 SyncVectorEnv.step over the batch (the device's mh_env_step contract)
template <class Env>
void step_all(HostEnv& h, const float* act, const float* rs_in, float* next_obs, float* real_obs, float* reward,
              uint8_t* term_out, uint8_t* trunc_out) {
  constexpr int D = Env::D, A = Env::A, S = Env::S, XS = Env::XS, RS = Env::RS;
  const double* tab = h.tab.empty() ? nullptr : h.tab.data();
  for (int64_t e = 0; e < h.E; ++e) {
    float* s = &h.state[e * S];
    double xs[XS > 0 ? XS : 1];
    for (int i = 0; i < XS; ++i) xs[i] = h.xstate[e * XS + i];
    float u[A], obs2[D], r;
    for (int i = 0; i < A; ++i) u[i] = act[e * A + i];
    const int k = h.steps[e];
    const uint32_t ctr = h.ctr[e];
    Env::step(s, xs, k, u, tab, obs2, &r);
    bool term = false;
    for (int i = 0; i < D; ++i) term = term || (obs2[i] < Env::obs_lo(i)) || (obs2[i] > Env::obs_hi(i));
    const bool trunc = k + 1 >= mh::MAX_STEP;
    for (int i = 0; i < XS; ++i) h.xstate[e * XS + i] = xs[i];
    h.steps[e] = k + 1;
    h.ctr[e] = ctr + 1u;  // one counter per env-step, as the rollout kernel
    if (real_obs)
      for (int i = 0; i < D; ++i) real_obs[e * D + i] = obs2[i];
    if (term || trunc) {
      float rs[RS];
      if (rs_in) {
        for (int i = 0; i < RS; ++i) rs[i] = rs_in[e * RS + i];
      } else {
        mh::ResetDraw<Env>::draw(mh::make_rng(h.seed, (uint64_t)e, ctr), rs);
      }
      double xr[XS > 0 ? XS : 1];
      float o[D];
      Env::reset_from(rs, s, xr, tab, o);
      for (int i = 0; i < XS; ++i) h.xstate[e * XS + i] = xr[i];
      h.steps[e] = 0;
      for (int i = 0; i < D; ++i) next_obs[e * D + i] = o[i];
    } else {
      for (int i = 0; i < D; ++i) next_obs[e * D + i] = obs2[i];
    }
    if (reward) reward[e] = r;
    if (term_out) term_out[e] = term ? 1 : 0;
    if (trunc_out) trunc_out[e] = trunc ? 1 : 0;
  }
}

#define MHH_DISPATCH(id, CALL)                          \
  switch (id) {                                         \
    case MH_ENV_VANDERPOL: { using Env = mh::VanderPol; CALL; break; }          \
    case MH_ENV_PENDULUM: { using Env = mh::Pendulum; CALL; break; }            \
    case MH_ENV_DUCTEDFAN: { using Env = mh::DuctedFan; CALL; break; }          \
    case MH_ENV_TWOLINK: { using Env = mh::TwoLink; CALL; break; }              \
    case MH_ENV_SINGLETRACKCAR: { using Env = mh::SingleTrackCar; CALL; break; } \
    case MH_ENV_QUADTRACKING: { using Env = mh::QuadTracking; CALL; break; }    \
    default: return fail(MH_EINVAL, "unknown env id");  \
  }

template <class Env>
void fill_info(mh_env_info_t* o) {
  memset(o, 0, sizeof(*o));
  o->obs_dim = Env::D;
  o->act_dim = Env::A;
  o->state_dim = Env::S;
  o->xstate_dim = Env::XS;
  o->reset_dim = Env::RS;
  o->control_step = Env::K;
  o->max_step = mh::MAX_STEP;
  o->record_floats = ((2 * Env::D + Env::A + 4) + 3) / 4 * 4;
  for (int i = 0; i < Env::D; ++i) {
    o->obs_low[i] = Env::obs_lo(i);
    o->obs_high[i] = Env::obs_hi(i);
  }
  for (int i = 0; i < Env::A; ++i) {
    o->act_low[i] = Env::act_lo(i);
    o->act_high[i] = Env::act_hi(i);
  }
}

int set_dims(HostEnv& h, int env_id) {
  MHH_DISPATCH(env_id, dims<Env>(h));
  return MH_OK;
}

inline float relu_grad(float a) { return a > 0.0f ? 1.0f : (a == 0.0f ? 0.5f : 0.0f); }
inline float torch_min(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : (a < b ? a : b); }

}  // namespace

extern "C" {

int mhh_abi_version(void) { return 1; }
const char* mhh_last_error(void) { return g_err.c_str(); }

int mhh_env_info(int32_t env_id, mh_env_info_t* out) {
  if (!out) return fail(MH_EINVAL, "mhh_env_info: null out");
  MHH_DISPATCH(env_id, fill_info<Env>(out));
  return MH_OK;
}

int mhh_env_create(int32_t env_id, int64_t num_envs, uint64_t seed, mhh_env_t* out) {
  if (!out) return fail(MH_EINVAL, "mhh_env_create: null out");
  *out = nullptr;
  if (num_envs <= 0) return fail(MH_EINVAL, "mhh_env_create: num_envs must be positive");
  HostEnv* h = new HostEnv();
  h->env_id = env_id;
  h->E = num_envs;
  h->seed = seed;
  if (set_dims(*h, env_id) != MH_OK) {
    delete h;
    return fail(MH_EINVAL, "mhh_env_create: unknown env id");
  }
  h->state.assign((size_t)num_envs * h->S, 0.0f);
  h->xstate.assign((size_t)num_envs * (h->XS > 0 ? h->XS : 1), 0.0);
  h->steps.assign((size_t)num_envs, 0);
  h->ctr.assign((size_t)num_envs, 0u);
  if (env_id == MH_ENV_QUADTRACKING) {
    h->tab.assign((size_t)(mh::MAX_STEP + 1) * mh::QT_ROW, 0.0);
    mh::quad_fill_table(h->tab.data(), mh::MAX_STEP + 1);
    if (!mh::quad_row0_matches(h->tab.data())) {  // resets use the constant row 0
      delete h;
      return fail(MH_ESTATE, "mhh_env_create: desired-trajectory row 0 differs from QuadTracking::row0");
    }
  }
  *out = h;
  return MH_OK;
}

int mhh_env_destroy(mhh_env_t h) {
  delete static_cast<HostEnv*>(h);
  return MH_OK;
}

int mhh_env_reset(mhh_env_t hv, const float* reset_states, float* obs) {
  HostEnv* h = static_cast<HostEnv*>(hv);
  if (!h || !obs) return fail(MH_EINVAL, "mhh_env_reset: null pointer");
  for (int64_t e = 0; e < h->E; ++e) {
    const float* rs = reset_states ? reset_states + e * h->RS : nullptr;
    MHH_DISPATCH(h->env_id, reset_one<Env>(*h, e, rs, obs + e * h->D));
  }
  return MH_OK;
}

int mhh_env_step(mhh_env_t hv, const float* act, const float* reset_states, float* next_obs, float* real_next_obs,
                 float* reward, uint8_t* terminated, uint8_t* truncated) {
  HostEnv* h = static_cast<HostEnv*>(hv);
  if (!h || !act || !next_obs) return fail(MH_EINVAL, "mhh_env_step: null pointer");
  MHH_DISPATCH(h->env_id,
               step_all<Env>(*h, act, reset_states, next_obs, real_next_obs, reward, terminated, truncated));
  return MH_OK;
}

int mhh_env_get_state(mhh_env_t hv, float* state, double* xstate, int32_t* steps) {
  HostEnv* h = static_cast<HostEnv*>(hv);
  if (!h) return fail(MH_EINVAL, "mhh_env_get_state: null handle");
  if (state) memcpy(state, h->state.data(), sizeof(float) * h->state.size());
  if (xstate && h->XS > 0) memcpy(xstate, h->xstate.data(), sizeof(double) * (size_t)h->E * h->XS);
  if (steps) memcpy(steps, h->steps.data(), sizeof(int32_t) * h->steps.size());
  return MH_OK;
}

int mhh_env_set_state(mhh_env_t hv, const float* state, const double* xstate, const int32_t* steps) {
  HostEnv* h = static_cast<HostEnv*>(hv);
  if (!h) return fail(MH_EINVAL, "mhh_env_set_state: null handle");
  if (state) memcpy(h->state.data(), state, sizeof(float) * h->state.size());
  if (xstate && h->XS > 0) memcpy(h->xstate.data(), xstate, sizeof(double) * (size_t)h->E * h->XS);
  if (steps) memcpy(h->steps.data(), steps, sizeof(int32_t) * h->steps.size());
  return MH_OK;
}

// ------------------------------------------------------------------ MSACL target math (host)
// Element formulas of msacl_kernels.hip (float32, same operation order); batch sums in float64.
int mhh_msacl_q_target(const float* q1, const float* q2, const float* q1t, const float* q2t, const float* nlogp,
                       const float* rew, const float* done, const float* log_alpha, const float* weight, float gamma,
                       int32_t B, int32_t n, float* backup, float* dq1, float* dq2, float* loss_out, float* abs_td) {
  if (!q1 || !q2 || !q1t || !q2t || !nlogp || !rew || !done || !log_alpha || !backup || B <= 0 || n <= 0)
    return fail(MH_EINVAL, "mhh_msacl_q_target: bad arguments");
  const float alpha = expf(*log_alpha);
  const int64_t N = (int64_t)B * n;
  const float inv = (float)(1.0 / (double)N);
  double s1 = 0.0, s2 = 0.0;
  for (int b = 0; b < B; ++b) {
    const float wb = weight ? weight[b] : 1.0f;
    double atd = 0.0;
    for (int k = 0; k < n; ++k) {
      const int64_t i = (int64_t)b * n + k;
      const float nq = fminf(q1t[i], q2t[i]);
      const float bk = rew[i] + ((1.0f - done[i]) * gamma) * (nq - alpha * nlogp[i]);
      backup[i] = bk;
      const float e1 = q1[i] - bk, e2 = q2[i] - bk;
      s1 += (double)wb * (double)e1 * (double)e1;
      s2 += (double)wb * (double)e2 * (double)e2;
      if (dq1) dq1[i] = 2.0f * e1 * inv * wb;
      if (dq2) dq2[i] = 2.0f * e2 * inv * wb;
      atd += 0.5 * (fabs((double)q1[i] - (double)bk) + fabs((double)q2[i] - (double)bk));
    }
    if (abs_td) abs_td[b] = (float)(atd / n);
  }
  if (loss_out) loss_out[0] = (float)(s1 / (double)N) + (float)(s2 / (double)N);
  return MH_OK;
}

int mhh_msacl_lyapunov(const float* logp, const float* old_logp, const float* V, const float* V2, const float* obs,
                       const float* obs2, const float* c, const float* w, const float* s, float alpha1, float alpha2,
                       float pos_scale, float diff_scale, int32_t B, int32_t n, int32_t D, float* is_clip, float* esl,
                       float* lya_diff, float* loss_out, float* dV, float* dV2) {
  if (!logp || !old_logp || !V || !V2 || !obs || !obs2 || !c || !w || !s || !is_clip || !esl || !lya_diff || !dV ||
      !dV2 || B <= 0 || n <= 0 || D <= 0)
    return fail(MH_EINVAL, "mhh_msacl_lyapunov: bad arguments");
  const int64_t N = (int64_t)B * n;
  const float invN = (float)(1.0 / (double)N);
  const float invB = (float)(1.0 / (double)B);
  double bound = 0.0, diffs = 0.0;
  for (int b = 0; b < B; ++b) {
    float so = 0.0f;
    for (int d = 0; d < D; ++d) {
      const float x = obs[((int64_t)b * n) * D + d];
      so = so + x * x;
    }
    const float start_norm = sqrtf(so);
    const float V0 = V[(int64_t)b * n];
    float p = 1.0f, dV0 = 0.0f, rowsum = 0.0f;
    for (int k = 0; k < n; ++k) {
      const int64_t i = (int64_t)b * n + k;
      const float ratio = expf(logp[i] - old_logp[i]);
      p = p * fminf(fmaxf(ratio, 0.0f), 1.0f);  // cumprod(clamp(ratio, 0, 1))
      is_clip[i] = p;
      float pw = 0.0f, o2 = 0.0f;
      for (int d = 0; d < D; ++d) {
        const float x = obs[i * D + d];
        pw = pw + x * x;
        const float y = obs2[i * D + d];
        o2 = o2 + y * y;
      }
      const float Vi = V[i];
      const float l1 = alpha1 * pw - Vi, l2 = Vi - alpha2 * pw;
      bound += (double)fmaxf(l1, 0.0f) + (double)fmaxf(l2, 0.0f);
      const float g = pos_scale * invN * (-relu_grad(l1) + relu_grad(l2));
      const float diff = start_norm * c[k] - sqrtf(o2);
      const float E_ = diff >= 0.0f ? 1.0f : -1.0f;
      esl[i] = E_;
      const float t = E_ * (V2[i] - V0 * s[k]);
      rowsum = rowsum + w[k] * (p * fmaxf(t, 0.0f));
      const float gt = diff_scale * invB * w[k] * p * relu_grad(t);
      dV2[i] = gt * E_;
      dV0 = dV0 + gt * E_ * (-s[k]);
      dV[i] = g;
    }
    lya_diff[b] = rowsum;
    dV[(int64_t)b * n] = dV[(int64_t)b * n] + dV0;
    diffs += (double)rowsum;
  }
  if (loss_out) loss_out[0] = (float)(bound / (double)N) * pos_scale + (float)(diffs / (double)B) * diff_scale;
  return MH_OK;
}

int mhh_msacl_stability_adv(const float* V0, const float* V2, const float* w, const float* s, int32_t B, int32_t n,
                            float* adv_raw, double* stats_out) {
  if (!V0 || !V2 || !w || !s || !adv_raw || !stats_out || B <= 0 || n <= 0)
    return fail(MH_EINVAL, "mhh_msacl_stability_adv: bad arguments");
  double a1 = 0.0, a2 = 0.0;
  for (int b = 0; b < B; ++b) {
    float acc = 0.0f;
    const float v0 = V0[b];
    for (int k = 0; k < n; ++k) acc = acc + w[k] * ((v0 * s[k]) - V2[(int64_t)b * n + k]);
    adv_raw[b] = acc;
    a1 += (double)acc;
    a2 += (double)acc * (double)acc;
  }
  stats_out[0] = a1;
  stats_out[1] = a2;
  return MH_OK;
}

int mhh_msacl_ppo_clip(const float* ratio, const float* adv_raw, const double* stats, double n_total, float eps,
                       int32_t B, float* adv, float* loss_out, float* d_ratio) {
  if (!ratio || !adv_raw || !stats || !adv || !loss_out || !d_ratio || B <= 0 || n_total < 2.0)
    return fail(MH_EINVAL, "mhh_msacl_ppo_clip: bad arguments");
  const double mean = stats[0] / n_total;
  double var = (stats[1] - n_total * mean * mean) / (n_total - 1.0);
  var = var > 0.0 ? var : 0.0;
  const float meanf = (float)mean, stdf = (float)sqrt(var);
  const float lo = 1.0f - eps, hi = 1.0f + eps;
  const float invB = (float)(1.0 / (double)B);
  double acc = 0.0;
  for (int b = 0; b < B; ++b) {
    const float A = (adv_raw[b] - meanf) / (stdf + 1e-8f);
    adv[b] = A;
    const float r = ratio[b];
    const float rc = fminf(fmaxf(r, lo), hi);
    const float s1 = r * A, s2 = rc * A;
    acc += (double)fminf(s1, s2);
    const float gclip = (r >= lo && r <= hi) ? 1.0f : 0.0f;
    const float g = s1 < s2 ? A : (s1 > s2 ? gclip * A : 0.5f * A + 0.5f * gclip * A);
    d_ratio[b] = g * invB;
  }
  loss_out[0] = (float)(acc / (double)B);
  return MH_OK;
}

int mhh_msacl_policy_loss(const float* q1, const float* q2, const float* logp, const float* log_alpha, int64_t N,
                          float* loss_out, float* entropy_out) {
  if (!q1 || !q2 || !logp || !log_alpha || !loss_out || !entropy_out || N <= 0)
    return fail(MH_EINVAL, "mhh_msacl_policy_loss: bad arguments");
  const float alpha = expf(*log_alpha);
  double a = 0.0, b = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    a += (double)(torch_min(q1[i], q2[i]) - alpha * logp[i]);
    b += (double)logp[i];
  }
  loss_out[0] = (float)(a / (double)N);
  entropy_out[0] = -(float)(b / (double)N);
  return MH_OK;
}

int mhh_msacl_policy_loss_backward(const float* q1, const float* q2, const float* log_alpha, const float* g_loss,
                                   int64_t N, float* dq1, float* dq2, float* dlogp) {
  if (!q1 || !q2 || !log_alpha || !g_loss || !dq1 || !dq2 || !dlogp || N <= 0)
    return fail(MH_EINVAL, "mhh_msacl_policy_loss_backward: bad arguments");
  const float alpha = expf(*log_alpha);
  const float gg = *g_loss * (1.0f / (float)N);
  for (int64_t i = 0; i < N; ++i) {
    const float a = q1[i], b = q2[i];
    dq1[i] = a == b ? gg / 2.0f : (a > b ? 0.0f : gg);
    dq2[i] = a == b ? gg / 2.0f : (a < b ? 0.0f : gg);
    dlogp[i] = (-gg) * alpha;
  }
  return MH_OK;
}

int mhh_msacl_ratio0(const float* lp, const float* old, int32_t B, int32_t n, float* ratio) {
  if (!lp || !old || !ratio || B <= 0 || n <= 0) return fail(MH_EINVAL, "mhh_msacl_ratio0: bad arguments");
  for (int b = 0; b < B; ++b) ratio[b] = expf(lp[(int64_t)b * n] - old[(int64_t)b * n]);
  return MH_OK;
}

int mhh_msacl_ratio0_backward(const float* ratio, const float* g, int32_t B, int32_t n, float* dlp) {
  if (!ratio || !g || !dlp || B <= 0 || n <= 0) return fail(MH_EINVAL, "mhh_msacl_ratio0_backward: bad arguments");
  for (int64_t i = 0; i < (int64_t)B * n; ++i) {
    const int64_t b = i / n;
    dlp[i] = (i - b * n) == 0 ? g[b] * ratio[b] : 0.0f;
  }
  return MH_OK;
}

}  // extern "C"
