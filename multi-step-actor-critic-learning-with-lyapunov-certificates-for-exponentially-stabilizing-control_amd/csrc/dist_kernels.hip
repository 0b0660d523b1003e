// dist_kernels.hip — TanhGaussDistribution's reparameterised sample and log-prob, forward and
// backward, as single kernels (gfx950). RL/utils/act_distribution_cls.py:15-85:
//   rsample:  z = mu + std * eps,  a = h tanh(z) + m   (h = (high - low)/2, m = (high + low)/2)
//             logp = sum_i [-(z - mu)^2 / (2 std^2) - log std - log sqrt(2 pi)]
//                    - sum_i log(1 + 1e-6 - tanh(z)^2) - sum_i log h
//   log_prob(a): z = atanh((1 - 1e-6)(2a - (high + low)) / (high - low))
//             logp = sum_i [Normal(mu, std).log_prob(z)] - sum_i log(h (1 + 1e-6 - tanh(z)^2))
// logits = [mean | std] rows (StochaPolicy output). In PyTorch each of these is ~25 elementwise
// and reduction launches forward and ~30 backward; here one launch each way, one thread per row
// (A <= 8 action dims). The backward recomputes z/tanh from (logits, eps) and follows the
// derivative of each reference expression (including the z - mu terms that cancel in exact
// arithmetic), so gradients agree with autograd's to float32 rounding. Accurate libm functions
// (tanhf/logf/atanhf), float32 throughout, as torch evaluates the reference expressions.
#include "rollout.h"

namespace mh {

constexpr float kLogSqrt2Pi = 0.918938533204672742f;  // math.log(math.sqrt(2 * math.pi))

// rsample forward: act [M][A], logp [M]
__global__ __launch_bounds__(256) void k_tg_rsample(const float* __restrict__ logits, const float* __restrict__ eps,
                                                    const float* __restrict__ high, const float* __restrict__ low,
                                                    int64_t M, int A, float* __restrict__ act,
                                                    float* __restrict__ logp) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  float lg = 0.0f, lt = 0.0f, lh = 0.0f;
  for (int i = 0; i < A; ++i) {
    const float mu = logits[r * 2 * A + i], sd = logits[r * 2 * A + A + i];
    const float z = mu + sd * eps[r * A + i];
    const float df = z - mu;
    const float var = sd * sd;
    lg = lg + ((-(df * df) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi);
    const float t = tanhf(z);
    lt = lt + logf(1.000001f - t * t);
    const float h = (high[i] - low[i]) / 2.0f, m = (high[i] + low[i]) / 2.0f;
    lh = lh + logf(h);
    act[r * A + i] = h * t + m;
  }
  logp[r] = (lg - lt) - lh;
}

// rsample backward: d_logits [M][2A] from d_act [M][A] (nullable) and d_logp [M] (nullable)
__global__ __launch_bounds__(256) void k_tg_rsample_bwd(const float* __restrict__ logits,
                                                        const float* __restrict__ eps,
                                                        const float* __restrict__ high, const float* __restrict__ low,
                                                        const float* __restrict__ d_act,
                                                        const float* __restrict__ d_logp, int64_t M, int A,
                                                        float* __restrict__ d_logits) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  const float gl = d_logp ? d_logp[r] : 0.0f;
  for (int i = 0; i < A; ++i) {
    const float mu = logits[r * 2 * A + i], sd = logits[r * 2 * A + A + i];
    const float e = eps[r * A + i];
    const float z = mu + sd * e;
    const float df = z - mu;
    const float var = sd * sd;
    const float t = tanhf(z);
    const float h = (high[i] - low[i]) / 2.0f;
    const float ga = d_act ? d_act[r * A + i] : 0.0f;
    // a = h t + m ; -log(1 + 1e-6 - t^2) ; t = tanh z
    const float u = 1.000001f - t * t;
    const float dt = ga * h + gl * (2.0f * t / u);
    float dz = dt * (1.0f - t * t);
    // Normal log-prob: -(df^2) / (2 var) with df = z - mu, var = sd^2; - log sd
    const float q = df / var;
    dz = dz + gl * (-q);
    const float dmu = dz + gl * q;
    const float dvar = gl * (df * df) / (2.0f * var * var);
    const float dsd = dz * e + dvar * (2.0f * sd) - gl / sd;
    d_logits[r * 2 * A + i] = dmu;
    d_logits[r * 2 * A + A + i] = dsd;
  }
}

// log_prob(action) forward
__global__ __launch_bounds__(256) void k_tg_log_prob(const float* __restrict__ logits, const float* __restrict__ a,
                                                     const float* __restrict__ high, const float* __restrict__ low,
                                                     int64_t M, int A, float* __restrict__ logp) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  float lg = 0.0f, lj = 0.0f;
  for (int i = 0; i < A; ++i) {
    const float mu = logits[r * 2 * A + i], sd = logits[r * 2 * A + A + i];
    const float hl = high[i] + low[i], dl = high[i] - low[i];
    const float z = atanhf(0.999999f * (2.0f * a[r * A + i] - hl) / dl);  // float32(1 - 1e-6)
    const float df = z - mu;
    lg = lg + ((-(df * df) / (2.0f * (sd * sd)) - logf(sd)) - kLogSqrt2Pi);
    const float t = tanhf(z);
    lj = lj + logf(dl / 2.0f * (1.000001f - t * t));
  }
  logp[r] = lg - lj;
}

// log_prob backward w.r.t. logits (the action is data)
__global__ __launch_bounds__(256) void k_tg_log_prob_bwd(const float* __restrict__ logits,
                                                         const float* __restrict__ a,
                                                         const float* __restrict__ high,
                                                         const float* __restrict__ low,
                                                         const float* __restrict__ d_logp, int64_t M, int A,
                                                         float* __restrict__ d_logits) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  const float gl = d_logp[r];
  for (int i = 0; i < A; ++i) {
    const float mu = logits[r * 2 * A + i], sd = logits[r * 2 * A + A + i];
    const float hl = high[i] + low[i], dl = high[i] - low[i];
    const float z = atanhf(0.999999f * (2.0f * a[r * A + i] - hl) / dl);  // float32(1 - 1e-6)
    const float df = z - mu;
    const float var = sd * sd;
    d_logits[r * 2 * A + i] = gl * (df / var);
    d_logits[r * 2 * A + A + i] = gl * ((df * df) / (2.0f * var * var)) * (2.0f * sd) - gl / sd;
  }
}

// StochaPolicy head (RL/apprfunc/mlp.py:132-136): out = [mean | exp(clamp(log_std, lo, hi))] from the
// MLP's raw [mean | log_std], and its backward d_raw = [d_mean | d_std * std * (lo <= log_std <= hi)]
// (torch's exp / clamp backward). One thread per element of the [M][2A] block.
__global__ __launch_bounds__(256) void k_stocha_head(const float* __restrict__ raw, int64_t total, int A, float lo,
                                                     float hi, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const float x = raw[i];
  out[i] = (int)(i % (2 * A)) < A ? x : expf(fminf(fmaxf(x, lo), hi));
}
__global__ __launch_bounds__(256) void k_stocha_head_bwd(const float* __restrict__ raw, const float* __restrict__ out,
                                                         const float* __restrict__ dout, int64_t total, int A,
                                                         float lo, float hi, float* __restrict__ draw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const float d = dout[i];
  if ((int)(i % (2 * A)) < A) {
    draw[i] = d;
  } else {
    const float x = raw[i];
    const float gx = d * out[i];
    draw[i] = (x >= lo && x <= hi) ? gx : gx * 0.0f;
  }
}

// The MSACL update's policy head (msacl.py:242-251, 270-273, 340-394): StochaPolicy's
// [mean | exp(clamp(log_std))] of the MLP's raw rows, then any of
//   rsample (eps given): act = h tanh(mu + std eps) + m and its log-prob (k_tg_rsample's math),
//     the act written into the critic input row xq = [obs | act] (ActionValue's concat);
//   log_prob(old_act) (old_act given): k_tg_log_prob's math;
// in one launch instead of stocha_head + rsample + log_prob + a concat per critic. One LANE per
// (row, action dim) in groups of PH_G = 8 lanes per row (A <= 8): each lane evaluates its
// dimension's terms (the transcendental chain of one dimension instead of A of them per thread:
// the kernel is latency-bound at B*n = 5,120 rows), and the row's sums are formed by the group's
// first lane over the A lane values in dimension order, 0 + t0 + t1 + ..., exactly the
// per-row loop's order: every value is the separate kernels' bit for bit.
constexpr int PH_G = 8;

__device__ __forceinline__ float ph_row_sum(float v, int A, int base) {  // sum_{i < A} v(lane base + i), in order
  float s = 0.0f;
  for (int i = 0; i < A; ++i) s = s + __shfl(v, base + i, 64);
  return s;
}

// In-kernel rsample noise (eps null, eps_out set): lane (r, i) draws its standard normal from
// Philox4x32-10 keyed by (seed, row r, launch counter ctr[0]) — Box-Muller normal4f, stream i / 4,
// component i % 4 — and writes it to eps_out for the backward. ctr[0] advances by one per launch:
// the last workgroup to arrive (ctr[1], an arrival count every workgroup bumps after it has read
// ctr[0]) increments it and re-arms ctr[1], so a captured graph draws fresh noise on every replay
// without a host-side generator (the torch normal_ launch it replaces).
__global__ __launch_bounds__(256) void k_policy_head(const float* __restrict__ raw, const float* __restrict__ eps,
                                                     const float* __restrict__ obs, const float* __restrict__ old_act,
                                                     const float* __restrict__ high, const float* __restrict__ low,
                                                     int64_t M, int A, int D, float lo, float hi,
                                                     float* __restrict__ xq, float* __restrict__ new_logp,
                                                     float* __restrict__ old_logp, uint64_t seed,
                                                     unsigned long long* ctr, float* __restrict__ eps_out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = t / PH_G;
  const int i = (int)(t % PH_G);
  const int base = (threadIdx.x & 63) & ~(PH_G - 1);
  const bool row_ok = r < M;  // (whole groups share a row: the shuffles below stay in the group)
  const bool on = row_ok && i < A;
  const bool draw = !eps && eps_out && ctr;
  float e_draw = 0.0f;
  if (draw) {
    const unsigned long long c = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (on) {
      float nv[4];
      make_rng(seed, (uint64_t)r, (uint64_t)c).normal4f((uint32_t)(i >> 2), nv);
      e_draw = nv[i & 3];
      eps_out[r * A + i] = e_draw;
    }
    __syncthreads();  // every lane of the workgroup has read ctr[0] (its value consumed above)
    // RELAXED arrival (optim.hip's Adam ticket): the only ordering needed is that every workgroup's
    // read of ctr[0] returned before its arrival, and the read was consumed before the barrier. No
    // data passes between workgroups, so no agent-scope fence / acquire-release (each an L2
    // writeback + invalidate: the draw cost 12.5 us at 5,120 rows with them, tools/head_bench.py)
    if (threadIdx.x == 0) {
#ifdef MH_REDUCE_FENCED  // A/B only: the former fenced arrival
      __threadfence();
#endif
      const unsigned int arrived =
          __hip_atomic_fetch_add(reinterpret_cast<unsigned int*>(ctr + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (arrived == gridDim.x - 1) {  // the last workgroup: every other has read the counter
        __hip_atomic_store(reinterpret_cast<unsigned int*>(ctr + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  const int W = D + A;
  if (row_ok && xq && obs) {
    for (int j = i; j < D; j += PH_G) xq[r * W + j] = obs[r * D + j];
  }
  float lgv = 0.0f, ltv = 0.0f, lhv = 0.0f, ogv = 0.0f, ojv = 0.0f;
  if (on) {
    const float mu = raw[r * 2 * A + i];
    const float sd = expf(fminf(fmaxf(raw[r * 2 * A + A + i], lo), hi));
    if (eps || draw) {
      const float z = mu + sd * (draw ? e_draw : eps[r * A + i]);
      const float df = z - mu;
      const float var = sd * sd;
      lgv = (-(df * df) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi;
      const float tz = tanhf(z);
      ltv = logf(1.000001f - tz * tz);
      const float h = (high[i] - low[i]) / 2.0f, m = (high[i] + low[i]) / 2.0f;
      lhv = logf(h);
      if (xq) xq[r * W + D + i] = h * tz + m;
    }
    if (old_act) {
      const float hl = high[i] + low[i], dl = high[i] - low[i];
      const float z = atanhf(0.999999f * (2.0f * old_act[r * A + i] - hl) / dl);
      const float df = z - mu;
      ogv = (-(df * df) / (2.0f * (sd * sd)) - logf(sd)) - kLogSqrt2Pi;
      const float tz = tanhf(z);
      ojv = logf(dl / 2.0f * (1.000001f - tz * tz));
    }
  }
  if ((eps || draw) && new_logp) {
    const float lg = ph_row_sum(lgv, A, base), lt = ph_row_sum(ltv, A, base), lh = ph_row_sum(lhv, A, base);
    if (row_ok && i == 0) new_logp[r] = (lg - lt) - lh;
  }
  if (old_act && old_logp) {
    const float og = ph_row_sum(ogv, A, base), oj = ph_row_sum(ojv, A, base);
    if (row_ok && i == 0) old_logp[r] = og - oj;
  }
}

// Its backward: d_raw from the gradients of the critic input's action columns (d_xq), of the
// sample's log-prob (d_new_logp) and of log_prob(old_act) (d_old_logp), any of them null:
// k_tg_rsample_bwd's and k_tg_log_prob_bwd's expressions, their d_logits added as autograd
// accumulates them (one term alone is not added to anything), then k_stocha_head_bwd's. One lane
// per (row, action dim): the dimensions are independent.
__global__ __launch_bounds__(256) void k_policy_head_bwd(const float* __restrict__ raw, const float* __restrict__ eps,
                                                         const float* __restrict__ old_act,
                                                         const float* __restrict__ high, const float* __restrict__ low,
                                                         const float* __restrict__ d_xq,
                                                         const float* __restrict__ d_new_logp,
                                                         const float* __restrict__ d_old_logp, int64_t M, int A, int D,
                                                         float lo, float hi, float* __restrict__ d_raw) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = t / PH_G;
  const int i = (int)(t % PH_G);
  if (r >= M || i >= A) return;
  const int W = D + A;
  const bool samp = eps && (d_xq || d_new_logp);
  const bool score = old_act && d_old_logp;
  const float gl = d_new_logp ? d_new_logp[r] : 0.0f;
  const float go = score ? d_old_logp[r] : 0.0f;
  const float mu = raw[r * 2 * A + i];
  const float x = raw[r * 2 * A + A + i];
  const float sd = expf(fminf(fmaxf(x, lo), hi));
  float dmu = 0.0f, dsd = 0.0f;
  if (samp) {
    const float e = eps[r * A + i];
    const float z = mu + sd * e;
    const float df = z - mu;
    const float var = sd * sd;
    const float tz = tanhf(z);
    const float h = (high[i] - low[i]) / 2.0f;
    const float ga = d_xq ? d_xq[r * W + D + i] : 0.0f;
    const float u = 1.000001f - tz * tz;
    const float dt = ga * h + gl * (2.0f * tz / u);
    float dz = dt * (1.0f - tz * tz);
    const float q = df / var;
    dz = dz + gl * (-q);
    dmu = dz + gl * q;
    const float dvar = gl * (df * df) / (2.0f * var * var);
    dsd = dz * e + dvar * (2.0f * sd) - gl / sd;
  }
  if (score) {
    const float hl = high[i] + low[i], dl = high[i] - low[i];
    const float z = atanhf(0.999999f * (2.0f * old_act[r * A + i] - hl) / dl);
    const float df = z - mu;
    const float var = sd * sd;
    const float m2 = go * (df / var);
    const float s2 = go * ((df * df) / (2.0f * var * var)) * (2.0f * sd) - go / sd;
    dmu = samp ? dmu + m2 : m2;
    dsd = samp ? dsd + s2 : s2;
  }
  d_raw[r * 2 * A + i] = dmu;
  const float gx = dsd * sd;
  d_raw[r * 2 * A + A + i] = (x >= lo && x <= hi) ? gx : gx * 0.0f;
}

static inline unsigned grid_rows(int64_t M) { return (unsigned)((M + 255) / 256); }
static inline unsigned grid_row_lanes(int64_t M) { return (unsigned)((M * PH_G + 255) / 256); }

hipError_t launch_policy_head(const float* raw, const float* eps, const float* obs, const float* old_act,
                              const float* high, const float* low, int64_t M, int A, int D, float lo, float hi,
                              float* xq, float* new_logp, float* old_logp, hipStream_t st, uint64_t seed,
                              unsigned long long* ctr, float* eps_out) {
  if (M <= 0) return hipSuccess;
  if (A <= 0 || A > PH_G) return hipErrorInvalidValue;
  k_policy_head<<<grid_row_lanes(M), 256, 0, st>>>(raw, eps, obs, old_act, high, low, M, A, D, lo, hi, xq, new_logp,
                                                   old_logp, seed, ctr, eps_out);
  return hipGetLastError();
}
hipError_t launch_policy_head_bwd(const float* raw, const float* eps, const float* old_act, const float* high,
                                  const float* low, const float* d_xq, const float* d_new_logp,
                                  const float* d_old_logp, int64_t M, int A, int D, float lo, float hi, float* d_raw,
                                  hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (A <= 0 || A > PH_G) return hipErrorInvalidValue;
  k_policy_head_bwd<<<grid_row_lanes(M), 256, 0, st>>>(raw, eps, old_act, high, low, d_xq, d_new_logp, d_old_logp, M,
                                                       A, D, lo, hi, d_raw);
  return hipGetLastError();
}

hipError_t launch_stocha_head(const float* raw, int64_t M, int A, float lo, float hi, float* out, hipStream_t st) {
  const int64_t total = M * 2 * A;
  if (total <= 0) return hipSuccess;
  k_stocha_head<<<grid_rows(total), 256, 0, st>>>(raw, total, A, lo, hi, out);
  return hipGetLastError();
}
hipError_t launch_stocha_head_bwd(const float* raw, const float* out, const float* dout, int64_t M, int A, float lo,
                                  float hi, float* draw, hipStream_t st) {
  const int64_t total = M * 2 * A;
  if (total <= 0) return hipSuccess;
  k_stocha_head_bwd<<<grid_rows(total), 256, 0, st>>>(raw, out, dout, total, A, lo, hi, draw);
  return hipGetLastError();
}

hipError_t launch_tg_rsample(const float* logits, const float* eps, const float* high, const float* low, int64_t M,
                             int A, float* act, float* logp, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_tg_rsample<<<grid_rows(M), 256, 0, st>>>(logits, eps, high, low, M, A, act, logp);
  return hipGetLastError();
}
hipError_t launch_tg_rsample_bwd(const float* logits, const float* eps, const float* high, const float* low,
                                 const float* d_act, const float* d_logp, int64_t M, int A, float* d_logits,
                                 hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_tg_rsample_bwd<<<grid_rows(M), 256, 0, st>>>(logits, eps, high, low, d_act, d_logp, M, A, d_logits);
  return hipGetLastError();
}
hipError_t launch_tg_log_prob(const float* logits, const float* a, const float* high, const float* low, int64_t M,
                              int A, float* logp, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_tg_log_prob<<<grid_rows(M), 256, 0, st>>>(logits, a, high, low, M, A, logp);
  return hipGetLastError();
}
hipError_t launch_tg_log_prob_bwd(const float* logits, const float* a, const float* high, const float* low,
                                  const float* d_logp, int64_t M, int A, float* d_logits, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  k_tg_log_prob_bwd<<<grid_rows(M), 256, 0, st>>>(logits, a, high, low, d_logp, M, A, d_logits);
  return hipGetLastError();
}

}  // namespace mh
