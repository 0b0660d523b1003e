// msacl_kernels.hip — fused MSACL target / certificate math (RL/algorithm/msacl.py).
//
// The replay batch is [B][n] (B = 256, n = 20 at the reference config: 5,120 elements, 20 KB
// per tensor). Each op below replaces a chain of 8-20 tiny PyTorch launches with ONE kernel:
// one wavefront per window row keeps the n-step scan (cumprod, lambda-weighted sums) in
// registers (q_target / lyapunov: 4 rows per workgroup, B/4 workgroups; the small advantage
// ops: one workgroup), and the batch-global means are reduced in float64 in a fixed order, so
// results are bitwise reproducible run to run. q_target and lyapunov keep their cross-workgroup
// partials in a library-owned per-device scratch: calls of one of them on one device must be
// stream-ordered (they are: the MSACL update issues them on one stream).
// Each kernel also emits the analytic gradient w.r.t. its network-produced inputs, which the
// Python layer feeds to autograd (custom autograd.Function), so the MLP backward stays PyTorch.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <string>

#include "msacl_hip.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 1024;  // one workgroup; 16 wavefronts

// torch.maximum / torch.minimum backward: ties split the gradient in half.
__device__ __forceinline__ float relu_grad(float a) { return a > 0.0f ? 1.0f : (a == 0.0f ? 0.5f : 0.0f); }

// Workgroup sum of one double per thread, the same value returned to every thread: a butterfly
// within each wavefront, then the 16 wave totals added in wave order by every thread (two
// barriers; the 10-level LDS tree it replaces held 10 barriers per sum). `sh` needs TPB / 64 + 1
// entries. Deterministic: a fixed order for a fixed launch shape.
__device__ double block_sum(double v, double* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < TPB / 64; ++w) r += sh[w];
  __syncthreads();  // sh is reused by the next sum
  return r;
}

// Row kernels: one wavefront per window row b (lanes own the n steps), RPB rows per workgroup,
// ceil(B / RPB) workgroups. Batch-global sums go through per-workgroup float64 partials; the
// workgroup that finishes last adds them in workgroup order (deterministic) and resets the
// arrival counter, so no extra launch and no memset are needed.
constexpr int RPB = 4;             // rows (wavefronts) per workgroup
constexpr int RTPB = RPB * 64;

struct RowScratch {
  double* part = nullptr;          // [cap][4] per-workgroup partial sums (2 or 4 used)
  unsigned int* arrive = nullptr;  // arrival counter (0 between launches)
  int64_t cap = 0;
};

// Library-owned per-device scratch, grown outside graph capture (the first, eager call).
hipError_t row_scratch(int slot, int64_t blocks, RowScratch** out) {
  static RowScratch per_dev[2][64];  // [kernel slot][device]: each kernel owns its counter
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  RowScratch& r = per_dev[slot][dev];
  if (r.cap < blocks) {
    if (r.part) (void)hipFree(r.part);
    if (r.arrive) (void)hipFree(r.arrive);
    r.part = nullptr;
    r.arrive = nullptr;
    r.cap = 0;
    const int64_t cap = blocks < 4096 ? 4096 : blocks;
    e = hipMalloc(&r.part, sizeof(double) * 4 * cap);
    if (e == hipSuccess) e = hipMalloc(&r.arrive, sizeof(unsigned int));
    if (e == hipSuccess) e = hipMemset(r.arrive, 0, sizeof(unsigned int));
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    r.cap = cap;
  }
  *out = &r;
  return hipSuccess;
}

__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sum v[0..K) over the workgroup, publish the partials, and let the last workgroup total them.
// Returns true in thread 0 of the last workgroup with the batch sums in t[0..K).
template <int K>
__device__ bool rows_reduce(const double (&v)[K], double* part, unsigned int* arrive, double (&t)[K]) {
  __shared__ double sv[K][RPB];
  __shared__ bool last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double w[K];
#pragma unroll
  for (int j = 0; j < K; ++j) w[j] = wave_sum(v[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) sv[j][wave] = w[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      x[j] = 0.0;
      for (int q = 0; q < RPB; ++q) x[j] += sv[j][q];
    }
#ifdef MH_REDUCE_FENCED  // A/B only: the agent-scope fences (an L2 writeback + invalidate each)
#pragma unroll
    for (int j = 0; j < K; ++j) part[K * blockIdx.x + j] = x[j];
    __threadfence();
    last = atomicAdd(arrive, 1u) == gridDim.x - 1u;
#else
    // The partials as agent-scope atomic stores (written through to the device's coherence point,
    // not left in this XCD's L2), complete (vmcnt(0)) before the relaxed arrival; the last
    // workgroup reads them with agent-scope atomic loads. No fence: an agent-scope release /
    // acquire writes back / invalidates the whole L2, which inside the update holds the other
    // branch's dirty lines too (this launch took 25 us there with the fences).
    // Memory-model basis (LLVM AMDGPUUsage, "Memory Model GFX942" code sequences, which gfx950
    // follows): an agent-scope atomic store is a `global_store ... sc1`, written through to the
    // coherence point; `s_waitcnt vmcnt(0)` returns only once it is performed there, and the
    // relaxed arrival is issued after that wait in program order. The last workgroup reads the
    // partials with agent-scope atomic loads (`sc1`: from the coherence point, not a stale L1/L2
    // line), so it sees them without an acquire (MI355X_MICROARCH.md, "Hand-offs measured with
    // sc1 loads", row 1).
#pragma unroll
    for (int j = 0; j < K; ++j)
      __hip_atomic_store(part + K * blockIdx.x + j, x[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every store acknowledged
    last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
#endif
  }
  __syncthreads();
  if (!last) return false;
#ifdef MH_REDUCE_FENCED
  __threadfence();
  const volatile double* vp = part;
#define MH_PART(i) vp[i]
#else
#define MH_PART(i) __hip_atomic_load(part + (i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#endif
  // last workgroup: fixed-order total (lane-strided partials, then wave/LDS tree)
  double x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = 0.0;
  for (unsigned int g = threadIdx.x; g < gridDim.x; g += RTPB) {
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] += MH_PART(K * g + j);
  }
#undef MH_PART
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = wave_sum(x[j]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) sv[j][wave] = x[j];
  }
  __syncthreads();
  if (threadIdx.x != 0) return false;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double X = 0.0;
    for (int q = 0; q < RPB; ++q) X += sv[j][q];
    t[j] = X;
  }
#ifdef MH_REDUCE_FENCED
  *arrive = 0u;
#else
  __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
  return true;
}

// ------------------------------------------------------------------ Q backup (msacl.py:242-257)
__global__ __launch_bounds__(RTPB) void k_q_target(const float* q1, const float* q2, const float* q1t,
                                                   const float* q2t, const float* nlogp, const float* rew,
                                                   const float* done, const float* log_alpha, const float* weight,
                                                   float gamma, int B, int n, float* backup, float* dq1,
                                                   float* dq2, float* loss_out, float* abs_td, float* q_means,
                                                   double* part, unsigned int* arrive) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * RPB + (threadIdx.x >> 6);
  const float alpha = expf(*log_alpha);
  const int64_t N = (int64_t)B * n;
  const float inv = (float)(1.0 / (double)N);
  double acc1 = 0.0, acc2 = 0.0, atd = 0.0, sq1 = 0.0, sq2 = 0.0;
  if (b < B) {
    const float wb = weight ? weight[b] : 1.0f;
    for (int k = lane; k < n; k += 64) {
      const int64_t i = (int64_t)b * n + k;
      const float nq = fminf(q1t[i], q2t[i]);
      const float bk = rew[i] + ((1.0f - done[i]) * gamma) * (nq - alpha * nlogp[i]);
      backup[i] = bk;
      const float e1 = q1[i] - bk, e2 = q2[i] - bk;
      acc1 += (double)wb * (double)e1 * (double)e1;
      acc2 += (double)wb * (double)e2 * (double)e2;
      if (dq1) dq1[i] = 2.0f * e1 * inv * wb;
      if (dq2) dq2[i] = 2.0f * e2 * inv * wb;
      atd += 0.5 * (fabs((double)q1[i] - (double)bk) + fabs((double)q2[i] - (double)bk));
      sq1 += (double)q1[i];
      sq2 += (double)q2[i];
    }
    atd = wave_sum(atd);
    if (abs_td && lane == 0) abs_td[b] = (float)(atd / n);
  }
  // the loss sums, plus the q1 / q2 sums when the logged means are wanted (msacl.py:211-222)
  if (q_means) {
    double t[4];
    if (rows_reduce<4>({acc1, acc2, sq1, sq2}, part, arrive, t)) {
      if (loss_out) loss_out[0] = (float)(t[0] / (double)N) + (float)(t[1] / (double)N);
      q_means[0] = (float)(t[2] / (double)N);
      q_means[1] = (float)(t[3] / (double)N);
    }
  } else {
    double t[2];
    if (rows_reduce<2>({acc1, acc2}, part, arrive, t) && loss_out)
      loss_out[0] = (float)(t[0] / (double)N) + (float)(t[1] / (double)N);
  }
}

// --------------------------------------------------- Lyapunov certificate (msacl.py:279-332)
// cumprod of the clipped IS ratio is a wave-level inclusive product scan (n <= 64 per pass,
// chained across passes).
// DT: the observation width at compile time (1..16; the launcher dispatches on D), so the
// per-lane norm loops unroll and their loads issue together instead of one round trip per
// element (the runtime-D loop, DT = 0, waited out 2 D dependent loads per lane)
template <int DT>
__global__ __launch_bounds__(RTPB) void k_lyapunov(const float* logp, const float* old_logp, const float* V,
                                                   const float* V2, const float* obs, const float* obs2,
                                                   const float* c, const float* w, const float* s, float alpha1,
                                                   float alpha2, float pos_scale, float diff_scale, int B, int n,
                                                   int Drt, float* is_clip, float* esl, float* lya_diff,
                                                   float* loss_out, float* dV, float* dV2, double* part,
                                                   unsigned int* arrive) {
  const int D = DT > 0 ? DT : Drt;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * RPB + (threadIdx.x >> 6);
  const int64_t N = (int64_t)B * n;
  const float invN = (float)(1.0 / (double)N);
  const float invB = (float)(1.0 / (double)B);
  double bound_acc = 0.0, diff_acc = 0.0;
  if (b < B) {
    // ||obs[b, 0, :]||
    float so = 0.0f;
    for (int d = 0; d < D; ++d) {
      const float x = obs[((int64_t)b * n) * D + d];
      so = so + x * x;
    }
    const float start_norm = sqrtf(so);
    const float V0 = V[(int64_t)b * n];
    float carry = 1.0f;       // running cumprod across 64-lane passes
    float dV0_acc = 0.0f;     // d loss3 / d V(obs[b,0]) contributions
    float rowsum = 0.0f;
    for (int k0 = 0; k0 < n; k0 += 64) {
      const int k = k0 + lane;
      const bool ok = k < n;
      const int64_t i = (int64_t)b * n + (ok ? k : 0);
      float cr = 1.0f;
      if (ok) {
        const float ratio = expf(logp[i] - old_logp[i]);
        cr = fminf(fmaxf(ratio, 0.0f), 1.0f);   // torch.clamp(ratio, 0, 1)
      }
      // inclusive product scan over the wave (Hillis-Steele with shuffles)
      float p = cr;
      for (int off = 1; off < 64; off <<= 1) {
        const float o = __shfl_up(p, off, 64);
        if (lane >= off) p = p * o;
      }
      p = p * carry;
      carry = __shfl(p, 63, 64);
      if (ok) {
        is_clip[i] = p;
        // bound terms (loss_lya2): relu(a1*|x|^2 - V) + relu(V - a2*|x|^2)
        float pw = 0.0f;
        float o2 = 0.0f;
        for (int d = 0; d < D; ++d) {
          const float x = obs[i * D + d];
          pw = pw + x * x;
          const float y = obs2[i * D + d];
          o2 = o2 + y * y;
        }
        const float Vi = V[i];
        const float l1 = alpha1 * pw - Vi, l2 = Vi - alpha2 * pw;
        bound_acc += (double)fmaxf(l1, 0.0f) + (double)fmaxf(l2, 0.0f);
        float g = pos_scale * invN * (-relu_grad(l1) + relu_grad(l2));
        // exponential stability label (msacl.py:307-314)
        const float diff = start_norm * c[k] - sqrtf(o2);
        const float E_ = diff >= 0.0f ? 1.0f : -1.0f;
        esl[i] = E_;
        const float t = E_ * (V2[i] - V0 * s[k]);
        const float term = p * fmaxf(t, 0.0f);
        rowsum = rowsum + w[k] * term;
        const float gt = diff_scale * invB * w[k] * p * relu_grad(t);
        dV2[i] = gt * E_;
        dV0_acc = dV0_acc + gt * E_ * (-s[k]);
        dV[i] = g;  // the k = 0 entry also receives dV0 below
      }
    }
    // wave reductions: lambda-weighted row sum and the V(obs_b0) gradient
    for (int off = 32; off > 0; off >>= 1) {
      rowsum = rowsum + __shfl_xor(rowsum, off, 64);
      dV0_acc = dV0_acc + __shfl_xor(dV0_acc, off, 64);
    }
    if (lane == 0) {
      lya_diff[b] = rowsum;
      dV[(int64_t)b * n] = dV[(int64_t)b * n] + dV0_acc;
      diff_acc = (double)rowsum;
    }
  }
  double t[2];
  if (rows_reduce<2>({bound_acc, diff_acc}, part, arrive, t) && loss_out)
    loss_out[0] = (float)(t[0] / (double)N) * pos_scale + (float)(t[1] / (double)B) * diff_scale;
}

// ------------------------------------------------ stability advantage (msacl.py:383-399)
__global__ __launch_bounds__(TPB) void k_stab_adv(const float* V0, const float* V2, const float* w,
                                                  const float* s, int B, int n, float* adv, double* stats) {
  __shared__ double sh[TPB];
  double a1 = 0.0, a2 = 0.0;
  for (int b = threadIdx.x; b < B; b += TPB) {
    float acc = 0.0f;
    const float v0 = V0[b];
    for (int k = 0; k < n; ++k) acc = acc + w[k] * ((v0 * s[k]) - V2[(int64_t)b * n + k]);
    adv[b] = acc;
    a1 += (double)acc;
    a2 += (double)acc * (double)acc;
  }
  const double t1 = block_sum(a1, sh), t2 = block_sum(a2, sh);
  if (threadIdx.x == 0) {
    stats[0] = t1;
    stats[1] = t2;
  }
}

// --------------------------------------------------- PPO clip on the advantage (msacl.py:400-405)
__device__ __forceinline__ void ppo_clip_body(const float* ratio, const float* adv_raw, const double* stats,
                                              double n_total, float eps, int B, float* adv, float* loss_out,
                                              float* d_ratio, double* sh) {
  const double mean = stats[0] / n_total;
  double var = (stats[1] - n_total * mean * mean) / (n_total - 1.0);
  var = var > 0.0 ? var : 0.0;
  const float meanf = (float)mean, stdf = (float)sqrt(var);
  const float lo = 1.0f - eps, hi = 1.0f + eps;
  const float invB = (float)(1.0 / (double)B);
  double acc = 0.0;
  for (int b = threadIdx.x; b < B; b += TPB) {
    const float A = (adv_raw[b] - meanf) / (stdf + 1e-8f);
    adv[b] = A;
    const float r = ratio[b];
    const float rc = fminf(fmaxf(r, lo), hi);
    const float s1 = r * A, s2 = rc * A;
    acc += (double)fminf(s1, s2);
    const float gclip = (r >= lo && r <= hi) ? 1.0f : 0.0f;
    float g;
    if (s1 < s2)
      g = A;
    else if (s1 > s2)
      g = gclip * A;
    else
      g = 0.5f * A + 0.5f * gclip * A;
    d_ratio[b] = g * invB;
  }
  const double t = block_sum(acc, sh);
  if (threadIdx.x == 0) loss_out[0] = (float)(t / (double)B);
}
__global__ __launch_bounds__(TPB) void k_ppo_clip(const float* ratio, const float* adv_raw, const double* stats,
                                                  double n_total, float eps, int B, float* adv, float* loss_out,
                                                  float* d_ratio) {
  __shared__ double sh[TPB];
  ppo_clip_body(ratio, adv_raw, stats, n_total, eps, B, adv, loss_out, d_ratio, sh);
}

// --------------------------------------------------- policy loss pieces (msacl.py:383-405)
// loss_policy_q = (min(q1, q2) - alpha * logp).mean(), alpha = exp(log_alpha) (the reference's
// alpha.item()), and the entropy -logp.mean() as a by-product: one workgroup, fixed-order sums.
__device__ __forceinline__ float torch_min(float a, float b) {
  return (a != a || b != b) ? __builtin_nanf("") : (a < b ? a : b);  // torch.min propagates NaN
}
__device__ __forceinline__ void policy_loss_body(const float* q1, const float* q2, const float* logp,
                                                 const float* log_alpha, int64_t N, float* loss, float* entropy,
                                                 double* sh) {
  const float alpha = expf(*log_alpha);
  double a = 0.0, b = 0.0;
  // PL_U of a thread's elements per round, every load issued before the first sum (the plain
  // loop waited out one load round trip per element); the sums keep the element order
  constexpr int PL_U = 8;
  for (int64_t i0 = threadIdx.x; i0 < N; i0 += PL_U * TPB) {
    float x1[PL_U], x2[PL_U], xl[PL_U];
#pragma unroll
    for (int u = 0; u < PL_U; ++u) {
      const int64_t i = i0 + (int64_t)u * TPB, ic = i < N ? i : N - 1;
      x1[u] = q1[ic];
      x2[u] = q2[ic];
      xl[u] = logp[ic];
    }
#pragma unroll
    for (int u = 0; u < PL_U; ++u) {
      if (i0 + (int64_t)u * TPB < N) {
        const float m = torch_min(x1[u], x2[u]);
        a += (double)(m - alpha * xl[u]);
        b += (double)xl[u];
      }
    }
  }
  const double ta = block_sum(a, sh);
  const double tb = block_sum(b, sh);
  if (threadIdx.x == 0) {
    loss[0] = (float)(ta / (double)N);
    entropy[0] = -(float)(tb / (double)N);
  }
}
__global__ __launch_bounds__(TPB) void k_policy_loss(const float* q1, const float* q2, const float* logp,
                                                     const float* log_alpha, int64_t N, float* loss,
                                                     float* entropy) {
  __shared__ double sh[TPB];
  policy_loss_body(q1, q2, logp, log_alpha, N, loss, entropy, sh);
}
// autograd's backward of that expression for an upstream gradient g (device scalar):
// mean -> g / N; sub -> (+, -); mul by alpha; minimum -> the smaller input (ties: half each)
__global__ __launch_bounds__(256) void k_policy_loss_bwd(const float* q1, const float* q2, const float* log_alpha,
                                                         const float* g, int64_t N, float* dq1, float* dq2,
                                                         float* dlogp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const float alpha = expf(*log_alpha);
  const float gg = *g * (1.0f / (float)N);  // PyTorch's division by a scalar: times its f32 reciprocal
  const float a = q1[i], b = q2[i];
  // torch minimum's backward: where(a == b, g / 2, g), zeroed where the other input is smaller
  // (so a NaN pair passes the gradient to both, as autograd does)
  dq1[i] = a == b ? gg / 2.0f : (a > b ? 0.0f : gg);
  dq2[i] = a == b ? gg / 2.0f : (a < b ? 0.0f : gg);
  dlogp[i] = (-gg) * alpha;
}
// is_ratio = exp(logp_new - old_logp)[:, 0] (msacl.py:392-394; only step 0 of each window is used)
__global__ __launch_bounds__(256) void k_ratio0(const float* lp, const float* old, int B, int n, float* ratio) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) ratio[b] = expf(lp[(int64_t)b * n] - old[(int64_t)b * n]);
}
__global__ __launch_bounds__(256) void k_ratio0_bwd(const float* ratio, const float* g, int B, int n, float* dlp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * n) return;
  const int64_t b = i / n;
  dlp[i] = (i - b * n) == 0 ? g[b] * ratio[b] : 0.0f;
}

// loss_policy = -loss_policy_q - loss_policy_lya (msacl.py:401-405, the logged total) and the
// seed -d_ratio of the is_ratio backward, in one launch (instead of a negation, a subtraction and
// a second negation)
__global__ __launch_bounds__(256) void k_policy_combine(const float* loss_q, const float* loss_ppo,
                                                        const float* d_ratio, int B, float* loss_policy,
                                                        float* neg_d_ratio) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) neg_d_ratio[b] = -d_ratio[b];
  if (b == 0) loss_policy[0] = (-loss_q[0]) - loss_ppo[0];
}
// d/dlog_alpha of loss_alpha = exp(log_alpha) * (entropy - target_entropy) (msacl.py:429-437) as
// autograd forms it: mul's backward gives 1 * (entropy - target), exp's multiplies by its result
__global__ __launch_bounds__(64) void k_alpha_grad(const float* log_alpha, const float* entropy, float target,
                                                   float* grad) {
  if (threadIdx.x == 0) grad[0] = (entropy[0] - target) * expf(log_alpha[0]);
}

// The whole policy objective of a policy step (msacl.py:379-405) in ONE single-workgroup launch:
// loss_q = (min(q1, q2) - alpha logp).mean() and the entropy (k_policy_loss's body), the step-0
// importance ratio exp(lp_new - old_logp)[:, 0] (k_ratio0's), the normalised stability advantage
// with the PPO clip and its d_ratio (k_ppo_clip's body) and loss_policy = -loss_q - loss_ppo
// (k_policy_combine's): the same expressions in the same order, so the same bits as the four
// launches it replaces. Each thread's ratios are read back by the same thread (b = tid + k TPB).
__global__ __launch_bounds__(TPB) void k_policy_objective(const float* q1, const float* q2, const float* logp,
                                                          const float* log_alpha, const float* lp_new,
                                                          const float* old_logp, const float* adv_raw,
                                                          const double* stats, double n_total, float clip_eps, int B,
                                                          int n, float* loss_q, float* entropy, float* ratio,
                                                          float* adv, float* loss_ppo, float* d_ratio,
                                                          float* loss_policy) {
  __shared__ double sh[TPB];
  policy_loss_body(q1, q2, logp, log_alpha, (int64_t)B * n, loss_q, entropy, sh);
  for (int b = threadIdx.x; b < B; b += TPB) ratio[b] = expf(lp_new[(int64_t)b * n] - old_logp[(int64_t)b * n]);
  __syncthreads();
  ppo_clip_body(ratio, adv_raw, stats, n_total, clip_eps, B, adv, loss_ppo, d_ratio, sh);
  if (threadIdx.x == 0) loss_policy[0] = (-loss_q[0]) - loss_ppo[0];
}
// Its backward for an upstream gradient g of loss_policy (device scalar): d loss_q = -g through
// k_policy_loss_bwd's expressions (dq1, dq2, dlogp), d is_ratio = -g d_ratio through k_ratio0_bwd's
// (d lp_new: step 0 only). With g = 1 the same bits as the separate backward launches.
__global__ __launch_bounds__(256) void k_policy_objective_bwd(const float* q1, const float* q2,
                                                              const float* log_alpha, const float* ratio,
                                                              const float* d_ratio, const float* g, int B, int n,
                                                              float* dq1, float* dq2, float* dlogp, float* dlp_new) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t N = (int64_t)B * n;
  if (i >= N) return;
  const float alpha = expf(*log_alpha);
  const float gq = -*g;
  const float gg = gq * (1.0f / (float)N);
  const float a = q1[i], bq = q2[i];
  dq1[i] = a == bq ? gg / 2.0f : (a > bq ? 0.0f : gg);
  dq2[i] = a == bq ? gg / 2.0f : (a < bq ? 0.0f : gg);
  dlogp[i] = (-gg) * alpha;
  const int64_t b = i / n;
  dlp_new[i] = (i - b * n) == 0 ? (-(*g * d_ratio[b])) * ratio[b] : 0.0f;
}

// One policy step's objective AND its backward for the seed g = 1 (MSACL.model_update runs
// autograd.backward(loss_policy, 1)), plus the alpha gradient (msacl.py:429-437) from the same
// entropy: k_policy_objective, then k_policy_objective_bwd's element expressions with *g = 1 and
// k_alpha_grad's, in one single-workgroup launch (three launches before; the expressions and
// their order unchanged, so the same bits). alpha_grad may be null (no automatic alpha).
__global__ __launch_bounds__(TPB) void k_policy_objective_step(
    const float* q1, const float* q2, const float* logp, const float* log_alpha, const float* lp_new,
    const float* old_logp, const float* adv_raw, const double* stats, double n_total, float clip_eps, int B, int n,
    float* loss_q, float* entropy, float* ratio, float* adv, float* loss_ppo, float* d_ratio, float* loss_policy,
    float* dq1, float* dq2, float* dlogp, float* dlp_new, float target_entropy, float* alpha_grad) {
  __shared__ double sh[TPB];
  policy_loss_body(q1, q2, logp, log_alpha, (int64_t)B * n, loss_q, entropy, sh);
  for (int b = threadIdx.x; b < B; b += TPB) ratio[b] = expf(lp_new[(int64_t)b * n] - old_logp[(int64_t)b * n]);
  __syncthreads();
  ppo_clip_body(ratio, adv_raw, stats, n_total, clip_eps, B, adv, loss_ppo, d_ratio, sh);
  if (threadIdx.x == 0) loss_policy[0] = (-loss_q[0]) - loss_ppo[0];
  __syncthreads();  // d_ratio (written by the clip body) and entropy (thread 0) visible to all
  const int64_t N = (int64_t)B * n;
  const float alpha = expf(*log_alpha);
  const float g1 = 1.0f;
  const float gq = -g1;
  const float gg = gq * (1.0f / (float)N);
  constexpr int GU = 8;  // (loads first, as policy_loss_body)
  for (int64_t i0 = threadIdx.x; i0 < N; i0 += GU * TPB) {
    float x1[GU], x2[GU], dr[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int i = (int)(i0 + (int64_t)u * TPB), ic = i < N ? i : (int)N - 1;  // (N = B n < 2^31)
      const int b = ic / n;
      x1[u] = q1[ic];
      x2[u] = q2[ic];
      dr[u] = (ic - b * n) == 0 ? (-(g1 * d_ratio[b])) * ratio[b] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int64_t i = i0 + (int64_t)u * TPB;
      if (i < N) {
        const float a = x1[u], bq = x2[u];
        dq1[i] = a == bq ? gg / 2.0f : (a > bq ? 0.0f : gg);
        dq2[i] = a == bq ? gg / 2.0f : (a < bq ? 0.0f : gg);
        dlogp[i] = (-gg) * alpha;
        dlp_new[i] = dr[u];
      }
    }
  }
  if (alpha_grad && threadIdx.x == 0) alpha_grad[0] = (entropy[0] - target_entropy) * expf(log_alpha[0]);
}

// ------------------------------------------------------- logged scalars (msacl.py:211-222)
// [entropy, alpha, q1_mean, q2_mean, loss_q, loss_lya, loss_policy] in one launch (in place of
// an exp, a stack and the copy model_update snapshots).
__global__ void k_tb_pack(const float* entropy, const float* log_alpha, const float* q_means, const float* loss_q,
                          const float* loss_lya, const float* loss_policy, float* out) {
  if (threadIdx.x != 0) return;
  out[0] = entropy[0];
  out[1] = expf(log_alpha[0]);
  out[2] = q_means[0];
  out[3] = q_means[1];
  out[4] = loss_q[0];
  out[5] = loss_lya[0];
  out[6] = loss_policy[0];
}

// the same seven scalars into slot ctr % slots of a ring [slots][8] (element 7: the low 32 bits of
// the generation ctr, as float bits), ctr advanced: a replayed graph's logged values stay readable
// until `slots` later updates without a copy out of the graph's output
__global__ void k_tb_pack_ring(const float* entropy, const float* log_alpha, const float* q_means,
                               const float* loss_q, const float* loss_lya, const float* loss_policy, float* ring,
                               int64_t* ctr, int slots) {
  if (threadIdx.x != 0) return;
  const int64_t gen = ctr[0];
  float* out = ring + (gen % slots) * 8;
  out[0] = entropy[0];
  out[1] = expf(log_alpha[0]);
  out[2] = q_means[0];
  out[3] = q_means[1];
  out[4] = loss_q[0];
  out[5] = loss_lya[0];
  out[6] = loss_policy[0];
  out[7] = __uint_as_float((uint32_t)(uint64_t)gen);
  ctr[0] = gen + 1;
}

thread_local std::string g_merr;

}  // namespace

#define MH_CHECK_LAUNCH(name)                                    \
  do {                                                           \
    hipError_t _e = hipGetLastError();                           \
    if (_e != hipSuccess) return MH_EHIP;                        \
  } while (0)

extern "C" {

int mh_msacl_q_target_stats(const float* q1, const float* q2, const float* q1t, const float* q2t,
                            const float* next_logp, const float* rew, const float* done, const float* log_alpha,
                            const float* weight, float gamma, int32_t B, int32_t n, float* backup, float* dq1,
                            float* dq2, float* loss_out, float* abs_td, float* q_means, void* stream) {
  if (!q1 || !q2 || !q1t || !q2t || !next_logp || !rew || !done || !log_alpha || !backup || B <= 0 || n <= 0)
    return MH_EINVAL;
  const int64_t nb = ((int64_t)B + RPB - 1) / RPB;
  RowScratch* rs = nullptr;
  if (row_scratch(0, nb, &rs) != hipSuccess) return MH_EHIP;
  k_q_target<<<(unsigned)nb, RTPB, 0, (hipStream_t)stream>>>(q1, q2, q1t, q2t, next_logp, rew, done, log_alpha,
                                                             weight, gamma, B, n, backup, dq1, dq2, loss_out, abs_td,
                                                             q_means, rs->part, rs->arrive);
  MH_CHECK_LAUNCH("q_target");
  return MH_OK;
}

int mh_msacl_q_target(const float* q1, const float* q2, const float* q1t, const float* q2t,
                      const float* next_logp, const float* rew, const float* done, const float* log_alpha,
                      const float* weight, float gamma, int32_t B, int32_t n, float* backup, float* dq1,
                      float* dq2, float* loss_out, float* abs_td, void* stream) {
  return mh_msacl_q_target_stats(q1, q2, q1t, q2t, next_logp, rew, done, log_alpha, weight, gamma, B, n, backup,
                                 dq1, dq2, loss_out, abs_td, nullptr, stream);
}

int mh_msacl_tb_pack_ring(const float* entropy, const float* log_alpha, const float* q_means, const float* loss_q,
                          const float* loss_lya, const float* loss_policy, float* ring, int64_t* ctr, int32_t slots,
                          void* stream) {
  if (!entropy || !log_alpha || !q_means || !loss_q || !loss_lya || !loss_policy || !ring || !ctr || slots <= 0)
    return MH_EINVAL;
  k_tb_pack_ring<<<1, 64, 0, (hipStream_t)stream>>>(entropy, log_alpha, q_means, loss_q, loss_lya, loss_policy, ring,
                                                    ctr, slots);
  MH_CHECK_LAUNCH("tb_pack_ring");
  return MH_OK;
}

int mh_msacl_tb_pack(const float* entropy, const float* log_alpha, const float* q_means, const float* loss_q,
                     const float* loss_lya, const float* loss_policy, float* out, void* stream) {
  if (!entropy || !log_alpha || !q_means || !loss_q || !loss_lya || !loss_policy || !out) return MH_EINVAL;
  k_tb_pack<<<1, 64, 0, (hipStream_t)stream>>>(entropy, log_alpha, q_means, loss_q, loss_lya, loss_policy, out);
  MH_CHECK_LAUNCH("tb_pack");
  return MH_OK;
}

int mh_msacl_lyapunov(const float* logp, const float* old_logp, const float* lya_obs, const float* lya_obs2,
                      const float* obs, const float* obs2, const float* c, const float* w, const float* s,
                      float alpha1, float alpha2, float pos_scale, float diff_scale, int32_t B, int32_t n,
                      int32_t D, float* is_clip, float* esl, float* lya_diff, float* loss_out, float* d_lya_obs,
                      float* d_lya_obs2, void* stream) {
  if (!logp || !old_logp || !lya_obs || !lya_obs2 || !obs || !obs2 || !c || !w || !s || !is_clip || !esl ||
      !lya_diff || !d_lya_obs || !d_lya_obs2 || B <= 0 || n <= 0 || D <= 0)
    return MH_EINVAL;
  const int64_t nb = ((int64_t)B + RPB - 1) / RPB;
  RowScratch* rs = nullptr;
  if (row_scratch(1, nb, &rs) != hipSuccess) return MH_EHIP;
#define MH_LYA(DT)                                                                                     \
  k_lyapunov<DT><<<(unsigned)nb, RTPB, 0, (hipStream_t)stream>>>(                                      \
      logp, old_logp, lya_obs, lya_obs2, obs, obs2, c, w, s, alpha1, alpha2, pos_scale, diff_scale, B, n, D, \
      is_clip, esl, lya_diff, loss_out, d_lya_obs, d_lya_obs2, rs->part, rs->arrive)
  switch (D) {
    case 1: MH_LYA(1); break;
    case 2: MH_LYA(2); break;
    case 3: MH_LYA(3); break;
    case 4: MH_LYA(4); break;
    case 5: MH_LYA(5); break;
    case 6: MH_LYA(6); break;
    case 7: MH_LYA(7); break;
    case 8: MH_LYA(8); break;
    case 9: MH_LYA(9); break;
    case 10: MH_LYA(10); break;
    case 11: MH_LYA(11); break;
    case 12: MH_LYA(12); break;
    case 13: MH_LYA(13); break;
    case 14: MH_LYA(14); break;
    case 15: MH_LYA(15); break;
    case 16: MH_LYA(16); break;
    default: MH_LYA(0); break;
  }
#undef MH_LYA
  MH_CHECK_LAUNCH("lyapunov");
  return MH_OK;
}

int mh_msacl_stability_adv(const float* lya_obs0, const float* lya_obs2, const float* w, const float* s,
                           int32_t B, int32_t n, float* adv_raw, double* stats_out, void* stream) {
  if (!lya_obs0 || !lya_obs2 || !w || !s || !adv_raw || !stats_out || B <= 0 || n <= 0) return MH_EINVAL;
  k_stab_adv<<<1, TPB, 0, (hipStream_t)stream>>>(lya_obs0, lya_obs2, w, s, B, n, adv_raw, stats_out);
  MH_CHECK_LAUNCH("stab_adv");
  return MH_OK;
}

int mh_msacl_ppo_clip(const float* ratio, const float* adv_raw, const double* stats, double n_total,
                      float clip_eps, int32_t B, float* adv, float* loss_out, float* d_ratio, void* stream) {
  if (!ratio || !adv_raw || !stats || !adv || !loss_out || !d_ratio || B <= 0 || n_total < 2.0) return MH_EINVAL;
  k_ppo_clip<<<1, TPB, 0, (hipStream_t)stream>>>(ratio, adv_raw, stats, n_total, clip_eps, B, adv, loss_out,
                                                 d_ratio);
  MH_CHECK_LAUNCH("ppo_clip");
  return MH_OK;
}

int mh_msacl_policy_loss(const float* q1, const float* q2, const float* logp, const float* log_alpha, int64_t N,
                         float* loss_out, float* entropy_out, void* stream) {
  if (!q1 || !q2 || !logp || !log_alpha || !loss_out || !entropy_out || N <= 0) return MH_EINVAL;
  k_policy_loss<<<1, TPB, 0, (hipStream_t)stream>>>(q1, q2, logp, log_alpha, N, loss_out, entropy_out);
  MH_CHECK_LAUNCH("policy_loss");
  return MH_OK;
}

int mh_msacl_policy_loss_backward(const float* q1, const float* q2, const float* log_alpha, const float* g_loss,
                                  int64_t N, float* dq1, float* dq2, float* dlogp, void* stream) {
  if (!q1 || !q2 || !log_alpha || !g_loss || !dq1 || !dq2 || !dlogp || N <= 0) return MH_EINVAL;
  k_policy_loss_bwd<<<(unsigned)((N + 255) / 256), 256, 0, (hipStream_t)stream>>>(q1, q2, log_alpha, g_loss, N, dq1,
                                                                                  dq2, dlogp);
  MH_CHECK_LAUNCH("policy_loss_bwd");
  return MH_OK;
}

int mh_msacl_ratio0(const float* logp_new, const float* old_logp, int32_t B, int32_t n, float* ratio_out,
                    void* stream) {
  if (!logp_new || !old_logp || !ratio_out || B <= 0 || n <= 0) return MH_EINVAL;
  k_ratio0<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(logp_new, old_logp, B, n, ratio_out);
  MH_CHECK_LAUNCH("ratio0");
  return MH_OK;
}

int mh_msacl_ratio0_backward(const float* ratio, const float* g_ratio, int32_t B, int32_t n, float* d_logp_new,
                             void* stream) {
  if (!ratio || !g_ratio || !d_logp_new || B <= 0 || n <= 0) return MH_EINVAL;
  const int64_t total = (int64_t)B * n;
  k_ratio0_bwd<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(ratio, g_ratio, B, n, d_logp_new);
  MH_CHECK_LAUNCH("ratio0_bwd");
  return MH_OK;
}

int mh_msacl_policy_objective(const float* q1, const float* q2, const float* logp, const float* log_alpha,
                              const float* lp_new, const float* old_logp, const float* adv_raw, const double* stats,
                              double n_total, float clip_eps, int32_t B, int32_t n, float* loss_q, float* entropy,
                              float* ratio, float* adv, float* loss_ppo, float* d_ratio, float* loss_policy,
                              void* stream) {
  if (!q1 || !q2 || !logp || !log_alpha || !lp_new || !old_logp || !adv_raw || !stats || !loss_q || !entropy ||
      !ratio || !adv || !loss_ppo || !d_ratio || !loss_policy || B <= 0 || n <= 0)
    return MH_EINVAL;
  k_policy_objective<<<1, TPB, 0, (hipStream_t)stream>>>(q1, q2, logp, log_alpha, lp_new, old_logp, adv_raw, stats,
                                                         n_total, clip_eps, B, n, loss_q, entropy, ratio, adv,
                                                         loss_ppo, d_ratio, loss_policy);
  MH_CHECK_LAUNCH("policy_objective");
  return MH_OK;
}

int mh_msacl_policy_objective_step(const float* q1, const float* q2, const float* logp, const float* log_alpha,
                                   const float* lp_new, const float* old_logp, const float* adv_raw,
                                   const double* stats, double n_total, float clip_eps, int32_t B, int32_t n,
                                   float* loss_q, float* entropy, float* ratio, float* adv, float* loss_ppo,
                                   float* d_ratio, float* loss_policy, float* dq1, float* dq2, float* dlogp,
                                   float* dlp_new, float target_entropy, float* alpha_grad, void* stream) {
  if (!q1 || !q2 || !logp || !log_alpha || !lp_new || !old_logp || !adv_raw || !stats || !loss_q || !entropy ||
      !ratio || !adv || !loss_ppo || !d_ratio || !loss_policy || !dq1 || !dq2 || !dlogp || !dlp_new || B <= 0 ||
      n <= 0)
    return MH_EINVAL;
  k_policy_objective_step<<<1, TPB, 0, (hipStream_t)stream>>>(
      q1, q2, logp, log_alpha, lp_new, old_logp, adv_raw, stats, n_total, clip_eps, B, n, loss_q, entropy, ratio, adv,
      loss_ppo, d_ratio, loss_policy, dq1, dq2, dlogp, dlp_new, target_entropy, alpha_grad);
  MH_CHECK_LAUNCH("policy_objective_step");
  return MH_OK;
}

int mh_msacl_policy_objective_backward(const float* q1, const float* q2, const float* log_alpha, const float* ratio,
                                       const float* d_ratio, const float* g_loss, int32_t B, int32_t n, float* dq1,
                                       float* dq2, float* dlogp, float* dlp_new, void* stream) {
  if (!q1 || !q2 || !log_alpha || !ratio || !d_ratio || !g_loss || !dq1 || !dq2 || !dlogp || !dlp_new || B <= 0 ||
      n <= 0)
    return MH_EINVAL;
  const int64_t N = (int64_t)B * n;
  k_policy_objective_bwd<<<(unsigned)((N + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      q1, q2, log_alpha, ratio, d_ratio, g_loss, B, n, dq1, dq2, dlogp, dlp_new);
  MH_CHECK_LAUNCH("policy_objective_bwd");
  return MH_OK;
}

int mh_msacl_policy_combine(const float* loss_q, const float* loss_ppo, const float* d_ratio, int32_t B,
                            float* loss_policy, float* neg_d_ratio, void* stream) {
  if (!loss_q || !loss_ppo || !d_ratio || !loss_policy || !neg_d_ratio || B <= 0) return MH_EINVAL;
  k_policy_combine<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(loss_q, loss_ppo, d_ratio, B,
                                                                                 loss_policy, neg_d_ratio);
  MH_CHECK_LAUNCH("policy_combine");
  return MH_OK;
}

int mh_msacl_alpha_grad(const float* log_alpha, const float* entropy, float target_entropy, float* grad,
                        void* stream) {
  if (!log_alpha || !entropy || !grad) return MH_EINVAL;
  k_alpha_grad<<<1, 64, 0, (hipStream_t)stream>>>(log_alpha, entropy, target_entropy, grad);
  MH_CHECK_LAUNCH("alpha_grad");
  return MH_OK;
}

}  // extern "C"
