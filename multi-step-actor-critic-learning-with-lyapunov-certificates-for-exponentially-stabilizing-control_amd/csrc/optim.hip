// optim.hip — one Adam step over a list of parameter tensors in ONE launch (gfx950).
//
// torch.optim.Adam as every reference algorithm builds it (RL/algorithm/*.py
// `Adam(net.parameters(), lr=...)`: betas (0.9, 0.999), eps 1e-8, no weight decay, no amsgrad),
// in the form of PyTorch's fused / capturable implementation (float32 step counter on the
// device, bias corrections formed in float32 from it):
//   t += 1
//   m = lerp(m, g, 1 - b1)
//   v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// PyTorch's multi-tensor kernel gives each 65,536-element chunk of a tensor ONE workgroup, so a
// 256 x 256 MLP's update runs on a handful of workgroups (31 us per optimiser step, measured in
// the MSACL update) plus a separate step-count increment kernel. Here the tensors of one
// optimiser (pointer table passed by value in the kernel arguments: graph-capturable, no upload)
// are one flat index space over a full grid, and the step counters are advanced in the same
// launch by the last workgroup to finish (every workgroup has read the old count by then).
// HBM-bound: 4 arrays read, 3 written per element.
#include "rollout.h"

namespace mh {

// one element of the Adam update (the same float32 expressions for every layout)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float w2, float fb2,
                                          float bc2, float step_size, float feps) {
  m = m + w1 * (g - m);  // exp_avg.lerp_(grad, 1 - beta1)
  v = fb2 * v + w2 * (g * g);
  const float denom = sqrtf(v) / bc2 + feps;
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(256) void k_adam_multi(AdamList L, double b1, double b2, double eps,
                                                    uint32_t* __restrict__ ticket) {
  // the scalars as PyTorch forms them from the Python floats: (1 - beta) and the bias
  // corrections in double, each rounded once to float32 where the element math uses it; one
  // step counter per tensor (a tensor without a gradient on some steps has its own count)
  __shared__ float s_step_size[ADAM_MAX_TENSORS], s_bc2[ADAM_MAX_TENSORS], s_t[ADAM_MAX_TENSORS];
  if ((int)threadIdx.x < L.n) {
    const float t = *L.step[threadIdx.x] + 1.0f;
    s_t[threadIdx.x] = t;
    s_step_size[threadIdx.x] = (float)(L.lr[threadIdx.x] / (1.0 - pow(b1, (double)t)));
    s_bc2[threadIdx.x] = (float)sqrt(1.0 - pow(b2, (double)t));
  }
  __syncthreads();
  const float w1 = (float)(1.0 - b1), w2 = (float)(1.0 - b2);
  const float fb2 = (float)b2, feps = (float)eps;
  const int64_t total = L.start[L.n];
  // work units: 4-element vectors of the tensors that allow them (16-byte aligned, numel % 4 ==
  // 0), single elements of the rest; a thread's grid-stride units only move forward through the
  // tensor list, so its tensor index is carried from one unit to the next
  int k = 0;
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < total; u += (int64_t)gridDim.x * 256) {
    while (k + 1 < L.n && u >= L.start[k + 1]) ++k;
    const int64_t j = u - L.start[k];
    const float ss = s_step_size[k], bc2 = s_bc2[k];
    if (L.vec[k]) {
      float4 p = reinterpret_cast<const float4*>(L.p[k])[j];
      const float4 g = reinterpret_cast<const float4*>(L.g[k])[j];
      float4 m = reinterpret_cast<const float4*>(L.m[k])[j];
      float4 v = reinterpret_cast<const float4*>(L.v[k])[j];
      adam_elem(p.x, g.x, m.x, v.x, w1, w2, fb2, bc2, ss, feps);
      adam_elem(p.y, g.y, m.y, v.y, w1, w2, fb2, bc2, ss, feps);
      adam_elem(p.z, g.z, m.z, v.z, w1, w2, fb2, bc2, ss, feps);
      adam_elem(p.w, g.w, m.w, v.w, w1, w2, fb2, bc2, ss, feps);
      reinterpret_cast<float4*>(L.p[k])[j] = p;
      reinterpret_cast<float4*>(L.m[k])[j] = m;
      reinterpret_cast<float4*>(L.v[k])[j] = v;
    } else {
      float p = L.p[k][j], m = L.m[k][j], v = L.v[k][j];
      adam_elem(p, L.g[k][j], m, v, w1, w2, fb2, bc2, ss, feps);
      L.p[k][j] = p;
      L.m[k][j] = m;
      L.v[k][j] = v;
    }
  }
  // the last workgroup to finish advances every step counter. The arrival count is RELAXED: the
  // only ordering needed is that every workgroup has READ the old count before the last one
  // writes the new one, and each workgroup's read returned its value (consumed into s_t above,
  // before the barrier) before its arrival. No data is handed between workgroups, so no
  // agent-scope release / acquire (each one an L2 writeback + invalidate, ~3.5 us: with one per
  // workgroup this launch took 12-24 us for 70-140 k parameters)
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      for (int q = 0; q < L.n; ++q) *L.step[q] = s_t[q];
      *ticket = 0u;
    }
  }
}

hipError_t launch_adam_multi(const AdamList& L, double b1, double b2, double eps, uint32_t* ticket, hipStream_t st) {
  if (L.n <= 0) return hipSuccess;
  const int64_t total = L.start[L.n];
  const int64_t want = (total + 255) / 256;
  const int grid = (int)(want < 1 ? 1 : (want < 2048 ? want : 2048));
  k_adam_multi<<<grid, 256, 0, st>>>(L, b1, b2, eps, ticket);
  return hipGetLastError();
}

// Polyak averaging of target networks (sac.py:204-217, msacl.py:445-460):
//   p_t.mul_(polyak); p_t.add_((1 - polyak) * p)      (both scalars float32, two roundings)
// over a tensor list in one launch (PyTorch: three multi-tensor kernels per network).
__global__ __launch_bounds__(256) void k_polyak_multi(PolyakList L, float a, float b) {
  const int64_t total = L.start[L.n];
  int k = 0;  // (units as in k_adam_multi; the tensor index carried forward)
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < total; u += (int64_t)gridDim.x * 256) {
    while (k + 1 < L.n && u >= L.start[k + 1]) ++k;
    const int64_t j = u - L.start[k];
    if (L.vec[k]) {
      float4 t = reinterpret_cast<const float4*>(L.t[k])[j];
      const float4 s = reinterpret_cast<const float4*>(L.s[k])[j];
      t.x = t.x * a + s.x * b;
      t.y = t.y * a + s.y * b;
      t.z = t.z * a + s.z * b;
      t.w = t.w * a + s.w * b;
      reinterpret_cast<float4*>(L.t[k])[j] = t;
    } else {
      const float t = L.t[k][j] * a;
      L.t[k][j] = t + L.s[k][j] * b;
    }
  }
}

hipError_t launch_polyak_multi(const PolyakList& L, double polyak, hipStream_t st) {
  if (L.n <= 0) return hipSuccess;
  const int64_t total = L.start[L.n];
  if (total <= 0) return hipSuccess;
  const int64_t want = (total + 255) / 256;
  const int grid = (int)(want < 2048 ? want : 2048);
  k_polyak_multi<<<grid, 256, 0, st>>>(L, (float)polyak, (float)(1.0 - polyak));
  return hipGetLastError();
}

}  // namespace mh
