// optim.hip — Adam over one network's FLAT parameter buffer (gfx950).
//
// The update step of torch.optim.Adam (defaults of every reference algorithm: betas (0.9, 0.999),
// eps 1e-8, no weight decay, no amsgrad; RL/algorithm/*.py `Adam(net.parameters(), lr=...)`):
//   t += 1
//   m = lerp(m, g, 1 - b1)                 (torch lerp: m + w (g - m) for w < 0.5)
//   v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with the network's parameters, gradients and both moments each laid out contiguously (the
// Python side re-points every nn.Parameter's .data / .grad at views of the flat buffers), so one
// launch updates a whole network and zeroes its gradients for the next backward, where the
// PyTorch optimiser issues multi-tensor kernels plus a gradient fill per network. The step count
// lives on the device (incremented by the last workgroup to finish) so the update can be
// captured into a HIP graph; the bias corrections are formed in float64 from it, as PyTorch forms
// them in Python floats. HBM-bound: 4 arrays read, 4 written (the gradient zeroed).
#include "rollout.h"

namespace mh {

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, int64_t n, float lr, float b1, float b2,
                                              float eps, int zero_grad, int64_t* __restrict__ step,
                                              uint32_t* __restrict__ ticket) {
  const int64_t t = *step + 1;
  const double bc1 = 1.0 - pow((double)b1, (double)t);
  const double bc2 = 1.0 - pow((double)b2, (double)t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = 1.0f - b1, w2 = 1.0f - b2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i];
    vi = vi * b2 + w2 * (gi * gi);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
    m[i] = mi;
    v[i] = vi;
    if (zero_grad) g[i] = 0.0f;
  }
  // the last workgroup to finish advances the step counter (every workgroup read the old one)
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const uint32_t done = atomicAdd(ticket, 1u);
    if (done == gridDim.x - 1) {
      *step = t;
      *ticket = 0u;
    }
  }
}

hipError_t launch_adam(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
                       int zero_grad, int64_t* step, uint32_t* ticket, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t want = (n + 255) / 256;
  const int grid = (int)(want < 1024 ? want : 1024);
  k_adam<<<grid, 256, 0, st>>>(p, g, m, v, n, lr, b1, b2, eps, zero_grad, step, ticket);
  return hipGetLastError();
}

}  // namespace mh
