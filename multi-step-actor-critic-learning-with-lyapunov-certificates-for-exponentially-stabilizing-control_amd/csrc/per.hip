// per.hip — prioritized replay over the device window store (new component: the reference
// trainer calls buffer.update_batch(idx, priority) at RL/trainer/nstep_off_serial_trainer.py:93-95
// but ships no prioritized buffer). Proportional prioritisation p_i = (|td_i| + eps)^alpha over a
// float64 sum-tree in heap layout (tree[1] = root, leaves at [pow2, 2*pow2)).
//
// Rebuild is blocked for the MI355X memory system: kernel A reduces 1024-leaf subtrees
// entirely in LDS (one workgroup each, every leaf read once, coalesced), kernel B (one
// workgroup) builds the levels above the subtree roots. No atomics: the tree is bitwise
// deterministic for a given leaf vector.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "msacl_hip.h"
#include "philox.h"

namespace {

constexpr int SUB = 1024;  // leaves per subtree workgroup

__global__ __launch_bounds__(512) void k_tree_sub(double* tree, int64_t pow2) {
  __shared__ double sh[SUB];
  const int64_t base = (int64_t)blockIdx.x * SUB;
  for (int i = threadIdx.x; i < SUB; i += 512) sh[i] = tree[pow2 + base + i];
  __syncthreads();
  // level by level: width halves; heap index of node j at level with `width` nodes
  int64_t level_start = pow2 / 2;  // heap index of the first node one level above the leaves
  int64_t off = base / 2;
  for (int width = SUB / 2; width >= 1; width >>= 1) {
    double v0 = 0.0;
    const int t = threadIdx.x;
    if (t < width) v0 = sh[2 * t] + sh[2 * t + 1];
    __syncthreads();
    if (t < width) {
      sh[t] = v0;
      tree[level_start + off + t] = v0;
    }
    __syncthreads();
    level_start >>= 1;
    off >>= 1;
  }
}

// levels above the subtree roots (nodes [1, pow2/SUB)) — one workgroup
__global__ __launch_bounds__(1024) void k_tree_top(double* tree, int64_t top) {
  // top = number of subtree roots (pow2 / SUB), a power of two; nodes [top, 2*top) are ready
  for (int64_t width = top / 2; width >= 1; width >>= 1) {
    for (int64_t j = threadIdx.x; j < width; j += 1024) tree[width + j] = tree[2 * (width + j)] + tree[2 * (width + j) + 1];
    __syncthreads();
  }
}

// small trees (pow2 <= SUB): single workgroup full rebuild
__global__ __launch_bounds__(1024) void k_tree_small(double* tree, int64_t pow2) {
  for (int64_t width = pow2 / 2; width >= 1; width >>= 1) {
    for (int64_t j = threadIdx.x; j < width; j += 1024) tree[width + j] = tree[2 * (width + j)] + tree[2 * (width + j) + 1];
    __syncthreads();
  }
}

hipError_t rebuild(double* tree, int64_t pow2, hipStream_t st) {
  if (pow2 <= SUB) {
    k_tree_small<<<1, 1024, 0, st>>>(tree, pow2);
  } else {
    k_tree_sub<<<(int)(pow2 / SUB), 512, 0, st>>>(tree, pow2);
    k_tree_top<<<1, 1024, 0, st>>>(tree, pow2 / SUB);
  }
  return hipGetLastError();
}

__global__ void k_update_leaves(double* tree, int64_t pow2, const int64_t* idx, const float* prio, int64_t count,
                                float alpha, float eps, double* max_prio) {
  // one workgroup: deterministic max
  __shared__ double sh[1024];
  double m = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += 1024) {
    const double p = pow((double)fabsf(prio[i]) + (double)eps, (double)alpha);
    tree[pow2 + idx[i]] = p;
    m = fmax(m, p);
  }
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int off = 512; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + off]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *max_prio = fmax(*max_prio, sh[0]);
}

__global__ __launch_bounds__(256) void k_set_new(double* tree, int64_t pow2, const int64_t* before,
                                                const int64_t* after, int64_t capacity, const double* max_prio) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= capacity) return;
  int64_t cnt = after[2] - before[2];
  if (cnt <= 0) return;
  if (cnt > capacity) cnt = capacity;
  // rows written: the cnt rows ending just before after[0] (mod capacity)
  const int64_t end = after[0];
  const int64_t rel = ((end - 1 - r) % capacity + capacity) % capacity;  // distance back from end-1
  if (rel < cnt) tree[pow2 + r] = *max_prio > 0.0 ? *max_prio : 1.0;
}

__global__ __launch_bounds__(256) void k_sample(const double* tree, int64_t pow2, const int64_t* cursor, uint64_t seed,
                                               uint64_t counter, int64_t batch, float beta, int64_t* idx,
                                               float* weight) {
  __shared__ double sh[256];
  const double total = tree[1];
  const int64_t size = cursor[1];
  const double seg = total / (double)batch;
  double wmax = 0.0;
  for (int64_t b = threadIdx.x; b < batch; b += 256) {
    const mh::Rng r = mh::make_rng(seed, (uint64_t)b, counter);
    const mh::u32x4 q = r.draw(9);
    double u = ((double)b + mh::u01(q.x)) * seg;
    int64_t node = 1;
    while (node < pow2) {
      const double left = tree[2 * node];
      if (u < left) {
        node = 2 * node;
      } else {
        u -= left;
        node = 2 * node + 1;
      }
    }
    int64_t leaf = node - pow2;
    if (leaf >= size) leaf = size > 0 ? size - 1 : 0;
    idx[b] = leaf;
    const double p = tree[pow2 + leaf] / (total > 0.0 ? total : 1.0);
    const double wv = pow((double)(size > 0 ? size : 1) * (p > 0.0 ? p : 1e-300), -(double)beta);
    weight[b] = (float)wv;
    wmax = fmax(wmax, wv);
  }
  sh[threadIdx.x] = wmax;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + off]);
    __syncthreads();
  }
  const double mx = sh[0] > 0.0 ? sh[0] : 1.0;
  for (int64_t b = threadIdx.x; b < batch; b += 256) weight[b] = (float)((double)weight[b] / mx);
}

}  // namespace

extern "C" {

int mh_per_update(double* tree, int64_t pow2, const int64_t* idx, const float* prio, int64_t count, float alpha,
                  float eps, double* max_prio, void* stream) {
  if (!tree || !idx || !prio || !max_prio || pow2 <= 0 || (pow2 & (pow2 - 1))) return MH_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (count > 0) {
    k_update_leaves<<<1, 1024, 0, st>>>(tree, pow2, idx, prio, count, alpha, eps, max_prio);
    if (hipGetLastError() != hipSuccess) return MH_EHIP;
  }
  return rebuild(tree, pow2, st) == hipSuccess ? MH_OK : MH_EHIP;
}

int mh_per_set_new(double* tree, int64_t pow2, const int64_t* cursor_before, const int64_t* cursor_after,
                   int64_t capacity, const double* max_prio, void* stream) {
  if (!tree || !cursor_before || !cursor_after || !max_prio || capacity <= 0 || capacity > pow2) return MH_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  k_set_new<<<(int)((capacity + 255) / 256), 256, 0, st>>>(tree, pow2, cursor_before, cursor_after, capacity,
                                                          max_prio);
  if (hipGetLastError() != hipSuccess) return MH_EHIP;
  return rebuild(tree, pow2, st) == hipSuccess ? MH_OK : MH_EHIP;
}

int mh_per_sample(const double* tree, int64_t pow2, const int64_t* cursor, uint64_t seed, uint64_t counter,
                  int64_t batch, float beta, int64_t* idx_out, float* weight_out, void* stream) {
  if (!tree || !cursor || !idx_out || !weight_out || batch <= 0) return MH_EINVAL;
  k_sample<<<1, 256, 0, (hipStream_t)stream>>>(tree, pow2, cursor, seed, counter, batch, beta, idx_out, weight_out);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_EHIP;
}

}  // extern "C"
