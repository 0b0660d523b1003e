// per.hip — prioritized replay over the device window store (new component: the reference
// trainer calls buffer.update_batch(idx, priority) at RL/trainer/nstep_off_serial_trainer.py:93-95
// but ships no prioritized buffer). Proportional prioritisation p_i = (|td_i| + eps)^alpha over a
// float64 sum-tree in heap layout (tree[1] = root, leaves at [pow2, 2*pow2)); every internal node
// is exactly tree[2k] + tree[2k+1] (one f64 add, the order a level-by-level rebuild uses).
//
// Work per call is proportional to what changed, never to the capacity:
//   mh_per_update   B leaves -> leaf-to-root recompute of their ancestors, one workgroup,
//                   log2(pow2) barrier-separated levels (O(B log N)). Duplicate leaves in one
//                   batch resolve to the LAST entry (sequential last-write-wins), found in
//                   O(B) with the touched leaf slots as owner tags (atomic max of the entry
//                   index, then a compare-and-swap of the winner's tag for its priority).
//   mh_per_set_new  the rows the rollout just appended (a contiguous FIFO arc read from the
//                   device cursors) get the running max priority; only the 1024-leaf subtrees
//                   the arc touches are rebuilt (in LDS), then the ~pow2/1024 nodes above them
//                   (O(new + N/1024)). The grid covers every subtree (the count is device-side,
//                   so the launch is graph-capturable); untouched workgroups exit at once.
//   mh_per_sample   stratified proportional draws; the top 11 tree levels are staged in LDS so
//                   only the lower levels of each descent go to L2/HBM.
// For given inputs the tree, the indices and the weights are bitwise deterministic (the update's
// owner-tag atomics decide only WHICH entry writes a leaf, always the last one).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "msacl_hip.h"
#include "philox.h"

namespace {

constexpr int SUB = 1024;        // leaves per subtree workgroup (set_new)
constexpr int TOPC = 2048;       // heap nodes [1, TOPC) staged in LDS by the sampler
constexpr int UPD = 1024;        // update workgroup size
constexpr int LEAF_CACHE = 4096; // batch leaves kept in LDS by the update kernel

__device__ __forceinline__ double leaf_priority(float td, float alpha, float eps) {
  return pow((double)fabsf(td) + (double)eps, (double)alpha);
}

// ---------------------------------------------------------------- update (leaf-to-root)
__global__ __launch_bounds__(UPD) void k_update(double* tree, int64_t pow2, int log2p, const int64_t* idx,
                                                const float* prio, int64_t count, float alpha, float eps,
                                                double* max_prio) {
  __shared__ int64_t leaves[LEAF_CACHE];
  __shared__ double red[UPD];
  const int tid = threadIdx.x;
  double m = 0.0;
  // last-write-wins (entry i loses if a later entry names the same leaf), O(count): every
  // touched leaf slot is about to be overwritten, so it serves as its own owner slot first —
  // cleared, then the largest entry index + 1 naming it is kept by an L2 atomic max, and the
  // entry whose index it holds is the winner (one workgroup: barriers order the three passes)
  unsigned long long* owner = reinterpret_cast<unsigned long long*>(tree + pow2);
  for (int64_t i = tid; i < count; i += UPD) {
    const int64_t my = idx[i];
    if (my >= 0 && my < pow2) atomicExch(owner + my, 0ull);
  }
  __threadfence();
  __syncthreads();
  for (int64_t i = tid; i < count; i += UPD) {
    const int64_t my = idx[i];
    if (my >= 0 && my < pow2) atomicMax(owner + my, (unsigned long long)(i + 1));
  }
  __threadfence();
  __syncthreads();
  for (int64_t c0 = 0; c0 < count; c0 += UPD) {
    const int64_t i = c0 + tid;
    const int64_t my = i < count ? idx[i] : -1;
    const bool valid = my >= 0 && my < pow2;
    if (valid) {
      const double p = leaf_priority(prio[i], alpha, eps);
      m = fmax(m, p);
      // the winner swaps its own tag for the priority; every other entry's swap fails
      atomicCAS(owner + my, (unsigned long long)(i + 1), __double_as_longlong(p));
    }
    if (i < LEAF_CACHE && i < count) leaves[i] = valid ? my : -1;
  }
  __threadfence();
  // ancestors, one level per barrier: every node on a touched path is recomputed from its two
  // children, which are final after the previous level (several entries may share a node; they
  // store the same value)
  for (int lv = 1; lv <= log2p; ++lv) {
    __syncthreads();
    for (int64_t i = tid; i < count; i += UPD) {
      const int64_t my = i < LEAF_CACHE ? leaves[i] : idx[i];
      if (my < 0 || my >= pow2) continue;
      const int64_t node = (pow2 + my) >> lv;
      tree[node] = tree[2 * node] + tree[2 * node + 1];
    }
  }
  red[tid] = m;
  __syncthreads();
  for (int off = UPD / 2; off > 0; off >>= 1) {
    if (tid < off) red[tid] = fmax(red[tid], red[tid + off]);
    __syncthreads();
  }
  if (tid == 0) *max_prio = fmax(*max_prio, red[0]);
}

// ---------------------------------------------------------------- new rows (FIFO arc)
struct Arc {
  int64_t start, cnt;  // rows [start, start + cnt) mod capacity; cnt <= 0: nothing new
};

__device__ __forceinline__ Arc new_arc(const int64_t* before, const int64_t* after, int64_t capacity) {
  int64_t cnt = after[2] - before[2];
  if (cnt > capacity) cnt = capacity;
  const int64_t start = cnt > 0 ? ((after[0] - cnt) % capacity + capacity) % capacity : 0;
  return Arc{start, cnt};
}

__device__ __forceinline__ bool in_arc(const Arc& a, int64_t r, int64_t capacity) {
  return a.cnt > 0 && r < capacity && ((r - a.start) % capacity + capacity) % capacity < a.cnt;
}

// rebuild one subtree of `nleaf` leaves in LDS (sh holds the leaves); writes every internal node
// of the subtree (heap indices derived from the first leaf's heap index `first`)
__device__ void subtree_reduce(double* sh, double* tree, int64_t first, int nleaf) {
  int64_t level_first = first;
  for (int width = nleaf / 2; width >= 1; width >>= 1) {
    double v = 0.0;
    const int t = threadIdx.x;
    if (t < width) v = sh[2 * t] + sh[2 * t + 1];
    __syncthreads();
    level_first >>= 1;
    if (t < width) {
      sh[t] = v;
      tree[level_first + t] = v;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(SUB / 2) void k_new_sub(double* tree, int64_t pow2, const int64_t* before,
                                                     const int64_t* after, int64_t capacity,
                                                     const double* max_prio) {
  __shared__ double sh[SUB];
  const Arc a = new_arc(before, after, capacity);
  const int64_t base = (int64_t)blockIdx.x * SUB;
  if (a.cnt <= 0 || base >= capacity) return;
  const int64_t end = base + SUB < capacity ? base + SUB : capacity;
  // the arc meets [base, end) iff it starts inside it or covers its first row
  if (!((a.start >= base && a.start < end) || in_arc(a, base, capacity))) return;
  const double mp = *max_prio > 0.0 ? *max_prio : 1.0;
  for (int i = threadIdx.x; i < SUB; i += SUB / 2) {
    const int64_t r = base + i;
    double v = tree[pow2 + r];
    if (in_arc(a, r, capacity)) {
      v = mp;
      tree[pow2 + r] = v;
    }
    sh[i] = v;
  }
  __syncthreads();
  subtree_reduce(sh, tree, pow2 + base, SUB);
}

// levels above the subtree roots: nodes [1, top) from [top, 2 top), one workgroup
__global__ __launch_bounds__(1024) void k_new_top(double* tree, int64_t top, const int64_t* before,
                                                  const int64_t* after) {
  if (after[2] - before[2] <= 0) return;
  for (int64_t width = top / 2; width >= 1; width >>= 1) {
    for (int64_t j = threadIdx.x; j < width; j += 1024) tree[width + j] = tree[2 * (width + j)] + tree[2 * (width + j) + 1];
    __syncthreads();
  }
}

// whole tree in one workgroup (pow2 <= SUB)
__global__ __launch_bounds__(SUB) void k_new_small(double* tree, int64_t pow2, const int64_t* before,
                                                   const int64_t* after, int64_t capacity,
                                                   const double* max_prio) {
  __shared__ double sh[SUB];
  const Arc a = new_arc(before, after, capacity);
  if (a.cnt <= 0) return;
  const double mp = *max_prio > 0.0 ? *max_prio : 1.0;
  for (int i = threadIdx.x; i < pow2; i += SUB) {
    double v = tree[pow2 + i];
    if (in_arc(a, i, capacity)) {
      v = mp;
      tree[pow2 + i] = v;
    }
    sh[i] = v;
  }
  __syncthreads();
  subtree_reduce(sh, tree, pow2, (int)pow2);
}

// ---------------------------------------------------------------- sampling
__global__ __launch_bounds__(256) void k_sample(const double* tree, int64_t pow2, const int64_t* cursor, uint64_t seed,
                                               uint64_t counter, int64_t batch, float beta, int64_t* idx,
                                               float* weight) {
  __shared__ double top[TOPC];
  __shared__ double sh[256];
  const int64_t ncache = 2 * pow2 < TOPC ? 2 * pow2 : TOPC;
  for (int64_t i = threadIdx.x; i < ncache; i += 256) top[i] = tree[i];
  __syncthreads();
  const double total = top[1];
  const int64_t size = cursor[1];
  const double seg = total / (double)batch;
  double wmax = 0.0;
  for (int64_t b = threadIdx.x; b < batch; b += 256) {
    const mh::Rng r = mh::make_rng(seed, (uint64_t)b, counter);
    const mh::u32x4 q = r.draw(9);
    double u = ((double)b + mh::u01(q.x)) * seg;
    int64_t node = 1;
    while (node < pow2) {
      const int64_t l = 2 * node;
      const double left = l < ncache ? top[l] : tree[l];
      if (u < left) {
        node = l;
      } else {
        u -= left;
        node = l + 1;
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
  for (int64_t b = threadIdx.x; b < batch; b += 256) {
    const int64_t leaf = idx[b];
    const double p = tree[pow2 + leaf] / (total > 0.0 ? total : 1.0);
    const double wv = pow((double)(size > 0 ? size : 1) * (p > 0.0 ? p : 1e-300), -(double)beta);
    weight[b] = (float)(wv / mx);
  }
}

int log2_exact(int64_t pow2) {
  int l = 0;
  while (((int64_t)1 << l) < pow2) ++l;
  return l;
}

}  // namespace

extern "C" {

int mh_per_update(double* tree, int64_t pow2, const int64_t* idx, const float* prio, int64_t count, float alpha,
                  float eps, double* max_prio, void* stream) {
  if (!tree || !max_prio || pow2 <= 0 || (pow2 & (pow2 - 1)) || count < 0) return MH_EINVAL;
  if (count == 0) return MH_OK;
  if (!idx || !prio) return MH_EINVAL;
  k_update<<<1, UPD, 0, (hipStream_t)stream>>>(tree, pow2, log2_exact(pow2), idx, prio, count, alpha, eps, max_prio);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_EHIP;
}

int mh_per_set_new(double* tree, int64_t pow2, const int64_t* cursor_before, const int64_t* cursor_after,
                   int64_t capacity, const double* max_prio, void* stream) {
  if (!tree || !cursor_before || !cursor_after || !max_prio || capacity <= 0 || capacity > pow2 ||
      (pow2 & (pow2 - 1)))
    return MH_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (pow2 <= SUB) {
    k_new_small<<<1, SUB, 0, st>>>(tree, pow2, cursor_before, cursor_after, capacity, max_prio);
  } else {
    k_new_sub<<<(int)(pow2 / SUB), SUB / 2, 0, st>>>(tree, pow2, cursor_before, cursor_after, capacity, max_prio);
    if (hipGetLastError() != hipSuccess) return MH_EHIP;
    k_new_top<<<1, 1024, 0, st>>>(tree, pow2 / SUB, cursor_before, cursor_after);
  }
  return hipGetLastError() == hipSuccess ? MH_OK : MH_EHIP;
}

int mh_per_sample(const double* tree, int64_t pow2, const int64_t* cursor, uint64_t seed, uint64_t counter,
                  int64_t batch, float beta, int64_t* idx_out, float* weight_out, void* stream) {
  if (!tree || !cursor || !idx_out || !weight_out || batch <= 0 || pow2 <= 0 || (pow2 & (pow2 - 1)))
    return MH_EINVAL;
  k_sample<<<1, 256, 0, (hipStream_t)stream>>>(tree, pow2, cursor, seed, counter, batch, beta, idx_out, weight_out);
  return hipGetLastError() == hipSuccess ? MH_OK : MH_EHIP;
}

}  // extern "C"
