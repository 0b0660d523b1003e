// mlp_grad.hip — the activation backward and bias gradient of an MLP layer in one pass (gfx950).
//
// For y = act(x W^T + b) with act in {identity, ReLU, tanh} (the activations the reference's
// MLPs use, RL/utils/common_utils.py get_activation_func), autograd needs
//   g  = dy * act'(y)        (ReLU: y > 0; tanh: 1 - y^2; identity: 1)
//   db = sum over rows of g  (the bias gradient)
// before the two GEMMs (dx = g W, dW = g^T x). PyTorch issues an elementwise backward kernel and
// a separate reduction (14 us for 5,120 x 256 on MI355X). Here: a 2-D grid streams dy/y once,
// coalesced along the columns (64 columns x 4 row lanes per workgroup, every load of a thread
// issued before the first add: memory-level parallelism, not a latency chain), writes g and
// per-row-chunk column sums; the LAST workgroup of each column group to finish (agent-scope
// arrival counter) adds the chunk sums in a fixed order, so the bias gradient is deterministic
// and the layer backward is one launch. Cross-XCD hand-off per cdna_hip_programming.md's
// publish/consume recipe: the chunk sums are stored write-through (sc1), every storing wave
// drains (vmcnt(0)) before the workgroup barrier and the counter add, and the reducing
// workgroup reads them with sc1 loads (no stale L1/L2 copy can be hit).
#include "rollout.h"

namespace mh {

constexpr int AG_COLS = 64;   // columns per workgroup (one wavefront row)
constexpr int AG_RPT = 16;    // rows per thread
constexpr int AG_ROWS = 4 * AG_RPT;  // rows per workgroup (4 row lanes)

__global__ __launch_bounds__(256) void k_act_grad_colsum(const float* __restrict__ dy, const float* __restrict__ y,
                                                         int64_t M, int N, int act, float* __restrict__ g,
                                                         float* __restrict__ partial, float* __restrict__ db,
                                                         uint32_t* __restrict__ tickets) {
  __shared__ float red[4][AG_COLS];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * AG_COLS + tx;
  const int64_t m0 = (int64_t)blockIdx.y * AG_ROWS + ty;
  float acc = 0.0f;
  float gv[AG_RPT];
  if (n < N) {
    float d[AG_RPT], t[AG_RPT];
#pragma unroll
    for (int j = 0; j < AG_RPT; ++j) {
      const int64_t m = m0 + 4 * j;
      const bool ok = m < M;
      d[j] = ok ? dy[m * N + n] : 0.0f;
      t[j] = (ok && act != 0) ? y[m * N + n] : 0.0f;
    }
    // all of g first, then the stores: a store between two uses of loaded values would make
    // every later wait on the load queue also wait for that store (vmcnt counts both in order)
#pragma unroll
    for (int j = 0; j < AG_RPT; ++j) {
      gv[j] = d[j];
      if (act == 1) gv[j] = t[j] > 0.0f ? d[j] : 0.0f;
      else if (act == 2) gv[j] = d[j] * (1.0f - t[j] * t[j]);
    }
#pragma unroll
    for (int j = 0; j < AG_RPT; ++j) acc += gv[j];
  }
  red[ty][tx] = acc;
  __syncthreads();
  const float csum = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
  // g is written after the chunk sums are published: the drain before the arrival count then
  // waits for one store per thread, not for this thread's 16 g stores as well
  auto store_g = [&]() {
    if (g && n < N) {
#pragma unroll
      for (int j = 0; j < AG_RPT; ++j) {
        const int64_t m = m0 + 4 * j;
        if (m < M) g[m * N + n] = gv[j];
      }
    }
  };
  if (!tickets) {
    if (ty == 0 && n < N) partial[(int64_t)blockIdx.y * N + n] = csum;
    store_g();
    return;
  }
  // fused finish: publish this chunk's sums write-through, count arrivals per column group.
  // Memory-model basis (LLVM AMDGPUUsage, "Memory Model GFX942" code sequences, which gfx950
  // follows): the agent-scope atomic store is written through to the coherence point and is
  // performed when `s_waitcnt vmcnt(0)` returns; the arrival follows the workgroup barrier in
  // program order; the finishing chunk reads the sums with agent-scope atomic loads (`sc1`) from
  // the coherence point: no release / acquire fence (MI355X_MICROARCH.md, sc1 hand-off row 1).
  if (ty == 0 && n < N)
    __hip_atomic_store(partial + (int64_t)blockIdx.y * N + n, csum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    // release: this workgroup's published sums (drained above, ordered by the barrier) before
    // the arrival; acquire: the last arrival sees every other workgroup's sums
    const uint32_t a = __hip_atomic_fetch_add(tickets + blockIdx.x, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (a == gridDim.y - 1);
  }
  store_g();
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every reading thread, not only thread 0
  const int R = (int)gridDim.y;
  float s = 0.0f;
  if (n < N) {
    // the write-through loads go to memory: issue a batch of 16 before the first add, so a
    // batch costs one round trip (rows ty, ty + 4, ... in ascending order, as before)
    constexpr int NB = 16;
    for (int base = ty; base < R; base += 4 * NB) {
      float v[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int r = base + 4 * j;
        v[j] = r < R ? __hip_atomic_load(partial + (int64_t)r * N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0.0f;
      }
#pragma unroll
      for (int j = 0; j < NB; ++j)
        if (base + 4 * j < R) s = s + v[j];
    }
  }
  __syncthreads();  // everyone has read red[] above
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) db[n] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
  if (threadIdx.x == 0) __hip_atomic_store(tickets + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// db[n] = sum_r partial[r][n], r ascending within each of 4 interleaved lanes, lanes added in order
__global__ __launch_bounds__(256) void k_colsum_finish(const float* __restrict__ partial, int R, int N,
                                                       float* __restrict__ db) {
  __shared__ float red[4][AG_COLS];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * AG_COLS + tx;
  float s = 0.0f;
  if (n < N) {
    int r = ty;
    for (; r + 12 < R; r += 16) {  // 4 independent loads in flight per iteration
      const float a0 = partial[(int64_t)r * N + n], a1 = partial[(int64_t)(r + 4) * N + n];
      const float a2 = partial[(int64_t)(r + 8) * N + n], a3 = partial[(int64_t)(r + 12) * N + n];
      s = s + a0;
      s = s + a1;
      s = s + a2;
      s = s + a3;
    }
    for (; r < R; r += 4) s += partial[(int64_t)r * N + n];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) db[n] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}

// ------------------------------------------------------------------ output-layer backward
// The identity-activation output layer of a narrow head (n_out <= HB_MAX_OUT: the critics' 1,
// the policy's 2A) over many rows: dx = dy W (the gradient handed to the hidden layer below),
// dW = dy^T x and db = column sums of dy, in one pass over x instead of a bias-gradient kernel,
// an input-gradient GEMM and a weight-gradient GEMM with its split-K finish. Workgroup = HB_ROWS
// rows; its dy rows are staged in LDS; thread = input column j (and j + 256, ...):
// x[r][j] is read once (row-contiguous across the workgroup) and feeds both the dx element
// (W column j in registers) and the n_out dW partial sums; per-workgroup partials [blk][n_out][n_in]
// and [blk][n_out] are summed in block order by k_head_finish (deterministic).
constexpr int HB_MAX_OUT = 16;
constexpr int HB_ROWS = 64;

// rows per workgroup: 16 below 16,384 rows (the update's 5,120-row heads: 320 workgroups instead of
// 80 at 64 rows, so more than one per CU), 64 above
__host__ __device__ inline int hb_rows(int64_t M) { return M >= 16384 ? HB_ROWS : 16; }

// grouped launches (the twin critics' output layers): blockIdx.y = group q, whose dy, x, W, dx
// and partials sit at q x the strides; x and dx rows of leading dimension ldx / lddx
struct HeadGroup {
  int64_t ldx, lddx, s_dy, s_x, s_W, s_dx, s_part;
};

template <int NO>
__global__ __launch_bounds__(256) void k_head_backward(const float* __restrict__ dy, const float* __restrict__ x,
                                                       const float* __restrict__ W, int64_t M, int n_in,
                                                       float* __restrict__ dx, float* __restrict__ pdw,
                                                       float* __restrict__ pdb, HeadGroup hg) {
  __shared__ float sdy[HB_ROWS][NO];
  const int tid = threadIdx.x;
  if (blockIdx.y) {
    const int64_t q = blockIdx.y;
    dy += q * hg.s_dy;
    x += q * hg.s_x;
    W += q * hg.s_W;
    if (dx) dx += q * hg.s_dx;
    if (pdw) pdw += q * hg.s_part;
    if (pdb) pdb += q * hg.s_part;
  }
  const int64_t ldx = hg.ldx, lddx = hg.lddx;
  const int rpb = hb_rows(M);
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int nr = M - r0 < rpb ? (int)(M - r0) : rpb;
  for (int q = tid; q < rpb * NO; q += 256) {
    const int r = q / NO, o = q - r * NO;
    sdy[r][o] = r < nr ? dy[(r0 + r) * NO + o] : 0.0f;
  }
  __syncthreads();
  if (pdb && tid < NO) {  // bias partial: this block's rows in order
    float s = 0.0f;
    for (int r = 0; r < nr; ++r) s = s + sdy[r][tid];
    pdb[(int64_t)blockIdx.x * NO + tid] = s;
  }
  if (!pdw) {  // input gradient only (frozen heads): dx = dy W needs no x
    for (int j = tid; j < n_in; j += 256) {
      float w[NO];
#pragma unroll
      for (int o = 0; o < NO; ++o) w[o] = W[(int64_t)o * n_in + j];
      for (int r = 0; r < nr; ++r) {
        float d = 0.0f;
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          const float g = sdy[r][o];
          d = o == 0 ? g * w[0] : d + g * w[o];  // dy[r] . W[:, j], o ascending (as below)
        }
        if (dx) dx[(r0 + r) * lddx + j] = d;
      }
    }
    return;
  }
  for (int j = tid; j < n_in; j += 256) {
    float w[NO], acc[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      w[o] = W[(int64_t)o * n_in + j];
      acc[o] = 0.0f;
    }
    for (int rb = 0; rb < nr; rb += 16) {
      float xv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) xv[u] = rb + u < nr ? x[(r0 + rb + u) * ldx + j] : 0.0f;  // 16 in flight
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (rb + u >= nr) break;
        float d = 0.0f;
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          const float g = sdy[rb + u][o];
          d = o == 0 ? g * w[0] : d + g * w[o];  // dy[r] . W[:, j], o ascending
          acc[o] = acc[o] + g * xv[u];
        }
        if (dx) dx[(r0 + rb + u) * lddx + j] = d;
      }
    }
    if (pdw) {
#pragma unroll
      for (int o = 0; o < NO; ++o) pdw[((int64_t)blockIdx.x * NO + o) * n_in + j] = acc[o];
    }
  }
}

// dW[o][j] = sum over blocks of pdw[b][o][j] (and db[o] of pdb[b][o]): one wave per output, lane l
// adding blocks l, l + 64, ... in order, the 64 lane sums then added by a fixed butterfly
// (deterministic; every lane's loads in flight together: one round trip per 64 x 8 blocks, where
// one thread per output walking all blocks in batches of 16 paid nblk / 16 round trips)
__global__ __launch_bounds__(256) void k_head_finish(const float* __restrict__ pdw, const float* __restrict__ pdb,
                                                     int nblk, int n_out, int n_in, float* __restrict__ dw,
                                                     float* __restrict__ db, int64_t s_part, int64_t s_dw,
                                                     int64_t s_db) {
  if (blockIdx.y) {
    const int64_t q = blockIdx.y;
    if (pdw) pdw += q * s_part;
    if (pdb) pdb += q * s_part;
    if (dw) dw += q * s_dw;
    if (db) db += q * s_db;
  }
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)n_out * n_in;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nw + (db ? n_out : 0)) return;
  const bool isw = i < nw;
  const float* src = isw ? pdw + i : pdb + (i - nw);
  const int64_t stride = isw ? nw : n_out;
  float v = 0.0f;
  for (int b0 = lane; b0 < nblk; b0 += 8 * 64) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = b0 + 64 * u < nblk ? src[(int64_t)(b0 + 64 * u) * stride] : 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) v = v + t[u];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
  if (lane == 0) {
    if (isw) dw[i] = v;
    else db[i - nw] = v;
  }
}

int64_t head_backward_workspace(int64_t M, int n_out, int n_in) {
  const int rpb = hb_rows(M);
  const int64_t nblk = (M + rpb - 1) / rpb;
  return nblk * n_out * (int64_t)n_in + nblk * n_out;
}

hipError_t launch_head_backward_grouped(const float* dy, const float* x, const float* W, int64_t M, int n_out,
                                        int n_in, int64_t ldx, int64_t lddx, int groups, int64_t s_dy, int64_t s_x,
                                        int64_t s_W, int64_t s_dx, int64_t s_dw, int64_t s_db, float* dx, float* dw,
                                        float* db, float* workspace, hipStream_t st) {
  if (M <= 0 || n_out <= 0 || n_out > HB_MAX_OUT || n_in <= 0 || groups <= 0 || groups > 65535 || ldx < n_in ||
      (dx && lddx < n_in))
    return hipErrorInvalidValue;
  const int rpb = hb_rows(M);
  const int64_t nblk = (M + rpb - 1) / rpb;
  const int64_t wsg = head_backward_workspace(M, n_out, n_in);  // per group
  float* pdw = dw ? workspace : nullptr;
  float* pdb = db ? workspace + nblk * n_out * (int64_t)n_in : nullptr;
  const dim3 grid((unsigned)nblk, (unsigned)groups);
  const HeadGroup hg{ldx, lddx, s_dy, s_x, s_W, s_dx, wsg};
#define HB_CASE(K)                                                                                     \
  case K: k_head_backward<K><<<grid, 256, 0, st>>>(dy, x, W, M, n_in, dx, pdw, pdb, hg); break;
  switch (n_out) {
    HB_CASE(1) HB_CASE(2) HB_CASE(3) HB_CASE(4) HB_CASE(5) HB_CASE(6) HB_CASE(7) HB_CASE(8)
    HB_CASE(9) HB_CASE(10) HB_CASE(11) HB_CASE(12) HB_CASE(13) HB_CASE(14) HB_CASE(15) HB_CASE(16)
  }
#undef HB_CASE
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (!dw && !db)) return e;
  const int64_t outs = (int64_t)(dw ? n_out * (int64_t)n_in : 0) + (db ? n_out : 0);
  // (dw is always set with db: the C ABI rejects db without dw)
  k_head_finish<<<dim3((unsigned)((outs + 3) / 4), (unsigned)groups), 256, 0, st>>>(pdw, pdb, (int)nblk, n_out, n_in,
                                                                                   dw, db, wsg, s_dw, s_db);
  return hipGetLastError();
}

hipError_t launch_head_finish(const float* pdw, const float* pdb, int64_t nblk, int n_out, int n_in, int groups,
                              int64_t s_part, float* dw, int64_t s_dw, float* db, int64_t s_db, hipStream_t st) {
  if (nblk <= 0 || n_out <= 0 || n_in <= 0 || groups <= 0 || groups > 65535 || !pdw || !dw || (db && !pdb))
    return hipErrorInvalidValue;
  const int64_t outs = n_out * (int64_t)n_in + (db ? n_out : 0);
  k_head_finish<<<dim3((unsigned)((outs + 3) / 4), (unsigned)groups), 256, 0, st>>>(pdw, db ? pdb : nullptr, (int)nblk,
                                                                                   n_out, n_in, dw, db, s_part, s_dw,
                                                                                   s_db);
  return hipGetLastError();
}

hipError_t launch_head_backward(const float* dy, const float* x, const float* W, int64_t M, int n_out, int n_in,
                                float* dx, float* dw, float* db, float* workspace, hipStream_t st) {
  return launch_head_backward_grouped(dy, x, W, M, n_out, n_in, n_in, n_in, 1, 0, 0, 0, 0, 0, 0, dx, dw, db, workspace,
                                      st);
}

// LyapunovValue's V = sum_j y_j^2 over each row (RL/apprfunc/mlp.py: torch.pow(y, 2).sum(-1)) and
// its backward dy = g * (2 y) (pow's backward, bit for bit): one wave per row, a float4 per lane
// per 256-wide chunk, butterfly sum (replaces the pow and reduce launches and their two
// backward launches).
__global__ __launch_bounds__(256) void k_square_sum(const float* __restrict__ y, int64_t rows, int cols,
                                                    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* yr = y + r * cols;
  float acc = 0.0f;
  for (int c0 = 0; c0 < cols; c0 += 256) {
    const int c = c0 + 4 * lane;
    if (c + 3 < cols && (cols & 3) == 0) {
      const float4 v = *reinterpret_cast<const float4*>(yr + c);
      acc = acc + v.x * v.x;
      acc = acc + v.y * v.y;
      acc = acc + v.z * v.z;
      acc = acc + v.w * v.w;
    } else {
      for (int u = 0; u < 4; ++u)
        if (c + u < cols) acc = acc + yr[c + u] * yr[c + u];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
  if (lane == 0) out[r] = acc;
}
__global__ __launch_bounds__(256) void k_square_sum_bwd(const float* __restrict__ y, const float* __restrict__ g,
                                                        int64_t rows, int cols, float* __restrict__ dy) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  dy[i] = g[i / cols] * (2.0f * y[i]);
}

hipError_t launch_square_sum(const float* y, int64_t rows, int cols, float* out, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  k_square_sum<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(y, rows, cols, out);
  return hipGetLastError();
}
hipError_t launch_square_sum_bwd(const float* y, const float* g, int64_t rows, int cols, float* dy, hipStream_t st) {
  const int64_t n = rows * cols;
  if (n <= 0) return hipSuccess;
  k_square_sum_bwd<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(y, g, rows, cols, dy);
  return hipGetLastError();
}

// Input gradient of a layer with a narrow input (n_in <= DN_MAX_IN: the MLPs' first layers, e.g.
// a frozen critic's [obs | act] input in the policy step) when no weight / bias gradient is wanted:
// dx[r][c] = sum_j dy[r][j] act'(y[r][j]) W[j][c], act' formed on the fly (replaces the colsum
// pass writing g and the library GEMM reading it back). Workgroup = DN_ROWS rows: g rows and W
// staged in LDS (16-byte loads), thread = (row, input column), the n_out products summed in j order.
constexpr int DN_MAX_IN = 32;
constexpr int DN_ROWS = 16;
__global__ __launch_bounds__(256) void k_dx_narrow(const float* __restrict__ dy, const float* __restrict__ y,
                                                   int act, const float* __restrict__ W, int64_t M, int n_out,
                                                   int n_in, float* __restrict__ dx) {
  extern __shared__ float sm[];
  float* sg = sm;                    // [DN_ROWS][n_out]
  float* sw = sm + DN_ROWS * n_out;  // [n_out][n_in]
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * DN_ROWS;
  const int nr = M - r0 < DN_ROWS ? (int)(M - r0) : DN_ROWS;
  for (int q = tid; q < DN_ROWS * n_out; q += 256) {
    const int r = q / n_out;
    float g = 0.0f;
    if (r < nr) {
      const int64_t i = r0 * n_out + q;
      const float d = dy[i];
      g = d;
      if (act == 1) g = y[i] > 0.0f ? d : 0.0f;
      else if (act == 2) { const float t = y[i]; g = d * (1.0f - t * t); }
    }
    sg[q] = g;
  }
  for (int q = tid; q < n_out * n_in; q += 256) sw[q] = W[q];
  __syncthreads();
  for (int q = tid; q < nr * n_in; q += 256) {
    const int r = q / n_in, c = q - r * n_in;
    const float* gr = sg + r * n_out;
    float acc = gr[0] * sw[c];
    for (int j = 1; j < n_out; ++j) acc = acc + gr[j] * sw[j * n_in + c];
    dx[(r0 + r) * n_in + c] = acc;
  }
}

// The same product on the f32 MFMA for n_in <= 16 and n_out % 64 == 0 (the critics' [obs | act]
// layer: 5,120 x 256 -> 16). k_dx_narrow above sums each output over n_out LDS products in one
// dependent chain (17 us at 5,120 x 256 x 16: the chain's LDS latency, one workgroup per CU).
// Here workgroup = 16 rows, wave w = a quarter of the n_out range: per lane 4 x (n_out / 64)
// independent float4 loads of dy (and y), the 16 x 16 x 4 f32 MFMA over its k range
// (lane l supplies A[l & 15][k] and W[k][l & 15] with k = 16 s + 4 (l >> 4) + j: a permutation
// of k, so each lane's loads are row-contiguous float4), the four wave partials added in wave
// order through LDS. Summation order differs from k_dx_narrow's (f32 rounding level).
constexpr int DNM_MAX_S = 8;  // n_out / 64 <= 8 (n_out <= 512)
__device__ __forceinline__ float act_grad_v(float d, float t, int act) {  // k_dx_narrow's g
  if (act == 1) return t > 0.0f ? d : 0.0f;
  if (act == 2) return d * (1.0f - t * t);
  return d;
}
__global__ __launch_bounds__(256) void k_dx_narrow_mfma(const float* __restrict__ dy, const float* __restrict__ y,
                                                        int act, const float* __restrict__ W, int64_t M, int n_out,
                                                        int n_in, float* __restrict__ dx) {
  __shared__ float red[3][256];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const int64_t row = r0 + (lane & 15);
  const int S = n_out / 64;  // 16-deep k groups per wave
  const int kb = w * 16 * S;
  const int col = lane & 15;
  f32x4v a[DNM_MAX_S], t[DNM_MAX_S];
#pragma unroll
  for (int s = 0; s < DNM_MAX_S; ++s) {
    if (s < S) {
      const int k = kb + 16 * s + 4 * (lane >> 4);
      a[s] = row < M ? *reinterpret_cast<const f32x4v*>(dy + row * n_out + k) : f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      t[s] = (act != 0 && row < M) ? *reinterpret_cast<const f32x4v*>(y + row * n_out + k) : f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
  }
  f32x4v acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < DNM_MAX_S; ++s) {
    if (s < S) {
      const int k = kb + 16 * s + 4 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g = act_grad_v(a[s][j], t[s][j], act);
        const float b = col < n_in ? W[(int64_t)(k + j) * n_in + col] : 0.0f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(g, b, acc, 0, 0, 0);
      }
    }
  }
  // D map: column lane & 15, rows 4 (lane >> 4) + q
  if (w > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) red[w - 1][q * 64 + lane] = acc[q];
  }
  __syncthreads();
  if (w == 0 && col < n_in) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = ((acc[q] + red[0][q * 64 + lane]) + red[1][q * 64 + lane]) + red[2][q * 64 + lane];
      const int64_t r = r0 + 4 * (lane >> 4) + q;
      if (r < M) dx[r * n_in + col] = v;
    }
  }
}

hipError_t launch_dx_narrow(const float* dy, const float* y, int act, const float* W, int64_t M, int n_out,
                            int n_in, float* dx, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (n_in <= 0 || n_in > DN_MAX_IN || n_out <= 0 || n_out > 1024) return hipErrorInvalidValue;
  if (n_in <= 16 && n_out % 64 == 0 && n_out / 64 <= DNM_MAX_S && ((uintptr_t)dy & 15) == 0 &&
      (act == 0 || ((uintptr_t)y & 15) == 0)) {
    k_dx_narrow_mfma<<<(unsigned)((M + 15) / 16), 256, 0, st>>>(dy, y, act, W, M, n_out, n_in, dx);
    return hipGetLastError();
  }
  const size_t shm = sizeof(float) * ((size_t)DN_ROWS * n_out + (size_t)n_out * n_in);
  k_dx_narrow<<<(unsigned)((M + DN_ROWS - 1) / DN_ROWS), 256, shm, st>>>(dy, y, act, W, M, n_out, n_in, dx);
  return hipGetLastError();
}

int act_grad_chunks(int64_t M) { return (int)((M + AG_ROWS - 1) / AG_ROWS); }

int act_grad_tickets(int N) { return (N + AG_COLS - 1) / AG_COLS; }

hipError_t launch_act_grad_colsum(const float* dy, const float* y, int64_t M, int N, int act, float* g, float* db,
                                  float* partial, uint32_t* tickets, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (M <= 0) return db ? hipMemsetAsync(db, 0, sizeof(float) * (size_t)N, st) : hipSuccess;  // empty sum
  const int R = act_grad_chunks(M);
  const int cg = (N + AG_COLS - 1) / AG_COLS;
  // with tickets: one launch (the last chunk of each column group reduces); without: two
  k_act_grad_colsum<<<dim3(cg, R), 256, 0, st>>>(dy, y, M, N, act, g, partial, db, db ? tickets : nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !db || tickets) return e;
  k_colsum_finish<<<cg, 256, 0, st>>>(partial, R, N, db);
  return hipGetLastError();
}

}  // namespace mh
