// mfma_rate.hip — TOOL: cycles per v_mfma_f32_32x32x16_bf16 on gfx950 for accumulation-chain
// patterns (1 wave per SIMD, operands in registers): which pattern the policy kernel can use.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS, int DEPTH>
__global__ __launch_bounds__(256, 1) void k(const float* in, float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)in[lane * 8 + j];
    b[j] = (__bf16)in[512 + lane * 8 + j];
  }
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  }
  const long long t1 = clock64();
  float s = 0;
  for (int c = 0; c < CHAINS; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the policy kernel's layer-2 pattern: 8 output blocks x 2 tiles = 16 accumulators (256 regs),
// per step (ob, s) two 6-deep chains (tile 0, tile 1) on acc[t][ob], A/B operands varying
__global__ __launch_bounds__(256, 1) void kpat(const float* in, float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[3], b[4];
  for (int j = 0; j < 8; ++j) {
    for (int p = 0; p < 3; ++p) a[p][j] = (__bf16)in[p * 512 + lane * 8 + j];
    for (int p = 0; p < 4; ++p) b[p][j] = (__bf16)in[1536 + p * 512 + lane * 8 + j];
  }
  f32x16 acc[2][8];
  for (int t = 0; t < 2; ++t)
    for (int o = 0; o < 8; ++o) acc[t][o] = f32x16{};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int ob = st >> 1;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x16 x = acc[t][ob];
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[t], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t + 2], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[t + 1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[t], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t + 1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t], x, 0, 0, 0);
        acc[t][ob] = x;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const long long t1 = clock64();
  float s = 0;
  for (int t = 0; t < 2; ++t)
    for (int o = 0; o < 8; ++o)
      for (int r = 0; r < 16; ++r) s += acc[t][o][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

void runpat(float* in, float* out, long long* cyc) {
  const int iters = 100;
  hipLaunchKernelGGL(kpat, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kpat, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 256; ++i) avg += h[i];
  avg /= 256;
  const double n = (double)iters * 16 * 12;
  printf("policy layer-2 pattern (16 accumulators): %.1f clock64-cycles/MFMA, %.1f ns/MFMA\n", avg / n, ms * 1e6 / n);
}

template <int C, int D>
void run(float* in, float* out, long long* cyc) {
  const int iters = 2000;
  hipLaunchKernelGGL((k<C, D>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<C, D>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 256; ++i) avg += h[i];
  avg /= 256;
  const double n = (double)iters * C * D;
  printf("chains %d depth %d: %.1f clock64-cycles/MFMA, wall %.3f ms -> %.1f ns/MFMA (%.0f TF/s bf16)\n", C, D,
         avg / n, ms, ms * 1e6 / n, n * 1024 * 32768 / (ms * 1e-3) / 1e12);
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 4096 * 4 * 2);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 8);
  {
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 7919) % 1000) / 997.0f - 0.5f;  // non-zero data
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  }
  run<1, 12>(in, out, cyc);
  run<2, 6>(in, out, cyc);
  run<4, 3>(in, out, cyc);
  run<16, 1>(in, out, cyc);
  runpat(in, out, cyc);
  return 0;
}
