// Layout probe for v_mfma_f32_16x16x1_4b_f32 (gfx950): prints, for every (lane, register) of the
// result, the A lane (block, row) and B lane (block, column) whose product landed there.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void probe(float* out, int mode) {
  const int l = threadIdx.x;
  const float a = mode == 0 ? (float)(l + 1) : 1.0f;
  const float b = mode == 0 ? 1.0f : (float)(l + 1);
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = c[r];
}
int main() {
  float* d;
  hipMalloc(&d, 64 * 16 * 4);
  float h[2][64 * 16];
  for (int m = 0; m < 2; ++m) {
    probe<<<1, 64>>>(d, m);
    hipMemcpy(h[m], d, sizeof(h[m]), hipMemcpyDeviceToHost);
  }
  for (int l = 0; l < 64; l += 1) {
    printf("lane %2d:", l);
    for (int r = 0; r < 16; ++r) printf(" %2.0f/%2.0f", h[0][l * 16 + r] - 1, h[1][l * 16 + r] - 1);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
