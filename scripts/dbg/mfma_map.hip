// Probe of the forward's row-sum trick: lacc = mfma_16x16x32(sel, pa, 0) where lane l's pa holds
// 8 values of query (l & 31), half (l >> 5).  Expected: lane n, reg 0 = sum over query n; reg 1 = query n+16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__device__ float val(int q, int slot) { return (float)((q * 7 + slot * 3) % 17 + 1); }
__global__ void k(float* out) {
  int l = threadIdx.x;
  int row = l & 15, g = l >> 4;
  float one = (row == 0 && (g & 1) == 0) || (row == 1 && (g & 1) == 1) ? 1.f : 0.f;
  f32x8 s = {one, one, one, one, one, one, one, one};
  f32x8 p;
  for (int j = 0; j < 8; ++j) p[j] = val(l & 31, 8 * (l >> 5) + j);
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_convertvector(s, bf16x8), __builtin_convertvector(p, bf16x8), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  float* d; (void)hipMalloc(&d, 256 * 4); float h[256];
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int n = 0; n < 16; ++n) for (int r = 0; r < 2; ++r) {
    int q = n + 16 * r; float e = 0;
    for (int s = 0; s < 16; ++s) e += (float)((q * 7 + s * 3) % 17 + 1);
    float got = h[n * 4 + r];
    if (fabsf(got - e) > 0.5f) { ++bad; printf("n=%d r=%d got %g expect %g\n", n, r, got, e); }
  }
  printf("rows 2,3 lane0: %g %g ; bad=%d\n", h[2], h[3], bad);
  return 0;
}
