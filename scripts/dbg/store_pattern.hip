// Store-pattern microbenchmark: 25088 x 768 bf16 (38.5 MB) written by a persistent grid with
//  (a) 1 KiB contiguous per wave-instruction (copy-like), (b) 16 rows x 64 B per wave-instruction
//  (MFMA 16x16 C^T layout, 4 lanes per row), (c) 8 rows x 128 B (LDS-staged epilogue layout),
//  (d) pattern (b) with each row's 128-B line completed by the next instruction (p = 0, 1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int M = 25088, N = 768;
__global__ __launch_bounds__(256) void st_contig(uint4* out, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
    out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
// unit = 16 rows x 64 columns (128 B per row): lane (tok = lane & 15, g = lane >> 4)
__global__ __launch_bounds__(256) void st_mfma(uint16_t* out, int units) {
  const int lane = threadIdx.x & 63, w = (blockIdx.x * 4 + (threadIdx.x >> 6));
  const int nw = gridDim.x * 4, tok = lane & 15, g = lane >> 4;
  for (int u = w; u < units; u += nw) {
    const int rb = u / (N / 64), ch = u % (N / 64);
    const int64_t m = (int64_t)rb * 16 + tok;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      *(uint4*)(out + m * N + ch * 64 + 32 * p + 8 * g) = make_uint4(u, p, 2, 3);
  }
}
// unit = 8 rows x 64 columns per instruction: lane (row = lane >> 3, c = lane & 7): 128 B per row
__global__ __launch_bounds__(256) void st_rows(uint16_t* out, int units) {
  const int lane = threadIdx.x & 63, w = (blockIdx.x * 4 + (threadIdx.x >> 6));
  const int nw = gridDim.x * 4, r = lane >> 3, c = lane & 7;
  for (int u = w; u < units; u += nw) {
    const int rb = u / (N / 64), ch = u % (N / 64);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t m = (int64_t)rb * 16 + 8 * h + r;
      *(uint4*)(out + m * N + ch * 64 + 8 * c) = make_uint4(u, h, 2, 3);
    }
  }
}
// whole row per wave: 768 bf16 = 1536 B = 96 x 16 B, lanes 0..63 then 0..31
__global__ __launch_bounds__(256) void st_fullrow(uint16_t* out, int rows) {
  const int lane = threadIdx.x & 63, w = (blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
  for (int m = w; m < rows; m += nw) {
    uint4* p = (uint4*)(out + (int64_t)m * N);
    p[lane] = make_uint4(m, 0, 2, 3);
    if (lane < 32) p[64 + lane] = make_uint4(m, 1, 2, 3);
  }
}
int main() {
  uint16_t* d;
  hipMalloc(&d, (size_t)M * N * 2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int units = (M / 16) * (N / 64);
  for (int grid : {512, 1024, 2048}) {
    for (int k = 0; k < 4; ++k) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        for (int it = 0; it < 20; ++it) {
          if (k == 0) hipLaunchKernelGGL(st_contig, dim3(grid), dim3(256), 0, 0, (uint4*)d, (int64_t)M * N / 8);
          if (k == 1) hipLaunchKernelGGL(st_mfma, dim3(grid), dim3(256), 0, 0, d, units);
          if (k == 2) hipLaunchKernelGGL(st_rows, dim3(grid), dim3(256), 0, 0, d, units);
          if (k == 3) hipLaunchKernelGGL(st_fullrow, dim3(grid), dim3(256), 0, 0, d, M);
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep) printf("grid %4d %-8s %7.2f us  %6.0f GB/s\n", grid, k == 0 ? "contig" : k == 1 ? "mfma16" : k == 2 ? "rows8" : "fullrow",
                        ms * 1e3 / 20, (double)M * N * 2 / (ms * 1e-3 / 20) / 1e9);
      }
    }
  }
  return 0;
}
