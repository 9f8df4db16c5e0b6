// norm.hip — LayerNorm forward/backward over the hidden dim (mv:416-417,426,437; eps 1e-12).
//
// One wave per row; a lane holds columns lane + 64*i (coalesced 256-B wave accesses), so the
// row lives in registers between the statistics and the output pass (one HBM read of x).
// Backward reduces dgamma/dbeta per block in LDS and issues one f32 atomic per column per block.
#include "common.h"

namespace vs {

constexpr int kMaxPerLane = 16;  // cols <= 1024

template <typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float eps, TO* __restrict__ y, int64_t ldy,
                                                     float* __restrict__ mean, float* __restrict__ rstd, int64_t rows,
                                                     int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float v[kMaxPerLane];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < cols ? xr[c] : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    const float d = c < cols ? v[i] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / (float)cols + eps);
  TO* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) Elem<TO>::store(yr + c, (v[i] - mu) * rs * g[c] + b[c]);
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, int64_t lddy,
                                                     const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ g, const float* __restrict__ dres,
                                                     int64_t lddres, float* __restrict__ dx, int64_t lddx,
                                                     bf16_t* __restrict__ dx_lp, float* __restrict__ dg,
                                                     float* __restrict__ db, int64_t rows, int cols) {
  __shared__ float red[2][4][64 * kMaxPerLane / 4];  // reused per column chunk
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float pg[kMaxPerLane], pb[kMaxPerLane];
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) pg[i] = pb[i] = 0.f;

  for (int64_t row = blockIdx.x * 4 + wid; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[kMaxPerLane], gy[kMaxPerLane];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < kMaxPerLane; ++i) {
      const int c = lane + 64 * i;
      if (c < cols) {
        const float d = dy[row * lddy + c];
        xh[i] = (x[row * ldx + c] - mu) * rs;
        gy[i] = d * g[c];
        pg[i] += d * xh[i];
        pb[i] += d;
      } else {
        xh[i] = gy[i] = 0.f;
      }
      s1 += gy[i];
      s2 += gy[i] * xh[i];
    }
    const float inv = 1.f / (float)cols;
    const float m1 = wave_sum(s1) * inv, m2 = wave_sum(s2) * inv;
#pragma unroll
    for (int i = 0; i < kMaxPerLane; ++i) {
      const int c = lane + 64 * i;
      if (c < cols) {
        float o = rs * (gy[i] - m1 - xh[i] * m2);
        if (dres) o += dres[row * lddres + c];
        dx[row * lddx + c] = o;
        if (dx_lp) dx_lp[row * lddx + c] = f2bf(o);
      }
    }
  }
  // block reduction of the column partials: 4 waves -> wave 0 -> one atomic per column
  constexpr int CH = kMaxPerLane / 4;  // columns chunks of 4*64 handled per pass
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      red[0][wid][k * 64 + lane] = pg[pass * CH + k];
      red[1][wid][k * 64 + lane] = pb[pass * CH + k];
    }
    __syncthreads();
    if (wid == 0) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int c = lane + 64 * (pass * CH + k);
        if (c < cols) {
          const float a = (red[0][0][k * 64 + lane] + red[0][1][k * 64 + lane]) +
                          (red[0][2][k * 64 + lane] + red[0][3][k * 64 + lane]);
          const float bb = (red[1][0][k * 64 + lane] + red[1][1][k * 64 + lane]) +
                           (red[1][2][k * 64 + lane] + red[1][3][k * 64 + lane]);
          unsafeAtomicAdd(dg + c, a);
          unsafeAtomicAdd(db + c, bb);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace vs

using namespace vs;

extern "C" int vs_layernorm_fwd(int32_t y_dtype, int64_t rows, int64_t cols, const float* x, int64_t ldx,
                                const float* gamma, const float* beta, float eps, void* y, int64_t ldy, float* mean,
                                float* rstd, void* stream) {
  VS_REQUIRE(x && gamma && beta && y && mean && rstd, "vs_layernorm_fwd: null pointer");
  VS_REQUIRE(cols > 0 && cols <= 64 * kMaxPerLane, "vs_layernorm_fwd: cols must be in [1, 1024]");
  if (rows == 0) return VS_OK;
  dim3 grid((unsigned)cdiv(rows, 4));
  hipStream_t s = (hipStream_t)stream;
  if (y_dtype == VS_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, x, ldx, gamma, beta, eps, (bf16_t*)y, ldy, mean,
                       rstd, rows, (int)cols);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, s, x, ldx, gamma, beta, eps, (float*)y, ldy, mean,
                       rstd, rows, (int)cols);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_layernorm_bwd(int64_t rows, int64_t cols, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                const float* mean, const float* rstd, const float* gamma, const float* dres,
                                int64_t lddres, float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta,
                                void* stream) {
  VS_REQUIRE(dy && x && mean && rstd && gamma && dx && dgamma && dbeta, "vs_layernorm_bwd: null pointer");
  VS_REQUIRE(cols > 0 && cols <= 64 * kMaxPerLane, "vs_layernorm_bwd: cols must be in [1, 1024]");
  if (rows == 0) return VS_OK;
  int64_t nb = cdiv(rows, 4);
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, dy, lddy, x, ldx, mean,
                     rstd, gamma, dres, lddres, dx, lddx, (bf16_t*)dx_lp, dgamma, dbeta, rows, (int)cols);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
