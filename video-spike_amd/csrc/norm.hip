// norm.hip — LayerNorm forward/backward over the hidden dim (mv:416-417,426,437; eps 1e-12).
//
// One wave per row; a lane holds columns lane + 64*i (i < VPL = cols/64, a template parameter
// so no slot is predicated away), giving coalesced 256-B wave accesses and keeping the row in
// registers between the statistics and the output pass (one HBM read of x).  Each wave keeps
// RPW rows in flight (all loads issued before the first reduction) to hide HBM latency — the
// first version with one row per wave measured 64 us for a 25,088 x 192 backward (~4x its
// byte floor).  The backward reduces dgamma/dbeta per block in LDS: one f32 atomic per column
// per block.
#include "common.h"

namespace vs {

template <typename TO, int VPL, int RPW>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     float eps, TO* __restrict__ y, int64_t ldy,
                                                     float* __restrict__ mean, float* __restrict__ rstd, int64_t rows,
                                                     int cols) {
  const int lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  const float inv = 1.f / (float)cols;
  float v[RPW][VPL];
#pragma unroll
  for (int k = 0; k < RPW; ++k)
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int64_t row = row0 + k;
      const int c = lane + 64 * i;
      v[k][i] = (row < rows && c < cols) ? x[row * ldx + c] : 0.f;
    }
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t row = row0 + k;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) s += v[k][i];
    const float mu = wave_sum(s) * inv;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const float d = c < cols ? v[k][i] - mu : 0.f;
      q += d * d;
    }
    const float rs = rsqrtf(wave_sum(q) * inv + eps);
    if (row < rows) {
      TO* yr = y + row * ldy;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = lane + 64 * i;
        if (c < cols) Elem<TO>::store(yr + c, (v[k][i] - mu) * rs * g[c] + b[c]);
      }
      if (lane == 0) {
        mean[row] = mu;
        rstd[row] = rs;
      }
    }
  }
}

template <int VPL, int RPW>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, int64_t lddy,
                                                     const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ g, const float* __restrict__ dres,
                                                     int64_t lddres, float* __restrict__ dx, int64_t lddx,
                                                     bf16_t* __restrict__ dx_lp, float* __restrict__ dg,
                                                     float* __restrict__ db, int64_t rows, int cols) {
  __shared__ float red[2][4][64 * VPL];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float inv = 1.f / (float)cols;
  float gam[VPL], pg[VPL], pb[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    gam[i] = c < cols ? g[c] : 0.f;
    pg[i] = pb[i] = 0.f;
  }
  for (int64_t row0 = ((int64_t)blockIdx.x * 4 + wid) * RPW; row0 < rows; row0 += (int64_t)gridDim.x * 4 * RPW) {
    float d[RPW][VPL], xv[RPW][VPL], mu[RPW], rs[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int64_t row = row0 + k;
      const bool ok = row < rows;
      mu[k] = ok ? mean[row] : 0.f;
      rs[k] = ok ? rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = lane + 64 * i;
        const bool in = ok && c < cols;
        d[k][i] = in ? dy[row * lddy + c] : 0.f;
        xv[k][i] = in ? x[row * ldx + c] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int64_t row = row0 + k;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const float xh = (xv[k][i] - mu[k]) * rs[k];
        const float gy = d[k][i] * gam[i];
        pg[i] += d[k][i] * xh;
        pb[i] += d[k][i];
        xv[k][i] = xh;
        d[k][i] = gy;
        s1 += gy;
        s2 += gy * xh;
      }
      const float m1 = wave_sum(s1) * inv, m2 = wave_sum(s2) * inv;
      if (row < rows) {
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
          const int c = lane + 64 * i;
          if (c < cols) {
            float o = rs[k] * (d[k][i] - m1 - xv[k][i] * m2);
            if (dres) o += dres[row * lddres + c];
            dx[row * lddx + c] = o;
            if (dx_lp) dx_lp[row * lddx + c] = f2bf(o);
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    red[0][wid][i * 64 + lane] = pg[i];
    red[1][wid][i * 64 + lane] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    const int i = c >> 6, l = c & 63;
    const float a = (red[0][0][i * 64 + l] + red[0][1][i * 64 + l]) + (red[0][2][i * 64 + l] + red[0][3][i * 64 + l]);
    const float bb = (red[1][0][i * 64 + l] + red[1][1][i * 64 + l]) + (red[1][2][i * 64 + l] + red[1][3][i * 64 + l]);
    unsafeAtomicAdd(dg + c, a);
    unsafeAtomicAdd(db + c, bb);
  }
}

template <typename TO, int VPL>
static void launch_fwd(int64_t rows, int64_t cols, const float* x, int64_t ldx, const float* gamma, const float* beta,
                       float eps, void* y, int64_t ldy, float* mean, float* rstd, hipStream_t s) {
  constexpr int RPW = VPL <= 4 ? 4 : (VPL <= 8 ? 2 : 1);
  dim3 grid((unsigned)cdiv(rows, 4 * RPW));
  hipLaunchKernelGGL((ln_fwd_kernel<TO, VPL, RPW>), grid, dim3(256), 0, s, x, ldx, gamma, beta, eps, (TO*)y, ldy, mean,
                     rstd, rows, (int)cols);
}

template <int VPL>
static void launch_bwd(int64_t rows, int64_t cols, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                       const float* mean, const float* rstd, const float* gamma, const float* dres, int64_t lddres,
                       float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta, hipStream_t s) {
  constexpr int RPW = VPL <= 4 ? 4 : (VPL <= 8 ? 2 : 1);
  int64_t nb = cdiv(rows, 4 * RPW * 2);  // ~2 row-groups per wave: amortises the column reduction
  if (nb > 2048) nb = 2048;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL((ln_bwd_kernel<VPL, RPW>), dim3((unsigned)nb), dim3(256), 0, s, dy, lddy, x, ldx, mean, rstd,
                     gamma, dres, lddres, dx, lddx, (bf16_t*)dx_lp, dgamma, dbeta, rows, (int)cols);
}

}  // namespace vs

using namespace vs;

#define VS_LN_DISPATCH(CALL)              \
  do {                                    \
    const int64_t vpl = cdiv(cols, 64);   \
    if (vpl <= 2) CALL(2);                \
    else if (vpl <= 3) CALL(3);           \
    else if (vpl <= 4) CALL(4);           \
    else if (vpl <= 8) CALL(8);           \
    else if (vpl <= 12) CALL(12);         \
    else CALL(16);                        \
  } while (0)

extern "C" int vs_layernorm_fwd(int32_t y_dtype, int64_t rows, int64_t cols, const float* x, int64_t ldx,
                                const float* gamma, const float* beta, float eps, void* y, int64_t ldy, float* mean,
                                float* rstd, void* stream) {
  VS_REQUIRE(x && gamma && beta && y && mean && rstd, "vs_layernorm_fwd: null pointer");
  VS_REQUIRE(cols > 0 && cols <= 1024, "vs_layernorm_fwd: cols must be in [1, 1024]");
  if (rows == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (y_dtype == VS_BF16) {
#define F_(V) launch_fwd<bf16_t, V>(rows, cols, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, s)
    VS_LN_DISPATCH(F_);
#undef F_
  } else {
#define F_(V) launch_fwd<float, V>(rows, cols, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, s)
    VS_LN_DISPATCH(F_);
#undef F_
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_layernorm_bwd(int64_t rows, int64_t cols, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                const float* mean, const float* rstd, const float* gamma, const float* dres,
                                int64_t lddres, float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta,
                                void* stream) {
  VS_REQUIRE(dy && x && mean && rstd && gamma && dx && dgamma && dbeta, "vs_layernorm_bwd: null pointer");
  VS_REQUIRE(cols > 0 && cols <= 1024, "vs_layernorm_bwd: cols must be in [1, 1024]");
  if (rows == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
#define B_(V) launch_bwd<V>(rows, cols, dy, lddy, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx, dx_lp, dgamma, \
                            dbeta, s)
  VS_LN_DISPATCH(B_);
#undef B_
  VS_LAUNCH_CHECK();
  return VS_OK;
}
