// elementwise.hip — HBM-bound helpers of the hot path: tubelet im2col, sinusoid table, bias
// column sums, casts, fused PoissonNLL(+grad) and the fused AdamW step.
#include <math.h>

#include "common.h"

namespace vs {

// ---------------------------------------------------------------------------------------------
// im2col for the tubelet Conv3d (mv:176-181, 194-195), walked over the INPUT: a workgroup is 8 image
// rows x 32 lanes; lane w8 < W / 8 reads 8 consecutive pixels (32 B) of its row — a row's lanes read
// the whole 896-B row — and writes them as 8 consecutive columns (one 16-B bf16 / two 16-B f32
// stores) of their token's row: col = ((c t + tt) p + i) p + j.  (b, f) come from blockIdx.x and
// (c, h) from blockIdx.y and the lane's row, so the per-thread index math is a few shifts at the
// ViT geometry (T = 2, P = 16 compile-time).  57 us for the C2 batch (115 MB) against 59-60 us for
// the output-walking grid-stride versions: not index- or pattern-bound.
// ---------------------------------------------------------------------------------------------
template <typename T, int TT, int PP>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ px, T* __restrict__ out, int F, int C,
                                                     int H, int W, int t_rt, int p_rt) {
  const int t = TT > 0 ? TT : t_rt, p = PP > 0 ? PP : p_rt;
  const int w8 = threadIdx.x & 31, rsub = threadIdx.x >> 5;
  const int hc = blockIdx.y * 8 + rsub;  // c * H + h
  if (w8 * 8 >= W || hc >= C * H) return;
  const int bf = blockIdx.x;             // b * F + f (workgroup-uniform)
  const int b = bf / F, f = bf - b * F;
  const int c = hc / H, h = hc - c * H;
  const int Fp = F / t, Hp = H / p, Wp = W / p;
  const int ncol = C * t * p * p;
  const int w0 = 8 * w8;
  const float* src = px + (((int64_t)bf * C + c) * H + h) * W + w0;
  const float4 a = *(const float4*)src;
  const float4 bb = *(const float4*)(src + 4);
  const int fp = f / t, tt = f - fp * t, hp = h / p, i = h - hp * p, wp = w0 / p, j = w0 - wp * p;
  const int64_t row = (((int64_t)b * Fp + fp) * Hp + hp) * Wp + wp;
  const int col = ((c * t + tt) * p + i) * p + j;
  T* dst = out + row * ncol + col;
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    u.x = (uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16);
    u.y = (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16);
    u.z = (uint32_t)f2bf(bb.x) | ((uint32_t)f2bf(bb.y) << 16);
    u.w = (uint32_t)f2bf(bb.z) | ((uint32_t)f2bf(bb.w) << 16);
    *(uint4*)dst = u;
  } else {
    *(float4*)dst = a;
    *(float4*)(dst + 4) = bb;
  }
}

__global__ void sinusoid_kernel(int64_t n_pos, int64_t dim, float* out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n_pos * dim) return;
  const int64_t pos = i / dim, j = i % dim;
  const double angle = (double)pos / pow(10000.0, (double)(2 * (j / 2)) / (double)dim);
  out[i] = (float)((j % 2 == 0) ? sin(angle) : cos(angle));
}

// ---------------------------------------------------------------------------------------------
// column sums (bias gradients).  Vector kernel: block = 8 row-lanes x 32 column groups of 8
// columns (16-B bf16 / 2x16-B f32 loads), rows strided by 8 within the block's row range, 4 rows
// in flight per thread; partials reduced across row-lanes in LDS, one atomic per column per block.
// Scalar kernel: fallback for unaligned / cols % 8 != 0.
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void colsum8_kernel(const T* __restrict__ x, int64_t ldx, int64_t rows, int64_t cols,
                                                      float* __restrict__ out, int64_t rows_per_block) {
  __shared__ float part[8][257];
  const int cgi = threadIdx.x & 31, ry = threadIdx.x >> 5;
  const int64_t c = (blockIdx.x * 32 + cgi) * 8;
  const int64_t r0 = blockIdx.y * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > rows) r1 = rows;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + ry;
    for (; r + 24 < r1; r += 32) {
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const T* p = x + (r + 8 * u) * ldx + c;
        if constexpr (sizeof(T) == 2) {
          const uint4 w = *(const uint4*)p;
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[u][2 * k] = __uint_as_float(ww[k] << 16);
            v[u][2 * k + 1] = __uint_as_float(ww[k] & 0xffff0000u);
          }
        } else {
          const float4 a = *(const float4*)p, b = *(const float4*)((const float*)p + 4);
          v[u][0] = a.x; v[u][1] = a.y; v[u][2] = a.z; v[u][3] = a.w;
          v[u][4] = b.x; v[u][5] = b.y; v[u][6] = b.z; v[u][7] = b.w;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[u][k];
    }
    for (; r < r1; r += 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += Elem<T>::load(x + r * ldx + c + k);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[ry][cgi * 8 + k] = acc[k];
  __syncthreads();
  const int cc = threadIdx.x;  // one column per thread
  const int64_t col = blockIdx.x * 256 + cc;
  if (col < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += part[k][cc];
    unsafeAtomicAdd(out + col, s);
  }
}

template <typename T>
__global__ void colsum_kernel(const T* __restrict__ x, int64_t ldx, int64_t rows, int64_t cols, float* __restrict__ out,
                              int64_t rows_per_block) {
  __shared__ float part[4][64];
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t c = blockIdx.x * 64 + cx;
  const int64_t r0 = blockIdx.y * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > rows) r1 = rows;
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + ry; r < r1; r += 4) s += Elem<T>::load(x + r * ldx + c);
  part[ry][cx] = s;
  __syncthreads();
  if (ry == 0 && c < cols) unsafeAtomicAdd(out + c, part[0][cx] + part[1][cx] + part[2][cx] + part[3][cx]);
}

__global__ void cast_f32_bf16(const float* __restrict__ in, bf16_t* __restrict__ out, int64_t n) {
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * blockDim.x * 4) {
    if (i + 4 <= n) {
      const float4 v = *(const float4*)(in + i);
      ushort4 o;
      o.x = f2bf(v.x); o.y = f2bf(v.y); o.z = f2bf(v.z); o.w = f2bf(v.w);
      *(ushort4*)(out + i) = o;
    } else {
      for (int64_t k = i; k < n; ++k) out[k] = f2bf(in[k]);
    }
  }
}
__global__ void cast_bf16_f32(const bf16_t* __restrict__ in, float* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = bf2f(in[i]);
}

// ---------------------------------------------------------------------------------------------
// PoissonNLLLoss(log_input=True) or MSELoss, mean reduction, fused with its gradient.
// Stage 1: per-block partial sums (fixed order) + dx.  Stage 2: one block sums the partials in a
// fixed order -> deterministic loss.
// ---------------------------------------------------------------------------------------------
constexpr int kPoissonBlocks = 256;
enum { kLossPoisson = 0, kLossMse = 1 };

// the loss term and its derivative in x: Poisson exp(x) - y x, (exp(x) - y); MSE (x - y)^2, 2 (x - y)
template <int KIND>
__device__ __forceinline__ float loss_term(float x, float y, float& grad) {
  if constexpr (KIND == kLossPoisson) {
    const float ex = expf(x);
    grad = ex - y;
    return ex - y * x;
  } else {
    const float d = x - y;
    grad = 2.0f * d;
    return d * d;
  }
}

template <int KIND>
__global__ void loss_stage1(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ dx,
                            float gscale, int64_t n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float g;
    s += loss_term<KIND>(x[i], y[i], g);
    if (dx) dx[i] = gscale * g;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ void poisson_stage2(const float* __restrict__ partial, int nb, float inv_n, float* __restrict__ loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = ((red[0] + red[1]) + (red[2] + red[3])) * inv_n;
}
template <int KIND>
__global__ void loss_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ g,
                                float* __restrict__ dx, int64_t n) {
  const float s = g[0] / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gr;
    (void)loss_term<KIND>(x[i], y[i], gr);
    dx[i] = s * gr;
  }
}

// ---------------------------------------------------------------------------------------------
// AdamW (torch.optim.AdamW, single-tensor semantics, foreach=False/True agree):
//   p *= 1 - lr*wd;  m = m + (1-b1)*(g - m);  v = b2*v + (1-b2)*g*g
//   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// ---------------------------------------------------------------------------------------------
__global__ void adamw_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, bf16_t* __restrict__ plp, const float* __restrict__ hyper) {
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4], step = hyper[5],
              gs = hyper[6];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2s = sqrtf(1.f - powf(b2, step));
  const float step_size = lr / bc1;
  const float decay = 1.f - lr * wd;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float pi = p[i] * decay;
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (plp) plp[i] = f2bf(pi);
  }
}

static unsigned grid_for(int64_t n, int per_thread = 1) {
  int64_t b = cdiv(cdiv(n, per_thread), 256);
  if (b > 4096) b = 4096;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace vs

using namespace vs;

extern "C" int vs_patch_im2col(int32_t out_dtype, int64_t B, int64_t F, int64_t C, int64_t H, int64_t W,
                               int64_t tubelet, int64_t patch, const float* pixels, void* cols, void* stream) {
  VS_REQUIRE(pixels && cols, "vs_patch_im2col: null pointer");
  VS_REQUIRE(tubelet > 0 && patch > 0 && F % tubelet == 0 && H % patch == 0 && W % patch == 0,
             "vs_patch_im2col: frames/size must divide by tubelet/patch");
  VS_REQUIRE(patch % 8 == 0 && W % 4 == 0 && aligned16(pixels), "vs_patch_im2col: patch must be a multiple of 8");
  const int64_t total8 = B * (F / tubelet) * (H / patch) * (W / patch) * C * tubelet * patch * patch / 8;
  if (total8 == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_MISC, s, (double)total8 * 8.0 * (4.0 + (double)esize(out_dtype)));
  VS_REQUIRE(total8 < (1ll << 31) - 256 * 4096 && B * F * C * H * W < (1ll << 40), "vs_patch_im2col: batch too large");
  VS_REQUIRE((((uintptr_t)cols) & 15) == 0, "vs_patch_im2col: cols must be 16-byte aligned");
  VS_REQUIRE(W <= 256 && W % 8 == 0, "vs_patch_im2col: image width must be <= 256 and a multiple of 8");
  const dim3 grid((unsigned)(B * F), (unsigned)cdiv(C * H, 8));
  const bool vit = tubelet == 2 && patch == 16;  // the VideoMAE tubelet: compile-time index math
#define IM2COL_(TY, TT, PP)                                                                                           \
  hipLaunchKernelGGL((im2col_kernel<TY, TT, PP>), grid, dim3(256), 0, s, pixels, (TY*)cols, (int)F, (int)C, (int)H,   \
                     (int)W, (int)tubelet, (int)patch)
  if (out_dtype == VS_BF16) {
    if (vit) IM2COL_(bf16_t, 2, 16); else IM2COL_(bf16_t, 0, 0);
  } else {
    if (vit) IM2COL_(float, 2, 16); else IM2COL_(float, 0, 0);
  }
#undef IM2COL_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_sinusoid_table(int64_t n_pos, int64_t dim, float* out, void* stream) {
  VS_REQUIRE(out && n_pos >= 0 && dim > 0, "vs_sinusoid_table: bad args");
  if (n_pos == 0) return VS_OK;
  hipLaunchKernelGGL(sinusoid_kernel, dim3((unsigned)cdiv(n_pos * dim, 256)), dim3(256), 0, (hipStream_t)stream,
                     n_pos, dim, out);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_colsum(int32_t dtype, int64_t rows, int64_t cols, const void* x, int64_t ldx, float* out,
                         void* stream) {
  VS_REQUIRE(x && out && ldx >= cols, "vs_colsum: bad args");
  if (rows == 0 || cols == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_MISC, s, (double)rows * (double)cols * (double)esize(dtype) + (double)cols * 8.0);
  const int vec = dtype == VS_BF16 ? 8 : 4;
  if (cols % 8 == 0 && ldx % vec == 0 && aligned16(x)) {
    const int64_t cb = cdiv(cols, 256);
    int64_t rb = cdiv(512, cb);
    if (rb > cdiv(rows, 64)) rb = cdiv(rows, 64);
    if (rb < 1) rb = 1;
    const int64_t rpb = cdiv(rows, rb);
    dim3 grid((unsigned)cb, (unsigned)cdiv(rows, rpb));
    if (dtype == VS_BF16)
      hipLaunchKernelGGL(colsum8_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, rows, cols, out, rpb);
    else
      hipLaunchKernelGGL(colsum8_kernel<float>, grid, dim3(256), 0, s, (const float*)x, ldx, rows, cols, out, rpb);
  } else {
    const int64_t cb = cdiv(cols, 64);
    int64_t rb = cdiv(1024, cb);
    if (rb > cdiv(rows, 64)) rb = cdiv(rows, 64);
    if (rb < 1) rb = 1;
    const int64_t rpb = cdiv(rows, rb);
    dim3 grid((unsigned)cb, (unsigned)cdiv(rows, rpb));
    if (dtype == VS_BF16)
      hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, rows, cols, out, rpb);
    else
      hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)x, ldx, rows, cols, out, rpb);
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_cast(int32_t in_dtype, int32_t out_dtype, int64_t n, const void* in, void* out, void* stream) {
  VS_REQUIRE(in && out && n >= 0, "vs_cast: bad args");
  if (n == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_MISC, s, (double)n * (double)(esize(in_dtype) + esize(out_dtype)));
  if (in_dtype == VS_F32 && out_dtype == VS_BF16) {
    VS_REQUIRE(aligned16(in) && (((uintptr_t)out) & 7u) == 0, "vs_cast: misaligned");
    hipLaunchKernelGGL(cast_f32_bf16, dim3(grid_for(n, 4)), dim3(256), 0, s, (const float*)in, (bf16_t*)out, n);
  } else if (in_dtype == VS_BF16 && out_dtype == VS_F32) {
    hipLaunchKernelGGL(cast_bf16_f32, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)in, (float*)out, n);
  } else if (in_dtype == out_dtype) {
    hipError_t e = hipMemcpyAsync(out, in, n * esize(in_dtype), hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return (int)e;
    return VS_OK;
  } else {
    VS_REQUIRE(false, "vs_cast: bad dtype pair");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" size_t vs_poisson_workspace_bytes(int64_t n) {
  (void)n;
  return kPoissonBlocks * sizeof(float);
}

template <int KIND>
static int loss_fwd(int64_t n, const float* x, const float* y, float* loss_out, float* dx, float grad_scale,
                    void* workspace, hipStream_t s) {
  ScopedTimer timer(VS_TIMER_MISC, s, (double)n * (dx ? 12.0 : 8.0));
  int nb = (int)cdiv(n, 256);
  if (nb > kPoissonBlocks) nb = kPoissonBlocks;
  hipLaunchKernelGGL((loss_stage1<KIND>), dim3(nb), dim3(256), 0, s, x, y, dx, grad_scale / (float)n, n,
                     (float*)workspace);
  hipLaunchKernelGGL(poisson_stage2, dim3(1), dim3(256), 0, s, (const float*)workspace, nb, 1.0f / (float)n, loss_out);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_poisson_nll(int64_t n, const float* log_rate, const float* target, float* loss_out, float* dx,
                              float grad_scale, void* workspace, void* stream) {
  VS_REQUIRE(n > 0 && log_rate && target && loss_out && workspace, "vs_poisson_nll: bad args");
  return loss_fwd<kLossPoisson>(n, log_rate, target, loss_out, dx, grad_scale, workspace, (hipStream_t)stream);
}

extern "C" int vs_poisson_nll_bwd(int64_t n, const float* log_rate, const float* target, const float* grad_out,
                                  float* dx, void* stream) {
  VS_REQUIRE(n > 0 && log_rate && target && grad_out && dx, "vs_poisson_nll_bwd: bad args");
  hipLaunchKernelGGL((loss_bwd_kernel<kLossPoisson>), dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, log_rate,
                     target, grad_out, dx, n);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_mse_loss(int64_t n, const float* pred, const float* target, float* loss_out, float* dx,
                           float grad_scale, void* workspace, void* stream) {
  VS_REQUIRE(n > 0 && pred && target && loss_out && workspace, "vs_mse_loss: bad args");
  return loss_fwd<kLossMse>(n, pred, target, loss_out, dx, grad_scale, workspace, (hipStream_t)stream);
}

extern "C" int vs_mse_loss_bwd(int64_t n, const float* pred, const float* target, const float* grad_out, float* dx,
                               void* stream) {
  VS_REQUIRE(n > 0 && pred && target && grad_out && dx, "vs_mse_loss_bwd: bad args");
  hipLaunchKernelGGL((loss_bwd_kernel<kLossMse>), dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, pred, target,
                     grad_out, dx, n);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_adamw(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_lp,
                        const float* hyper, void* stream) {
  VS_REQUIRE(param && grad && exp_avg && exp_avg_sq && hyper && n >= 0, "vs_adamw: bad args");
  if (n == 0) return VS_OK;
  // algorithmic bytes: param, exp_avg, exp_avg_sq read + written, grad read, bf16 shadow written
  ScopedTimer timer(VS_TIMER_ADAMW, (hipStream_t)stream, (double)n * (28.0 + (param_lp ? 2.0 : 0.0)));
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, param, grad, exp_avg,
                     exp_avg_sq, (bf16_t*)param_lp, hyper);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
