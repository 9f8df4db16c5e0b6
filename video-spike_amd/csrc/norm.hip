// norm.hip — LayerNorm forward/backward over the hidden dim (mv:416-417,426,437; eps 1e-12).
//
// One wave per row; a lane holds columns lane + 64*i (i < VPL = cols/64, a template parameter
// so no slot is predicated away), giving coalesced 256-B wave accesses and keeping the row in
// registers between the statistics and the output pass (one HBM read of x).  Each wave keeps
// RPW rows in flight (all loads issued before the first reduction) to hide HBM latency — the
// first version with one row per wave measured 64 us for a 25,088 x 192 backward (~4x its
// byte floor).  The backward reduces dgamma/dbeta per block in LDS: one f32 atomic per column
// per block, or (with the workspace, as the ViT block passes it) one partial row per block that
// ln_partsum_kernel adds in a fixed order: bit-identical reruns.
#include <algorithm>

#include <cstdlib>

#include "common.h"

namespace vs {

// the backward's incoming gradient dy is f32, or bf16 in the bf16 ViT block (its dX products write
// dh in the compute dtype: one more bf16 rounding of a gradient, as every other bf16 operand)
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float4 ld4(const bf16_t* p) {
  const uint2 u = *(const uint2*)p;
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

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

template <int VPL, int RPW, typename TD>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD* __restrict__ dy, int64_t lddy,
                                                     const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ g, const float* __restrict__ dres,
                                                     int64_t lddres, float* __restrict__ dx, int64_t lddx,
                                                     bf16_t* __restrict__ dx_lp, float* __restrict__ dg,
                                                     float* __restrict__ db, float* __restrict__ part, int64_t rows,
                                                     int cols) {
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
        d[k][i] = in ? ld1(dy + row * lddy + c) : 0.f;
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
    if (part) {  // partial row of this block; ln_partsum_kernel adds the rows in a fixed order
      part[(int64_t)blockIdx.x * 2 * cols + c] = a;
      part[(int64_t)blockIdx.x * 2 * cols + cols + c] = bb;
    } else {
      unsafeAtomicAdd(dg + c, a);
      unsafeAtomicAdd(db + c, bb);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Vectorised variants for cols = LPR * VEC * 4 (192 = 16 x 3 x 4, 384, 768): a row belongs to a
// group of LPR lanes, each lane holds VEC float4 (16-B loads/stores), 64/LPR rows per wave at
// once, every input of the row issued before the first reduction, reductions by xor-shuffles
// inside the group.  The scalar kernels above (4-B accesses, 3 per lane at D = 192) measured
// 31-38 us for the 25,088 x 192 backward, ~40% of its byte floor.
// ---------------------------------------------------------------------------------------------
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void st4(float* p, float4 v) { *(float4*)p = v; }
__device__ __forceinline__ void st4(bf16_t* p, float4 v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
  u.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
  *(uint2*)p = u;
}

template <typename TO, int LPR, int VEC>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, TO* __restrict__ y, int64_t ldy,
                                                         float* __restrict__ mean, float* __restrict__ rstd,
                                                         int64_t rows) {
  constexpr int COLS = LPR * VEC * 4, GPB = 256 / LPR;  // groups (rows) per block pass
  const int gl = threadIdx.x % LPR;
  const float inv = 1.f / (float)COLS;
  float4 gam[VEC], bet[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    gam[j] = *(const float4*)(g + 4 * (gl + LPR * j));
    bet[j] = *(const float4*)(b + 4 * (gl + LPR * j));
  }
  for (int64_t row = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; row < rows; row += (int64_t)gridDim.x * GPB) {
    float4 v[VEC];
    const float* xr = x + row * ldx;
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = *(const float4*)(xr + 4 * (gl + LPR * j));
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float mu = group_sum<LPR>(s) * inv;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      v[j].x -= mu; v[j].y -= mu; v[j].z -= mu; v[j].w -= mu;
      q += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
    }
    const float rs = rsqrtf(group_sum<LPR>(q) * inv + eps);
    TO* yr = y + row * ldy;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float4 o;
      o.x = v[j].x * rs * gam[j].x + bet[j].x;
      o.y = v[j].y * rs * gam[j].y + bet[j].y;
      o.z = v[j].z * rs * gam[j].z + bet[j].z;
      o.w = v[j].w * rs * gam[j].w + bet[j].w;
      st4(yr + 4 * (gl + LPR * j), o);
    }
    if (gl == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
}

template <int LPR, int VEC, typename TD>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(const TD* __restrict__ dy, int64_t lddy,
                                                         const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const float* __restrict__ g,
                                                         const float* __restrict__ dres, int64_t lddres,
                                                         float* __restrict__ dx, int64_t lddx,
                                                         bf16_t* __restrict__ dx_lp, float* __restrict__ dg,
                                                         float* __restrict__ db, float* __restrict__ part,
                                                         int64_t rows) {
  constexpr int COLS = LPR * VEC * 4, GPB = 256 / LPR;
  __shared__ float red[2][4][COLS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, gl = threadIdx.x % LPR;
  const float inv = 1.f / (float)COLS;
  float4 gam[VEC], pg[VEC], pb[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    gam[j] = *(const float4*)(g + 4 * (gl + LPR * j));
    pg[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    pb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // rows strided by the grid; the next row's loads are issued before the current row's
  // reductions (software prefetch: the row loop was load-latency-bound at ~2 waves per SIMD)
  const int64_t stride = (int64_t)gridDim.x * GPB;
  int64_t row = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR;
  float4 d[VEC], xv[VEC], r[VEC];
  float mu = 0.f, rs = 0.f;
  auto load_row = [&](int64_t rw, float4* dd, float4* xx, float4* rr, float& m_, float& r_) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int c = 4 * (gl + LPR * j);
      dd[j] = ld4(dy + rw * lddy + c);
      xx[j] = *(const float4*)(x + rw * ldx + c);
      rr[j] = dres ? *(const float4*)(dres + rw * lddres + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    m_ = mean[rw];
    r_ = rstd[rw];
  };
  if (row < rows) load_row(row, d, xv, r, mu, rs);
  for (; row < rows; row += stride) {
    float4 dn[VEC], xn[VEC], rn[VEC];
    float mun = 0.f, rsn = 0.f;
    if (row + stride < rows) load_row(row + stride, dn, xn, rn, mun, rsn);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
#define VS_LNB(C)                          \
  {                                        \
    const float xh = (xv[j].C - mu) * rs;  \
    const float gy = d[j].C * gam[j].C;    \
    pg[j].C += d[j].C * xh;                \
    pb[j].C += d[j].C;                     \
    xv[j].C = xh;                          \
    d[j].C = gy;                           \
    s1 += gy;                              \
    s2 += gy * xh;                         \
  }
      VS_LNB(x) VS_LNB(y) VS_LNB(z) VS_LNB(w)
#undef VS_LNB
    }
    const float m1 = group_sum<LPR>(s1) * inv, m2 = group_sum<LPR>(s2) * inv;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int c = 4 * (gl + LPR * j);
      float4 o;
      o.x = rs * (d[j].x - m1 - xv[j].x * m2) + r[j].x;
      o.y = rs * (d[j].y - m1 - xv[j].y * m2) + r[j].y;
      o.z = rs * (d[j].z - m1 - xv[j].z * m2) + r[j].z;
      o.w = rs * (d[j].w - m1 - xv[j].w * m2) + r[j].w;
      *(float4*)(dx + row * lddx + c) = o;
      if (dx_lp) st4(dx_lp + row * lddx + c, o);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      d[j] = dn[j];
      xv[j] = xn[j];
      r[j] = rn[j];
    }
    mu = mun;
    rs = rsn;
  }
  // dgamma/dbeta: reduce the groups of the wave (same gl), then the 4 waves in LDS; one f32
  // atomic per column per block
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
#define VS_RED(V)                                                  \
  {                                                                \
    _Pragma("unroll") for (int o = LPR; o < 64; o <<= 1) {         \
      V.x += __shfl_xor(V.x, o, 64);                               \
      V.y += __shfl_xor(V.y, o, 64);                               \
      V.z += __shfl_xor(V.z, o, 64);                               \
      V.w += __shfl_xor(V.w, o, 64);                               \
    }                                                              \
  }
    VS_RED(pg[j]) VS_RED(pb[j])
#undef VS_RED
    if (lane < LPR) {
      *(float4*)&red[0][wid][4 * (gl + LPR * j)] = pg[j];
      *(float4*)&red[1][wid][4 * (gl + LPR * j)] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < COLS; c += 256) {
    const float a = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    const float bb = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
    if (part) {  // partial row of this block; ln_partsum_kernel adds the rows
      part[(int64_t)blockIdx.x * 2 * COLS + c] = a;
      part[(int64_t)blockIdx.x * 2 * COLS + COLS + c] = bb;
    } else {
      unsafeAtomicAdd(dg + c, a);
      unsafeAtomicAdd(db + c, bb);
    }
  }
}

// dgamma[c] += sum_b part[b][c], dbeta[c] += sum_b part[b][cols + c].  A block of 1024 threads owns
// 16 columns: thread t sums partial rows g, g+64, ... (g = t / 16: 64 row groups, 8 loads in
// flight), the 64 group sums meet in LDS and are added in group order: a fixed order (bitwise
// reproducible; the previous version finished with one f32 atomic per block and column).
__global__ __launch_bounds__(1024) void ln_partsum_kernel(const float* __restrict__ part, int nblk, int cols,
                                                          float* __restrict__ dg, float* __restrict__ db) {
  __shared__ float red[64][17];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4, ngrp = 64;
  const int c = blockIdx.x * 16 + cl, w = 2 * cols;
  float acc = 0.f;
  if (c < w) {
    int b = grp;
    for (; b + 7 * ngrp < nblk; b += 8 * ngrp) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(b + u * ngrp) * w + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < nblk; b += ngrp) acc += part[(int64_t)b * w + c];
  }
  red[grp][cl] = acc;
  __syncthreads();
  if (threadIdx.x < 16 && c < w) {
    float v = 0.f;
    for (int k = 0; k < 64; ++k) v += red[k][cl];
    if (c < cols) dg[c] += v;
    else db[c - cols] += v;
  }
}

constexpr int kLnBwdBlocks = 1024;  // vectorised backward grid cap (= partial rows in the workspace)

// cols -> (LPR, VEC) of the vectorised kernels; 0 = none
static inline int ln_vec_lpr(int64_t cols) {
  if (cols == 192) return 16;
  if (cols == 384) return 32;
  if (cols == 768) return 64;
  return 0;
}

template <typename TO, int VPL>
static void launch_fwd(int64_t rows, int64_t cols, const float* x, int64_t ldx, const float* gamma, const float* beta,
                       float eps, void* y, int64_t ldy, float* mean, float* rstd, hipStream_t s) {
  constexpr int RPW = VPL <= 4 ? 4 : (VPL <= 8 ? 2 : 1);
  dim3 grid((unsigned)cdiv(rows, 4 * RPW));
  hipLaunchKernelGGL((ln_fwd_kernel<TO, VPL, RPW>), grid, dim3(256), 0, s, x, ldx, gamma, beta, eps, (TO*)y, ldy, mean,
                     rstd, rows, (int)cols);
}

template <int VPL, typename TD>
static void launch_bwd(int64_t rows, int64_t cols, const TD* dy, int64_t lddy, const float* x, int64_t ldx,
                       const float* mean, const float* rstd, const float* gamma, const float* dres, int64_t lddres,
                       float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta, float* part,
                       hipStream_t s) {
  constexpr int RPW = VPL <= 4 ? 4 : (VPL <= 8 ? 2 : 1);
  int64_t nb = cdiv(rows, 4 * RPW * 2);  // ~2 row-groups per wave: amortises the column reduction
  if (nb > (part ? kLnBwdBlocks : 2048)) nb = part ? kLnBwdBlocks : 2048;   // (part: one row per block)
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL((ln_bwd_kernel<VPL, RPW, TD>), dim3((unsigned)nb), dim3(256), 0, s, dy, lddy, x, ldx, mean, rstd,
                     gamma, dres, lddres, dx, lddx, (bf16_t*)dx_lp, dgamma, dbeta, part, rows, (int)cols);
  if (part)
    hipLaunchKernelGGL(ln_partsum_kernel, dim3((unsigned)cdiv(2 * cols, 16)), dim3(1024), 0, s, part, (int)nb,
                       (int)cols, dgamma, dbeta);
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
  // algorithmic bytes: x read, y written, mean / rstd written, gamma / beta read
  ScopedTimer timer(VS_TIMER_LN_FWD, s,
                    (double)rows * (double)cols * (4.0 + (double)esize(y_dtype)) + (double)rows * 8.0 + (double)cols * 8.0);
  const int lpr = ln_vec_lpr(cols);
  if (lpr && ldx % 4 == 0 && ldy % 4 == 0 && aligned16(x) && aligned16(gamma) && aligned16(beta) &&
      (((uintptr_t)y) & (y_dtype == VS_BF16 ? 7 : 15)) == 0) {
    // grid cap 768 by default (was 2,048: 1,792 blocks fit the chip at 66 VGPRs, the rest ran as a tail;
    // fewer, longer-lived blocks measured faster still: C3 width 189.5 -> 168.7 us, profiles/r06_lnf_ab.json;
    // per-row work, so the outputs are bitwise the same); VS_KNOB_LN_FWD_BLOCKS overrides
    const int fk = knob(VS_KNOB_LN_FWD_BLOCKS);
    const unsigned grid = (unsigned)std::min<int64_t>(cdiv(rows, 256 / lpr), fk > 0 ? fk : 768);
#define FV_(TO, L) \
  hipLaunchKernelGGL((ln_fwd_vec_kernel<TO, L, 3>), dim3(grid), dim3(256), 0, s, x, ldx, gamma, beta, eps, (TO*)y, ldy, mean, rstd, rows)
    if (y_dtype == VS_BF16) {
      if (lpr == 16) FV_(bf16_t, 16); else if (lpr == 32) FV_(bf16_t, 32); else FV_(bf16_t, 64);
    } else {
      if (lpr == 16) FV_(float, 16); else if (lpr == 32) FV_(float, 32); else FV_(float, 64);
    }
#undef FV_
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
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

namespace vs {
void launch_ln_partsum(const float* part, int nblk, int cols, float* dgamma, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(ln_partsum_kernel, dim3((unsigned)cdiv(2 * cols, 16)), dim3(1024), 0, s, part, nblk, cols, dgamma,
                     dbeta);
}
}  // namespace vs

extern "C" size_t vs_layernorm_bwd_workspace_bytes(int64_t rows, int64_t cols) {
  (void)rows;
  return (size_t)kLnBwdBlocks * 2 * (size_t)(cols > 0 ? cols : 0) * sizeof(float);
}

template <typename TD>
static int layernorm_bwd_t(int64_t rows, int64_t cols, const TD* dy, int64_t lddy, const float* x, int64_t ldx,
                           const float* mean, const float* rstd, const float* gamma, const float* dres, int64_t lddres,
                           float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta, void* workspace,
                           hipStream_t s) {
  constexpr bool BF = sizeof(TD) == 2;
  // algorithmic bytes: dy, x, (dres) read, dx (+ its bf16 copy) written, row stats, gamma, dgamma/dbeta
  ScopedTimer timer(VS_TIMER_LN_BWD, s,
                    (double)rows * (double)cols * ((BF ? 2.0 : 4.0) + 8.0 + (dres ? 4.0 : 0.0) + (dx_lp ? 2.0 : 0.0)) +
                        (double)rows * 8.0 + (double)cols * 20.0);
  const int lpr = ln_vec_lpr(cols);
  if (lpr && lddy % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 && (!dres || (lddres % 4 == 0 && aligned16(dres))) &&
      (((uintptr_t)dy) & (BF ? 7 : 15)) == 0 && aligned16(x) && aligned16(dx) && aligned16(gamma) &&
      (!dx_lp || (((uintptr_t)dx_lp) & 7) == 0)) {
    // grid cap (= partial rows) 512 by default: at ~160 VGPRs only 3 of these 4-wave blocks fit a CU, so
    // 1,024 blocks ran as one full round plus a one-third-occupied tail (C3 LN': 535 -> 444 us per launch,
    // C2 width 139 -> 120 us; profiles/r06_ln_ab.json); VS_KNOB_LN_BLOCKS overrides
    const int kc = knob(VS_KNOB_LN_BLOCKS);
    const int cap = kc > 0 && kc <= kLnBwdBlocks ? kc : 512;
    const unsigned grid = (unsigned)std::min<int64_t>(cdiv(rows, 256 / lpr), cap);
    float* part = (float*)workspace;
#define BV_(L)                                                                                                       \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<L, 3, TD>), dim3(grid), dim3(256), 0, s, dy, lddy, x, ldx, mean, rstd, gamma, \
                     dres, lddres, dx, lddx, (bf16_t*)dx_lp, dgamma, dbeta, part, rows)
    if (lpr == 16) BV_(16); else if (lpr == 32) BV_(32); else BV_(64);
#undef BV_
    if (part)
      hipLaunchKernelGGL(ln_partsum_kernel, dim3((unsigned)cdiv(2 * cols, 16)), dim3(1024), 0, s, part, (int)grid,
                         (int)cols, dgamma, dbeta);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
#define B_(V) launch_bwd<V, TD>(rows, cols, dy, lddy, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx, dx_lp, dgamma, \
                                dbeta, (float*)workspace, s)
  VS_LN_DISPATCH(B_);
#undef B_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_layernorm_bwd(int64_t rows, int64_t cols, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                const float* mean, const float* rstd, const float* gamma, const float* dres,
                                int64_t lddres, float* dx, int64_t lddx, void* dx_lp, float* dgamma, float* dbeta,
                                void* workspace, void* stream) {
  return vs_layernorm_bwd_dt(VS_F32, rows, cols, dy, lddy, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx, dx_lp,
                             dgamma, dbeta, workspace, stream);
}

extern "C" int vs_layernorm_bwd_dt(int32_t dy_dtype, int64_t rows, int64_t cols, const void* dy, int64_t lddy,
                                   const float* x, int64_t ldx, const float* mean, const float* rstd,
                                   const float* gamma, const float* dres, int64_t lddres, float* dx, int64_t lddx,
                                   void* dx_lp, float* dgamma, float* dbeta, void* workspace, void* stream) {
  VS_REQUIRE(dy && x && mean && rstd && gamma && dx && dgamma && dbeta, "vs_layernorm_bwd: null pointer");
  VS_REQUIRE(cols > 0 && cols <= 1024, "vs_layernorm_bwd: cols must be in [1, 1024]");
  VS_REQUIRE(dy_dtype == VS_F32 || dy_dtype == VS_BF16, "vs_layernorm_bwd: dy must be f32 or bf16");
  if (rows == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dy_dtype == VS_BF16)
    return layernorm_bwd_t(rows, cols, (const bf16_t*)dy, lddy, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx,
                           dx_lp, dgamma, dbeta, workspace, s);
  return layernorm_bwd_t(rows, cols, (const float*)dy, lddy, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx, dx_lp,
                         dgamma, dbeta, workspace, s);
}
