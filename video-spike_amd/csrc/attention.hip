// attention.hip — non-causal MHA over frame-patch tokens, head dim 64 (mv:230-266, 286-294).
//
// bf16 (performance) path — v_mfma_f32_32x32x16_bf16, f32 accumulation, online softmax:
//   forward: workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32 queries.
//     S^T = K Q^T is computed with the KEY on the accumulator row and the QUERY on the lane, so a
//     lane owns one query's whole softmax state (max, sum) — no cross-lane reductions except one
//     xor-32 swap per 64-key tile.  The exponentiated S^T accumulator is directly the B operand of
//     O^T += V^T P^T (no LDS round trip); V^T fragments come from ds_read_tr16_b64 on the V tile.
//     K/V tiles (64 keys) are register-staged into double-buffered, XOR-swizzled LDS images.
//   backward: two atomic-free kernels.  dK/dV is key-major (each wave keeps 32 keys' K, V as MFMA
//     operands and dK^T, dV^T in accumulators while sweeping 32-query blocks); dQ is query-major
//     like the forward (LSE and delta are per-lane constants).  Summing dQ across key blocks with
//     f32 atomics instead was measured atomic-rate-bound (~489 MB of adds per ViT-Tiny launch at
//     ~1.3 TB/s: 466 us/launch, profiles/r01_v0_kernel_stats.csv), so dQ recomputes S and dP.
// f32 (parity) path — exact-f32 VALU kernels: 4 lanes per query/key row, K/V (or Q/dO) tiles in
//   LDS, expf/logf in f32.  Used for the 1e-4-relative parity mode.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace vs {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ============================================================================================
// f32 kernels
// ============================================================================================
__global__ __launch_bounds__(256) void attn_fwd_f32_kernel(const float* __restrict__ qkv, int64_t ldq,
                                                           float* __restrict__ o, int64_t ldo, float* __restrict__ lse,
                                                           int N, int H, float scale) {
  __shared__ float sK[64][68];
  __shared__ float sV[64][68];
  const int tid = threadIdx.x, sub = tid & 3;
  const int qi = blockIdx.x * 64 + (tid >> 2);
  const int h = blockIdx.y, b = blockIdx.z, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const float* Qp = qkv + row0 * ldq + h * 64;
  const float* Kp = Qp + D;
  const float* Vp = Qp + 2 * D;
  float q[16], acc[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    q[d] = qi < N ? Qp[(int64_t)qi * ldq + sub * 16 + d] : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int nkt = (N + 63) / 64;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63, gk = kt * 64 + r;
      sK[r][c] = gk < N ? Kp[(int64_t)gk * ldq + c] : 0.f;
      sV[r][c] = gk < N ? Vp[(int64_t)gk * ldq + c] : 0.f;
    }
    __syncthreads();
    float s[64];
    float mt = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 64; ++kk) {
      float part = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) part = fmaf(q[d], sK[kk][sub * 16 + d], part);
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      s[kk] = (kt * 64 + kk < N) ? part * scale : -INFINITY;
      mt = fmaxf(mt, s[kk]);
    }
    const float mn = fmaxf(m, mt);
    const float alpha = expf(m - mn);
    l *= alpha;
#pragma unroll
    for (int d = 0; d < 16; ++d) acc[d] *= alpha;
#pragma unroll
    for (int kk = 0; kk < 64; ++kk) {
      const float p = expf(s[kk] - mn);
      l += p;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] = fmaf(p, sV[kk][sub * 16 + d], acc[d]);
    }
    m = mn;
  }
  if (qi < N) {
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < 16; ++d) o[(row0 + qi) * ldo + h * 64 + sub * 16 + d] = acc[d] * inv;
    if (sub == 0) lse[((int64_t)b * H + h) * N + qi] = m + logf(l);
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dkdv_f32_kernel(const float* __restrict__ qkv, int64_t ldq,
                                                                const float* __restrict__ dout, int64_t lddo,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                float* __restrict__ dqkv, int64_t ldd, int N, int H,
                                                                float scale) {
  __shared__ float sQ[64][68];
  __shared__ float sD[64][68];
  __shared__ float sL[64], sDel[64];
  const int tid = threadIdx.x, sub = tid & 3;
  const int ki = blockIdx.x * 64 + (tid >> 2);
  const int h = blockIdx.y, b = blockIdx.z, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const float* Qp = qkv + row0 * ldq + h * 64;
  const float* Kp = Qp + D;
  const float* Vp = Qp + 2 * D;
  const float* Dp = dout + row0 * lddo + h * 64;
  const float* L = lse + ((int64_t)b * H + h) * N;
  const float* Del = delta + ((int64_t)b * H + h) * N;
  float k[16], v[16], dk[16], dv[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    k[d] = ki < N ? Kp[(int64_t)ki * ldq + sub * 16 + d] : 0.f;
    v[d] = ki < N ? Vp[(int64_t)ki * ldq + sub * 16 + d] : 0.f;
    dk[d] = dv[d] = 0.f;
  }
  const int nqt = (N + 63) / 64;
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63, gq = qt * 64 + r;
      sQ[r][c] = gq < N ? Qp[(int64_t)gq * ldq + c] : 0.f;
      sD[r][c] = gq < N ? Dp[(int64_t)gq * lddo + c] : 0.f;
    }
    if (tid < 64) {
      const int gq = qt * 64 + tid;
      sL[tid] = gq < N ? L[gq] : INFINITY;
      sDel[tid] = gq < N ? Del[gq] : 0.f;
    }
    __syncthreads();
    for (int qq = 0; qq < 64; ++qq) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        s = fmaf(sQ[qq][sub * 16 + d], k[d], s);
        dp = fmaf(sD[qq][sub * 16 + d], v[d], dp);
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      dp += __shfl_xor(dp, 1, 64);
      dp += __shfl_xor(dp, 2, 64);
      const float p = expf(s * scale - sL[qq]);
      const float ds = p * (dp - sDel[qq]);
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        dv[d] = fmaf(p, sD[qq][sub * 16 + d], dv[d]);
        dk[d] = fmaf(ds, sQ[qq][sub * 16 + d], dk[d]);
      }
    }
  }
  if (ki < N) {
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      dqkv[(row0 + ki) * ldd + D + h * 64 + sub * 16 + d] = dk[d] * scale;
      dqkv[(row0 + ki) * ldd + 2 * D + h * 64 + sub * 16 + d] = dv[d];
    }
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_f32_kernel(const float* __restrict__ qkv, int64_t ldq,
                                                              const float* __restrict__ dout, int64_t lddo,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta, float* __restrict__ dqkv,
                                                              int64_t ldd, int N, int H, float scale) {
  __shared__ float sK[64][68];
  __shared__ float sV[64][68];
  const int tid = threadIdx.x, sub = tid & 3;
  const int qi = blockIdx.x * 64 + (tid >> 2);
  const int h = blockIdx.y, b = blockIdx.z, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const float* Qp = qkv + row0 * ldq + h * 64;
  const float* Kp = Qp + D;
  const float* Vp = Qp + 2 * D;
  const float* Dp = dout + row0 * lddo + h * 64;
  float q[16], g[16], dq[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    q[d] = qi < N ? Qp[(int64_t)qi * ldq + sub * 16 + d] : 0.f;
    g[d] = qi < N ? Dp[(int64_t)qi * lddo + sub * 16 + d] : 0.f;
    dq[d] = 0.f;
  }
  const float li = qi < N ? lse[((int64_t)b * H + h) * N + qi] : INFINITY;
  const float deli = qi < N ? delta[((int64_t)b * H + h) * N + qi] : 0.f;
  const int nkt = (N + 63) / 64;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63, gk = kt * 64 + r;
      sK[r][c] = gk < N ? Kp[(int64_t)gk * ldq + c] : 0.f;
      sV[r][c] = gk < N ? Vp[(int64_t)gk * ldq + c] : 0.f;
    }
    __syncthreads();
    const int lim = N - kt * 64 < 64 ? N - kt * 64 : 64;
    for (int kk = 0; kk < lim; ++kk) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        s = fmaf(q[d], sK[kk][sub * 16 + d], s);
        dp = fmaf(g[d], sV[kk][sub * 16 + d], dp);
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      dp += __shfl_xor(dp, 1, 64);
      dp += __shfl_xor(dp, 2, 64);
      const float p = expf(s * scale - li);
      const float ds = p * (dp - deli);
#pragma unroll
      for (int d = 0; d < 16; ++d) dq[d] = fmaf(ds, sK[kk][sub * 16 + d], dq[d]);
    }
  }
  if (qi < N) {
#pragma unroll
    for (int d = 0; d < 16; ++d) dqkv[(row0 + qi) * ldd + h * 64 + sub * 16 + d] = dq[d] * scale;
  }
}

// delta[b,h,n] = sum_d dO[n, h*64+d] * O[n, h*64+d]   (one wave per (row, head))
template <typename T>
__global__ __launch_bounds__(256) void attn_delta_kernel(const T* __restrict__ o, int64_t ldo, const T* __restrict__ dout,
                                                         int64_t lddo, float* __restrict__ delta, int64_t rows, int N,
                                                         int H) {
  const int lane = threadIdx.x & 63;
  const int64_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= rows * H) return;
  const int64_t row = w / H;
  const int h = (int)(w % H);
  float v = Elem<T>::load(o + row * ldo + h * 64 + lane) * Elem<T>::load(dout + row * lddo + h * 64 + lane);
  v = wave_sum(v);
  if (lane == 0) {
    const int64_t b = row / N, n = row % N;
    delta[(b * H + h) * N + n] = v;
  }
}

// ============================================================================================
// bf16 MFMA kernels
// ============================================================================================
__device__ __forceinline__ int swz_row(int r) { return (r >> 1) & 7; }           // 16-B chunk XOR
__device__ __forceinline__ int swz_half(int r) { return ((r >> 1) & 1) << 2; }   // 64-B half XOR

// byte offset of element (r, c) (c multiple of 4 for tr reads) in a 128-B-row image
__device__ __forceinline__ int off_rowswz(int r, int c) { return r * 128 + (((c >> 3) ^ swz_row(r)) << 4) + (c & 7) * 2; }
__device__ __forceinline__ int off_halfswz(int r, int c) { return r * 128 + (((c >> 3) ^ swz_half(r)) << 4) + (c & 7) * 2; }

__device__ __forceinline__ bf16x8 tr_pair(const char* lds, int off0, int off1) {
  short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(lds + off0));
  short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(lds + off1));
  typedef __attribute__((ext_vector_type(8))) short short8v;
  short8v s = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, s);
}

typedef __attribute__((ext_vector_type(8))) float f32x8;
// 8 f32 -> 8 bf16 as four v_cvt_pk_bf16_f32 (element-wise casts cost one cvt per value)
__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int base) {
  const f32x8 v = {a[base], a[base + 1], a[base + 2], a[base + 3], a[base + 4], a[base + 5], a[base + 6], a[base + 7]};
  return __builtin_convertvector(v, bf16x8);
}
__device__ __forceinline__ bf16x8 pack8f(const float* a) {
  const f32x8 v = {a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
  return __builtin_convertvector(v, bf16x8);
}

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  uint2 u;
  u.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
  u.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16);
  return u;
}

// ------------------------------------------------------------------ forward
// Per 64-key tile and wave (32 queries): 8 MFMAs for S^T = K (c Q)^T and 8 for O^T += V^T P^T.
// VALU per score is minimised:
//   * Q is pre-scaled by c = log2(e)/sqrt(64) when loaded, and the running max enters the QK^T
//     chain as the MFMA's C operand (a splat of -m that is only rewritten when m moves), so the
//     accumulator IS log2(p): p = v_exp_f32(acc) with no per-score FMA;
//   * the max is lazily raised (only when a lane's scores exceed m by 2^kRescaleThr, guide T13);
//     the O/l rescale is a wave-uniform branch that is skipped in steady state, P <= 2^kRescaleThr;
//   * max via v_max3 (asm: hipcc canonicalises fmaxf operands), xor-32 exchange via
//     v_permlane32_swap (no LDS), staging loads unconditional (clamped row + select);
//   * the tile loop is unrolled over the two LDS buffers so every LDS address is a per-lane base
//     plus an immediate offset.
// Softmax VALU of sub-block j overlaps the MFMAs of sub-block j+1 (issue order QK1, SM0, PV0,
// SM1, PV1).
constexpr float kRescaleThr = 8.0f;
constexpr float kRefBand = 32.0f;
#ifndef VS_FWD_TOPBAR
#define VS_FWD_TOPBAR 0
#endif  // forward: p <= 2^32 relative to the reference (f32/bf16-safe)

__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max16(const f32x16& x) {
  const float a = max3f(x[0], x[1], x[2]), b = max3f(x[3], x[4], x[5]), c = max3f(x[6], x[7], x[8]);
  const float d = max3f(x[9], x[10], x[11]), e = max3f(x[12], x[13], x[14]);
  return max3f(max3f(a, b, c), max3f(d, e, x[15]), -INFINITY);
}
// v_permlane32_swap(v, v) returns {v[lane & 31], v[32 + (lane & 31)]}: both halves' values in
// every lane, so a pair reduction over lanes l and l^32 needs no LDS round trip.
__device__ __forceinline__ float pair_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max3f(__uint_as_float(r[0]), __uint_as_float(r[1]), -INFINITY);
}
__device__ __forceinline__ float pair_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}


// VS_ATTN_PRIO (diagnostic builds): every 32x32x16 MFMA issued at raised wave priority
// (s_setprio 1 / 0 around it), so a wave with an MFMA ready wins the issue port over VALU work
__device__ __forceinline__ f32x16 mfma32p(const bf16x8& a, const bf16x8& b, const f32x16& c) {
#ifdef VS_ATTN_PRIO
  __builtin_amdgcn_s_setprio(1);
  const f32x16 r = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
  return r;
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}

// VS_ATTN_DIAG (diagnostic builds only): bit 0 = the forward streams only its first two K/V tiles,
// bit 1 = the backward (both passes) only its first two Q/dO or K/V slices: the rest of the tiles are
// computed on stale LDS data, which times the kernels without their LDS-DMA fill (results WRONG)
#ifndef VS_ATTN_DIAG
#define VS_ATTN_DIAG 0
#endif

#ifdef VS_STAMP
// Diagnostic build only (-DVS_STAMP): per wave {start, end} realtime ticks (100 MHz), HW ids, and
// shader-clock cycles accumulated in the forward's barrier and vmcnt waits; read back with
// vs_dbg_stamps().  Not part of the product library.
__device__ unsigned long long g_stamp[8 * 8192];
__device__ __forceinline__ void stamp(int slot, bool end) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w < 8192) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (!end) {
      g_stamp[8 * w] = t;
      g_stamp[8 * w + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      g_stamp[8 * w + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    } else {
      g_stamp[8 * w + 1] = t;
    }
  }
  (void)slot;
}
__device__ __forceinline__ void stamp_acc(int slot, unsigned long long v) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w < 8192) g_stamp[8 * w + slot] = v;
}
#define VS_CLK() __builtin_amdgcn_s_memtime()
#define VS_STAMP_AT(end) stamp(0, end)
#else
#define VS_STAMP_AT(end)
#define VS_CLK() 0ull
#endif

// Row sums of P on the matrix pipe.  For v_mfma_f32_16x16x32_bf16 with P's packed half (pa or pb,
// this lane's 8 keys of query lane&31) as the B operand, column n = lane&15 collects lanes n, n+16,
// n+32, n+48 = queries n, n+16, n, n+16 in k-slot groups g = lane>>4 = 0..3.  The constant A
// operand `sel` has row 0 = ones over groups {0, 2} and row 1 = ones over groups {1, 3}, so row 0
// of the product is query n's sum over the block's keys and row 1 query n+16's.  Two 16-cycle
// MFMAs per 32-key block replace 15 v_add_f32 per lane (60 VALU issue cycles).
__device__ __forceinline__ bf16x8 rowsum_selector(int lane) {
  const int row = lane & 15, g = lane >> 4;
  const float one = (row == 0 && (g & 1) == 0) || (row == 1 && (g & 1) == 1) ? 1.f : 0.f;
  const f32x8 v = {one, one, one, one, one, one, one, one};
  return __builtin_convertvector(v, bf16x8);
}

// workgroups of the bf16 forward that re-ran their tile under the safe softmax (a query's scores
// left the fast pass's band): read / reset by vs_attn_redo_count
__device__ unsigned long long g_attn_redo = 0;

// ORD: the order of a 64-key tile's work (blocks a = keys 0..31, b = 32..63)
//   0: QK(a), softmax(a), PV(a), QK(b), softmax(b), PV(b)                (round 2)
//   1: QK(b) issued before PV(a), so softmax(b) waits on a chain that ran under PV(a)'s MFMAs (round 3)
//   2: software-pipelined across tiles: every softmax runs under the NEXT block's QK MFMAs, including
//      softmax(b) under QK(a) of tile kt + 1 (ORD 1 leaves softmax(b) with only its two row-sum
//      MFMAs to hide under): per tile  [QK(b) | softmax(a)] [PV(a) | V(b) reads] barrier
//      [QK(a') | softmax(b)] [PV(b) | V(a'), K(b') reads]  (round 6, VS_KNOB_ATTN_VARIANT 7).  Its two
//      blocks' live state needs ~206 VGPRs: 2 waves per SIMD, measured 9 % SLOWER than ORD 1's 3 waves
//      (at 3 waves / 168 VGPRs it spills 81); bitwise the same outputs
//   ORD 1 with the last tile peeled (no tail branch in the steady loop, so QK(b)'s MFMAs and softmax(a)
//   share one basic block) spilled 52 VGPRs at 168 and was dropped (round 6)
template <int ORD = 1>
__global__ __launch_bounds__(256, ORD == 2 ? 2 : 3) void attn_fwd_bf16_kernel(const bf16_t* __restrict__ qkv, int64_t ldq,
                                                               bf16_t* __restrict__ o, int64_t ldo,
                                                               float* __restrict__ lse, int N, int H,
                                                               float scale_log2) {
  constexpr int TILE = 64 * 128;  // bytes of one 64-key x 64-dh bf16 tile
  // Two K/V stages as separate __shared__ objects (DMA into one while the other is read).
  __shared__ __attribute__((aligned(16))) char smem0[2 * TILE];
  __shared__ __attribute__((aligned(16))) char smem1[2 * TILE];
  __shared__ int redo_flag;
  VS_STAMP_AT(false);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb128 = (N + 127) / 128, blk = xcd_remap(blockIdx.x, gridDim.x), qb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const int q0w = qb * 128 + wid * 32;  // this wave's first query
  const int qi = q0w + (lane & 31);
  const float c = scale_log2;
  if (tid == 0) redo_flag = 0;

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int qr = qi < N ? qi : N - 1;
    const bf16x8 q = *(const bf16x8*)(Qp + (int64_t)qr * ldq + 16 * s + 8 * hh);
    f32x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)q[j] * c;
    qf[s] = __builtin_convertvector(v, bf16x8);
  }
  const bf16x8 sel = rowsum_selector(lane);
  f32x16 oacc[2], zero16;
  f32x4 lacc;
  float m_run, l_half;

  // Per-lane LDS byte offsets, tile-invariant.  Every read is a lane base plus an immediate:
  //  K rows key = kb*32 + (lane&31): swz_row(key + 32) == swz_row(key), so kb adds 32*128 B;
  //  the 4 k-chunks XOR (2s+hh) into the swizzled chunk index -> one base per s.
  //  V^T reads rows k0 = kb*32 + 16s + 4hh + q4 (+8): swz_half(k0) depends on q4 bit 1 only, so
  //  kb/s/+8 are immediates and dt (64-B half) just selects one of two bases.
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = ((lane >> 4) & 1) * 16;
  int kbase[4];
  {
    const int key = lane & 31;
#pragma unroll
    for (int s = 0; s < 4; ++s) kbase[s] = key * 128 + (((2 * s + hh) ^ swz_row(key)) << 4);
  }
  int vbase[2];
  {
    const int k0 = 4 * hh + q4;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) vbase[dt] = TILE + off_halfswz(k0, dt * 32 + g16 + p4);
  }
  // K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4): one wave-instruction fills a 1-KiB
  // piece = 8 rows x 128 B, lane L writing position L*16.  The LDS images keep their XOR swizzles
  // because each lane loads the SOURCE chunk that belongs at its position: (L&7) ^ swz(row).  Wave
  // w fills K pieces 2w, 2w+1 and V pieces 2w, 2w+1.  The asm DMA (SGPR tile base + per-lane
  // offset) is invisible to hipcc's waitcnt insertion, which would otherwise drain the in-flight
  // tile before LDS reads of the other stage; ordering is the loop's explicit vmcnt(0) + barrier.
  const int prow0 = wid * 16 + (lane >> 3), ppos = lane & 7;  // rows prow0 and prow0 + 8
  const uint32_t gk0 = (uint32_t)(prow0 * 2 * ldq + ((ppos ^ swz_row(prow0)) << 4));
  const uint32_t gk1 = (uint32_t)((prow0 + 8) * 2 * ldq + ((ppos ^ swz_row(prow0 + 8)) << 4));
  const uint32_t gv0 = (uint32_t)(prow0 * 2 * ldq + ((ppos ^ swz_half(prow0)) << 4));
  const uint32_t gv1 = (uint32_t)((prow0 + 8) * 2 * ldq + ((ppos ^ swz_half(prow0 + 8)) << 4));
  const int64_t tile_bytes = 64 * 2 * ldq, vdelta = 2 * (int64_t)D;
  auto load_tile = [&](int kt, char* buf) {
    const char* kb = (const char*)Kp + kt * tile_bytes;
    const char* vb = kb + vdelta;
    char* dk = buf + wid * 2048;
    char* dv = buf + TILE + wid * 2048;
    if ((kt + 1) * 64 <= N) {
      glds16_asm_so(kb, gk0, dk);
      glds16_asm_so(kb, gk1, dk + 1024);
      glds16_asm_so(vb, gv0, dv);
      glds16_asm_so(vb, gv1, dv + 1024);
    } else {  // partial last tile: rows past N re-read row N-1 (finite data; its scores are masked)
      const int r0 = kt * 64 + prow0, r1 = r0 + 8;
      const uint32_t c0 = (uint32_t)((r0 < N ? r0 : N - 1) - kt * 64) * (uint32_t)(2 * ldq);
      const uint32_t c1 = (uint32_t)((r1 < N ? r1 : N - 1) - kt * 64) * (uint32_t)(2 * ldq);
      glds16_asm_so(kb, c0 + ((ppos ^ swz_row(prow0)) << 4), dk);
      glds16_asm_so(kb, c1 + ((ppos ^ swz_row(prow0 + 8)) << 4), dk + 1024);
      glds16_asm_so(vb, c0 + ((ppos ^ swz_half(prow0)) << 4), dv);
      glds16_asm_so(vb, c1 + ((ppos ^ swz_half(prow0 + 8)) << 4), dv + 1024);
    }
  };
  struct KFrag {
    bf16x8 k[4];
  };
  struct VFrag {
    bf16x8 v[4];
  };
  auto kread = [&](const char* base, int kb) {
    KFrag f;
#pragma unroll
    for (int s = 0; s < 4; ++s) f.k[s] = *(const bf16x8*)(base + kb * 4096 + kbase[s]);
    return f;
  };
  auto vread = [&](const char* base, int kb) {
    VFrag f;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const char* vb = base + kb * 4096 + s * 2048;
        f.v[2 * s + dt] = tr_pair(vb, vbase[dt], vbase[dt] + 1024);
      }
    return f;
  };
  auto pv = [&](const VFrag& f, const bf16x8& pa, const bf16x8& pb) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
        oacc[dt] = mfma32p(f.v[2 * s + dt], s == 0 ? pa : pb, oacc[dt]);
  };

  // Softmax of one 32-key block.  acc = log2-domain scores s (Q pre-scaled by c; the MFMA chain
  // starts from 0).
  //  FAST pass (SAFE = 0): p = exp2(s) against a fixed reference 0 — no row maximum, no rescale,
  //    no per-score subtraction; row sums on the matrix pipe (lacc).  Exact whenever every query's
  //    scores stay within about [-100, 85] (log2 units); the epilogue checks the row sums and, if
  //    any query of the workgroup is outside that band (or overflowed), the workgroup re-runs
  //  SAFE pass (SAFE = 1): online softmax against a running reference that is raised lazily (a
  //    wave-uniform rare branch when a score exceeds it by 2^kRefBand, guide T13) and is set from
  //    the first block's maximum; p = exp2(s - m); VALU row sums.
  // maskc: IC<1> where the block may hold keys past N (the last tile), IC<0> in the pipelined loop's
  // full tiles (no tail branch there: a branch between QK(b)'s MFMAs and softmax(a)'s VALU splits the
  // basic block and the in-order wave then issues the two back to back instead of interleaved)
  auto softmax_m = [&](auto safec, auto maskc, f32x16& acc, int key0, bool first_blk, bf16x8& pa, bf16x8& pb) {
    constexpr bool SAFE = decltype(safec)::value;
    if (decltype(maskc)::value && key0 + 32 > N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key0 + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) acc[r] = -INFINITY;
    }
    float p[16];
    if constexpr (!SAFE) {
#pragma unroll
      for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(acc[r]);
    } else {
      const float mx = max16(acc);
      if (__any(first_blk || mx > m_run + kRefBand)) {
        const float mxp = pair_max(mx);  // the query's maximum over this block's 32 keys
        const bool move = first_blk || mxp > m_run + kRefBand;
        const float m_new = move ? mxp : m_run;  // identical in both lanes of a query
        const float alpha = first_blk ? 1.f : __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        l_half *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          oacc[0][r] *= alpha;
          oacc[1][r] *= alpha;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(acc[r] - m_run);
      l_half += ((((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]))) +
                 (((p[8] + p[9]) + (p[10] + p[11])) + ((p[12] + p[13]) + (p[14] + p[15]))));
    }
    pa = pack8f(p);
    pb = pack8f(p + 8);
    if constexpr (!SAFE) {
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pa, lacc, 0, 0, 0);
      lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pb, lacc, 0, 0, 0);
    }
  };
  auto softmax = [&](auto safec, f32x16& acc, int key0, bool first_blk, bf16x8& pa, bf16x8& pb) {
    softmax_m(safec, IC<1>{}, acc, key0, first_blk, pa, pb);
  };

  // Software pipeline over 64-key tiles (halves a, b).  Fragments are read one phase before their
  // MFMAs; sched_barriers pin the reads where they are issued (left alone, the scheduler sinks each
  // read next to its MFMA behind an lgkmcnt(0)):
  //   QK(a) [V(a) reads] | K(b) reads, softmax(a) | PV(a) | QK(b) [V(b) reads] | softmax(b) |
  //   vmcnt(0) + barrier: tile kt+1 landed, every wave's reads of this tile retired |
  //   DMA tile kt+2 into this buffer, K(a) reads of tile kt+1 | PV(b) (registers only)
  const int nkt = (N + 63) / 64;
  const bool active = q0w < N;  // wave-uniform: a wave whose queries are all past N only stages K/V
  unsigned long long t_vm = 0, t_bar = 0;
  const unsigned long long t_begin = VS_CLK();
  auto pass = [&](auto safec) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      oacc[0][r] = 0.f;
      oacc[1][r] = 0.f;
      zero16[r] = 0.f;
    }
    lacc = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run = 0.f;
    l_half = 0.f;
    load_tile(0, smem0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (nkt > 1) load_tile(1, smem1);
    KFrag ka = kread(smem0, 0);
    auto iter = [&](int kt, auto bufc) {
      constexpr int BUF = decltype(bufc)::value;
      using MaskC = IC<1>;
      const bool has_next = kt + 1 < nkt;
      char* cur = BUF ? smem1 : smem0;
      const char* nxt = BUF ? smem0 : smem1;
      bf16x8 b0, b1;
      if (active) {
        f32x16 sa = mfma32p(ka.k[0], qf[0], zero16);
        __builtin_amdgcn_sched_barrier(0);
        const VFrag va = vread(cur, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 1; s < 4; ++s) sa = mfma32p(ka.k[s], qf[s], sa);
        const KFrag kb = kread(cur, 1);
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 a0, a1;
        softmax_m(safec, MaskC{}, sa, kt * 64, kt == 0, a0, a1);
        f32x16 sb;
        VFrag vb;
        if constexpr (ORD == 1) {
          sb = mfma32p(kb.k[0], qf[0], zero16);
#pragma unroll
          for (int s = 1; s < 4; ++s) sb = mfma32p(kb.k[s], qf[s], sb);
          __builtin_amdgcn_sched_barrier(0);
          vb = vread(cur, 1);
          __builtin_amdgcn_sched_barrier(0);
          pv(va, a0, a1);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          pv(va, a0, a1);
          sb = mfma32p(kb.k[0], qf[0], zero16);
          __builtin_amdgcn_sched_barrier(0);
          vb = vread(cur, 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 1; s < 4; ++s) sb = mfma32p(kb.k[s], qf[s], sb);
        }
        softmax_m(safec, MaskC{}, sb, kt * 64 + 32, false, b0, b1);
        __builtin_amdgcn_sched_barrier(0);
        if (has_next) {
#ifdef VS_STAMP
          const unsigned long long c0 = VS_CLK();
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const unsigned long long c1 = VS_CLK();
          __syncthreads();
          t_vm += c1 - c0;
          t_bar += VS_CLK() - c1;
#else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces of tile kt+1 landed
          __syncthreads();                                  // ... every wave's; all reads of `cur` retired
#endif
          if (kt + 2 < nkt && !(VS_ATTN_DIAG & 1)) load_tile(kt + 2, cur);
          ka = kread(nxt, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        pv(vb, b0, b1);
      } else if (has_next) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + 2 < nkt && !(VS_ATTN_DIAG & 1)) load_tile(kt + 2, cur);
      }
    };
    if constexpr (ORD != 2) {
      for (int kt = 0; kt < nkt; kt += 2) {
        iter(kt, IC<0>{});
        if (kt + 1 < nkt) iter(kt + 1, IC<1>{});
      }
    } else {
      // ORD 2: S(a), V(a) and K(b) of tile kt are in registers when iteration kt starts
      f32x16 sa_c;
      VFrag va_c;
      KFrag kb_c;
      if (active) {
        sa_c = mfma32p(ka.k[0], qf[0], zero16);
#pragma unroll
        for (int s = 1; s < 4; ++s) sa_c = mfma32p(ka.k[s], qf[s], sa_c);
        __builtin_amdgcn_sched_barrier(0);
        va_c = vread(smem0, 0);
        kb_c = kread(smem0, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      // LAST: the final tile (its blocks may hold keys past N: masked softmax; no next tile)
      auto iter2 = [&](int kt, auto bufc, auto lastc) {
        constexpr int BUF = decltype(bufc)::value;
        constexpr bool LAST = decltype(lastc)::value;
        char* cur = BUF ? smem1 : smem0;
        const char* nxt = BUF ? smem0 : smem1;
        if (active) {
          // [QK(b) | softmax(a)]
          f32x16 sb = mfma32p(kb_c.k[0], qf[0], zero16);
#pragma unroll
          for (int s = 1; s < 4; ++s) sb = mfma32p(kb_c.k[s], qf[s], sb);
          bf16x8 a0, a1;
          softmax_m(safec, lastc, sa_c, kt * 64, kt == 0, a0, a1);
          __builtin_amdgcn_sched_barrier(0);
          // [PV(a) | V(b) reads]
          const VFrag vb = vread(cur, 1);
          pv(va_c, a0, a1);
          __builtin_amdgcn_sched_barrier(0);
          bf16x8 b0, b1;
          if constexpr (!LAST) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces of tile kt+1 landed
            __syncthreads();                                  // ... every wave's; all reads of `cur` retired
            if (kt + 2 < nkt && !(VS_ATTN_DIAG & 1)) load_tile(kt + 2, cur);
            // [QK(a') | softmax(b)]
            const KFrag ka2 = kread(nxt, 0);
            sa_c = mfma32p(ka2.k[0], qf[0], zero16);
#pragma unroll
            for (int s = 1; s < 4; ++s) sa_c = mfma32p(ka2.k[s], qf[s], sa_c);
            softmax_m(safec, IC<0>{}, sb, kt * 64 + 32, false, b0, b1);
            __builtin_amdgcn_sched_barrier(0);
            // [PV(b) | V(a'), K(b') reads]
            va_c = vread(nxt, 0);
            kb_c = kread(nxt, 1);
            pv(vb, b0, b1);
            __builtin_amdgcn_sched_barrier(0);
          } else {
            softmax_m(safec, IC<1>{}, sb, kt * 64 + 32, false, b0, b1);
            pv(vb, b0, b1);
          }
        } else if (!LAST) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (kt + 2 < nkt && !(VS_ATTN_DIAG & 1)) load_tile(kt + 2, cur);
        }
      };
      int kt = 0;
      for (; kt + 2 < nkt; kt += 2) {
        iter2(kt, IC<0>{}, IC<0>{});
        iter2(kt + 1, IC<1>{}, IC<0>{});
      }
      if (kt + 1 < nkt) {
        iter2(kt, IC<0>{}, IC<0>{});
        iter2(kt + 1, IC<1>{}, IC<1>{});
      } else {
        iter2(kt, IC<0>{}, IC<1>{});
      }
    }
  };

  pass(IC<0>{});
  // Row sum of this lane's query (lane & 31): row (q >> 4) of lacc in lane (q & 15).
  float l;
  {
    const int q = lane & 31, src = (q & 15) << 2;
    // asm: hipcc folds "q < 16 ? bpermute(x0) : bpermute(x1)" into bpermute(q < 16 ? x0 : x1),
    // evaluating the select in the SOURCE lane (always x0 there) — wrong for queries 16..31.
    float l0, l1;
    asm volatile(
        "ds_bpermute_b32 %0, %2, %3\n\t"
        "ds_bpermute_b32 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(l0), "=&v"(l1)
        : "v"(src), "v"(lacc[0]), "v"(lacc[1])
        : "memory");
    l = q < 16 ? l0 : l1;
  }
  // Fast-pass validity: the row sum of every real query within [2^-100, 2^96] (false for NaN/inf) and
  // its O accumulators finite.  p = exp2(s) is a normal bf16 / f32 number from 2^-126 to 2^127, so
  // the band only guards the sums: l <= 2^96 keeps every p and the O sums (<= l * max|v|) finite for
  // |v| < 2^31, and l >= 2^-100 keeps the largest p normal.  (Round 4's [2^-60, 2^60] re-ran every
  // workgroup with a score above ~41 natural-log units: 1.9-2.2x the forward's time, which
  // pretrained attention sinks reach; profiles/r05_attn_logit_scale.txt.)
  bool ofin = true;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) ofin = ofin && __builtin_isfinite(oacc[dt][r]);
  const bool bad = active && qi < N && !(l >= 0x1p-100f && l <= 0x1p96f && ofin);
  __syncthreads();  // every wave is done with the last K/V tile; redo_flag = 0 is visible
  if (__any(bad) && lane == 0) redo_flag = 1;
  __syncthreads();
  if (redo_flag) {  // workgroup-uniform: the whole workgroup streams K/V again, safe softmax
    if (tid == 0) atomicAdd(&g_attn_redo, 1ull);
    pass(IC<1>{});
    l = pair_sum(l_half);
    __syncthreads();
  }

  // Epilogue: O^T accumulators -> normalised bf16 rows staged through LDS (wave-private 4 KB,
  // XOR-swizzled 16-B chunks), then written as whole 128-B rows (8 lanes per row).
  const float inv = 1.f / l;
  char* so = (wid < 2 ? smem0 : smem1) + (wid & 1) * 4096;
  const int oq = lane & 31;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int chunk = dt * 4 + g;  // 8 dims per 16-B chunk; this lane holds its 4hh half
      *(uint2*)(so + oq * 128 + ((chunk ^ (oq & 7)) << 4) + 8 * hh) =
          pack4(oacc[dt][4 * g] * inv, oacc[dt][4 * g + 1] * inv, oacc[dt][4 * g + 2] * inv,
                oacc[dt][4 * g + 3] * inv);
    }
  if (hh == 0 && qi < N) lse[((int64_t)b * H + h) * N + qi] = (m_run + __log2f(l)) * kLn2;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed (wave-private)
#pragma unroll
  for (int pss = 0; pss < 4; ++pss) {
    const int r = pss * 8 + (lane >> 3), ch = lane & 7;
    const uint4 v = *(const uint4*)(so + r * 128 + ((ch ^ (r & 7)) << 4));
    if (q0w + r < N) *(uint4*)(o + (row0 + q0w + r) * ldo + h * 64 + ch * 8) = v;
  }
  VS_STAMP_AT(true);
#ifdef VS_STAMP
  stamp_acc(4, t_vm);
  stamp_acc(5, t_bar);
  stamp_acc(6, VS_CLK() - t_begin);
#else
  (void)t_vm;
  (void)t_bar;
  (void)t_begin;
#endif
}

// ------------------------------------------------------------------ forward on 16x16x32 MFMAs
// The same wave tile as attn_fwd_bf16_kernel (32 queries x 64 dims of O, 64-key K/V tiles by LDS-DMA,
// fast pass with the safe-pass redo) on v_mfma_f32_16x16x32_bf16 (VS_KNOB_ATTN_VARIANT 8, round 6):
// same MFMA cycles per FLOP in twice the instructions; MI355X_MICROARCH.md "DVFS give-back" item 7
// measures this shape holding a higher clock on random data.  Lane l = (c, g) = (l & 15, l >> 4):
//   S^T tile (ks, qt) = K[16 keys] (cQ)^T[16 queries]: A = K rows (key c, dims 8g..8g+7, ds_read_b128),
//     B = this lane's Q fragment (query qt*16 + c); the lane holds query qt*16+c, keys 16ks + 4g + i;
//   P (qt) = {p(ks 0)[0..3], p(ks 1)[0..3]} is the B operand of O^T += V^T P^T with k-slot 8g + j <->
//     key 4g + j (j < 4) or 16 + 4g + j - 4; the V^T A operand (dim c, those keys) is two
//     ds_read_tr16_b64 of rows 4g..4g+3 and 16+4g..: a 16-lane group reads 4 rows x 16 dims;
//   row sums: A = all ones, so every lane's 4 accumulators hold its query's sum (no broadcast);
//   V image swizzle: 16-B chunk ^ 2((row >> 1) & 3): the 16 rows x 32 B of one tr read cover the 64
//     banks twice (the K image keeps swz_row: 16 rows x 16 B per group, conflict-free).
// A lane holds two queries (qt = 0, 1): the safe pass keeps two running references and reduces a
// query's max / sum over its four lanes (xor 16, xor 32).
__device__ __forceinline__ int swz_v16(int r) { return ((r >> 1) & 3) << 1; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256, 3) void attn_fwd16_bf16_kernel(const bf16_t* __restrict__ qkv, int64_t ldq,
                                                                bf16_t* __restrict__ o, int64_t ldo,
                                                                float* __restrict__ lse, int N, int H,
                                                                float scale_log2) {
  constexpr int TILE = 64 * 128;
  __shared__ __attribute__((aligned(16))) char smem0[2 * TILE];
  __shared__ __attribute__((aligned(16))) char smem1[2 * TILE];
  __shared__ int redo_flag;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb128 = (N + 127) / 128, blk = xcd_remap(blockIdx.x, gridDim.x), qb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const int q0w = qb * 128 + wid * 32;
  if (tid == 0) redo_flag = 0;

  bf16x8 qf[2][2];  // [query tile][32-dim chunk]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0w + qt * 16 + c, qr = qi < N ? qi : N - 1;
#pragma unroll
    for (int dc = 0; dc < 2; ++dc) {
      const bf16x8 q = *(const bf16x8*)(Qp + (int64_t)qr * ldq + dc * 32 + 8 * g);
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)q[j] * scale_log2;
      qf[qt][dc] = __builtin_convertvector(v, bf16x8);
    }
  }
  const bf16x8 ones = __builtin_convertvector((f32x8){1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f}, bf16x8);
  f32x4 oacc[4][2], lacc[2];
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  float m_run[2], l_half[2];

  int kbase[2], vbase[4];
#pragma unroll
  for (int dc = 0; dc < 2; ++dc) kbase[dc] = c * 128 + (((dc * 4 + g) ^ swz_row(c)) << 4);
  {
    const int r = 4 * g + (c >> 2), sw = swz_v16(r);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vbase[dt] = TILE + r * 128 + (((dt * 2 + ((c & 3) >> 1)) ^ sw) << 4) + (c & 1) * 8;
  }
  const int prow0 = wid * 16 + (lane >> 3), ppos = lane & 7;
  const uint32_t gk0 = (uint32_t)(prow0 * 2 * ldq + ((ppos ^ swz_row(prow0)) << 4));
  const uint32_t gk1 = (uint32_t)((prow0 + 8) * 2 * ldq + ((ppos ^ swz_row(prow0 + 8)) << 4));
  const uint32_t gv0 = (uint32_t)(prow0 * 2 * ldq + ((ppos ^ swz_v16(prow0)) << 4));
  const uint32_t gv1 = (uint32_t)((prow0 + 8) * 2 * ldq + ((ppos ^ swz_v16(prow0 + 8)) << 4));
  const int64_t tile_bytes = 64 * 2 * ldq, vdelta = 2 * (int64_t)D;
  auto load_tile = [&](int kt, char* buf) {
    const char* kb = (const char*)Kp + kt * tile_bytes;
    const char* vb = kb + vdelta;
    char* dk = buf + wid * 2048;
    char* dv = buf + TILE + wid * 2048;
    if ((kt + 1) * 64 <= N) {
      glds16_asm_so(kb, gk0, dk);
      glds16_asm_so(kb, gk1, dk + 1024);
      glds16_asm_so(vb, gv0, dv);
      glds16_asm_so(vb, gv1, dv + 1024);
    } else {
      const int r0 = kt * 64 + prow0, r1 = r0 + 8;
      const uint32_t c0 = (uint32_t)((r0 < N ? r0 : N - 1) - kt * 64) * (uint32_t)(2 * ldq);
      const uint32_t c1 = (uint32_t)((r1 < N ? r1 : N - 1) - kt * 64) * (uint32_t)(2 * ldq);
      glds16_asm_so(kb, c0 + ((ppos ^ swz_row(prow0)) << 4), dk);
      glds16_asm_so(kb, c1 + ((ppos ^ swz_row(prow0 + 8)) << 4), dk + 1024);
      glds16_asm_so(vb, c0 + ((ppos ^ swz_v16(prow0)) << 4), dv);
      glds16_asm_so(vb, c1 + ((ppos ^ swz_v16(prow0 + 8)) << 4), dv + 1024);
    }
  };
  struct KFrag {
    bf16x8 k[2][2];  // [16-key subtile][32-dim chunk]
  };
  struct VFrag {
    bf16x8 v[4];  // [16-dim tile]
  };
  struct SAcc {
    f32x4 s[2][2];  // [16-key subtile][query tile]
  };
  auto kread = [&](const char* base, int kb) {
    KFrag f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dc = 0; dc < 2; ++dc) f.k[ks][dc] = *(const bf16x8*)(base + kb * 4096 + ks * 2048 + kbase[dc]);
    return f;
  };
  auto vread = [&](const char* base, int kb) {
    VFrag f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) f.v[dt] = tr_pair(base + kb * 4096, vbase[dt], vbase[dt] + 2048);
    return f;
  };
  auto qk_first = [&](const KFrag& f, SAcc& a) { a.s[0][0] = mfma16(f.k[0][0], qf[0][0], zero4); };
  auto qk_rest = [&](const KFrag& f, SAcc& a) {
    a.s[0][1] = mfma16(f.k[0][0], qf[1][0], zero4);
    a.s[1][0] = mfma16(f.k[1][0], qf[0][0], zero4);
    a.s[1][1] = mfma16(f.k[1][0], qf[1][0], zero4);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) a.s[ks][qt] = mfma16(f.k[ks][1], qf[qt][1], a.s[ks][qt]);
  };
  auto pv = [&](const VFrag& f, const bf16x8 (&p)[2]) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = mfma16(f.v[dt], p[qt], oacc[dt][qt]);
  };
  auto qmax4 = [&](float v) {  // max over the query's four lanes (c, g = 0..3)
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
  };
  auto softmax = [&](auto safec, SAcc& a, int key0, bool first_blk, bf16x8 (&p)[2]) {
    constexpr bool SAFE = decltype(safec)::value;
    if (key0 + 32 > N) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (key0 + 16 * ks + 4 * g + i >= N) a.s[ks][qt][i] = -INFINITY;
    }
    float e[2][2][4];
    if constexpr (!SAFE) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int i = 0; i < 4; ++i) e[ks][qt][i] = __builtin_amdgcn_exp2f(a.s[ks][qt][i]);
    } else {
      float mx[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
        mx[qt] = max3f(max3f(a.s[0][qt][0], a.s[0][qt][1], a.s[0][qt][2]),
                       max3f(a.s[0][qt][3], a.s[1][qt][0], a.s[1][qt][1]), max3f(a.s[1][qt][2], a.s[1][qt][3], -INFINITY));
      if (__any(first_blk || mx[0] > m_run[0] + kRefBand || mx[1] > m_run[1] + kRefBand)) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const float mq = qmax4(mx[qt]);
          const bool move = first_blk || mq > m_run[qt] + kRefBand;
          const float m_new = move ? mq : m_run[qt];
          const float alpha = first_blk ? 1.f : __builtin_amdgcn_exp2f(m_run[qt] - m_new);
          m_run[qt] = m_new;
          l_half[qt] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) oacc[dt][qt][i] *= alpha;
        }
      }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        float sum = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            e[ks][qt][i] = __builtin_amdgcn_exp2f(a.s[ks][qt][i] - m_run[qt]);
            sum += e[ks][qt][i];
          }
        l_half[qt] += sum;
      }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const f32x8 v = {e[0][qt][0], e[0][qt][1], e[0][qt][2], e[0][qt][3],
                       e[1][qt][0], e[1][qt][1], e[1][qt][2], e[1][qt][3]};
      p[qt] = __builtin_convertvector(v, bf16x8);
    }
    if constexpr (!SAFE) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) lacc[qt] = mfma16(ones, p[qt], lacc[qt]);
    }
  };

  // the tile order of attn_fwd_bf16_kernel<1>: QK(a) [V(a) reads] | K(b) reads, softmax(a) |
  // QK(b) | V(b) reads | PV(a) | softmax(b) | vmcnt(0) + barrier, DMA tile kt+2, K(a') reads | PV(b)
  const int nkt = (N + 63) / 64;
  const bool active = q0w < N;
  auto pass = [&](auto safec) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = zero4;
    lacc[0] = zero4;
    lacc[1] = zero4;
    m_run[0] = m_run[1] = 0.f;
    l_half[0] = l_half[1] = 0.f;
    load_tile(0, smem0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (nkt > 1) load_tile(1, smem1);
    KFrag ka = kread(smem0, 0);
    auto iter = [&](int kt, auto bufc) {
      constexpr int BUF = decltype(bufc)::value;
      const bool has_next = kt + 1 < nkt;
      char* cur = BUF ? smem1 : smem0;
      const char* nxt = BUF ? smem0 : smem1;
      if (active) {
        SAcc sa, sb;
        qk_first(ka, sa);
        __builtin_amdgcn_sched_barrier(0);
        const VFrag va = vread(cur, 0);
        __builtin_amdgcn_sched_barrier(0);
        qk_rest(ka, sa);
        const KFrag kb = kread(cur, 1);
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 pa[2], pb[2];
        softmax(safec, sa, kt * 64, kt == 0, pa);
        qk_first(kb, sb);
        qk_rest(kb, sb);
        __builtin_amdgcn_sched_barrier(0);
        const VFrag vb = vread(cur, 1);
        __builtin_amdgcn_sched_barrier(0);
        pv(va, pa);
        __builtin_amdgcn_sched_barrier(0);
        softmax(safec, sb, kt * 64 + 32, false, pb);
        __builtin_amdgcn_sched_barrier(0);
        if (has_next) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (kt + 2 < nkt) load_tile(kt + 2, cur);
          ka = kread(nxt, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        pv(vb, pb);
      } else if (has_next) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + 2 < nkt) load_tile(kt + 2, cur);
      }
    };
    for (int kt = 0; kt < nkt; kt += 2) {
      iter(kt, IC<0>{});
      if (kt + 1 < nkt) iter(kt + 1, IC<1>{});
    }
  };

  pass(IC<0>{});
  float l[2] = {lacc[0][0], lacc[1][0]};  // every accumulator row holds the query's sum
  bool ofin = true;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int i = 0; i < 4; ++i) ofin = ofin && __builtin_isfinite(oacc[dt][qt][i]);
  bool bad = false;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
    bad = bad || (q0w + qt * 16 + c < N && !(l[qt] >= 0x1p-100f && l[qt] <= 0x1p96f && ofin));
  bad = active && bad;
  __syncthreads();
  if (__any(bad) && lane == 0) redo_flag = 1;
  __syncthreads();
  if (redo_flag) {
    if (tid == 0) atomicAdd(&g_attn_redo, 1ull);
    pass(IC<1>{});
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float v = l_half[qt];
      v += __shfl_xor(v, 16);
      l[qt] = v + __shfl_xor(v, 32);
    }
    __syncthreads();
  }

  // epilogue: lane (c, g) holds query qt*16 + c, dims 16dt + 4g .. +3 -> wave-private LDS rows
  char* so = (wid < 2 ? smem0 : smem1) + (wid & 1) * 4096;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float inv = 1.f / l[qt];
    const int qr = qt * 16 + c;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int chunk = dt * 2 + (g >> 1);
      *(uint2*)(so + qr * 128 + ((chunk ^ (qr & 7)) << 4) + (g & 1) * 8) =
          pack4(oacc[dt][qt][0] * inv, oacc[dt][qt][1] * inv, oacc[dt][qt][2] * inv, oacc[dt][qt][3] * inv);
    }
    if (g == 0 && q0w + qr < N) lse[((int64_t)b * H + h) * N + q0w + qr] = (m_run[qt] + __log2f(l[qt])) * kLn2;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
  for (int pss = 0; pss < 4; ++pss) {
    const int r = pss * 8 + (lane >> 3), ch = lane & 7;
    const uint4 v = *(const uint4*)(so + r * 128 + ((ch ^ (r & 7)) << 4));
    if (q0w + r < N) *(uint4*)(o + (row0 + q0w + r) * ldo + h * 64 + ch * 8) = v;
  }
}

// ------------------------------------------------------------------ backward: row constants
// Per (batch, head, query): nlse2 = -LSE * log2(e) and ndel = -delta (delta = rowsum(dO * O)),
// stored [B*H][Npad] with Npad = N rounded up to 64 and the padding set to (-inf, 0): the dK/dV
// kernel DMAs 64-query slices of them straight into LDS and seeds its S / dP accumulators with
// them, and a padded query then contributes exactly P = 0, dS = 0.  Four lanes per (row, head),
// two 16-B loads of O and of dO each, then a 2-step shuffle (one thread per (row, head) with 16
// loads in its chain was latency-bound: 14 us for 19 MB).
__global__ __launch_bounds__(256) void attn_rowprep_kernel(const bf16_t* __restrict__ o, int64_t ldo,
                                                           const bf16_t* __restrict__ dout, int64_t lddo,
                                                           const float* __restrict__ lse, float* __restrict__ nlse2,
                                                           float* __restrict__ ndel, int64_t B, int N, int H,
                                                           int Npad) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * 256;
  const int64_t pair = t >> 2;          // (row, head)
  const int q = (int)(t & 3);           // 16-column quarter of the head
  float acc = 0.f;
  const bool live = pair < B * N * H;
  int64_t row = 0;
  int h = 0;
  if (live) {
    row = pair / H;
    h = (int)(pair % H);
    const bf16x8* op = (const bf16x8*)(o + row * ldo + h * 64 + q * 16);
    const bf16x8* dp = (const bf16x8*)(dout + row * lddo + h * 64 + q * 16);
    const bf16x8 a0 = op[0], a1 = op[1], g0 = dp[0], g1 = dp[1];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = fmaf((float)a0[k], (float)g0[k], acc);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc = fmaf((float)a1[k], (float)g1[k], acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  if (live && q == 0) {
    const int64_t b = row / N, n = row % N;
    const int64_t w = (b * H + h) * Npad + n;
    ndel[w] = -acc;
    nlse2[w] = -lse[(b * H + h) * N + n] * kLog2e;
  }
  const int pad = Npad - N;
  for (int64_t i = t; i < B * H * pad; i += nthreads) {
    const int64_t w = (i / pad) * Npad + N + i % pad;
    nlse2[w] = -INFINITY;
    ndel[w] = 0.f;
  }
}

// ------------------------------------------------------------------ backward: dK, dV
// Key-major.  Workgroup = 4 waves x 32 keys; each wave holds its keys' K (pre-scaled by
// c = scale * log2 e, one bf16 rounding as the forward's Q) and V as MFMA B operands and dK^T,
// dV^T in accumulators while the workgroup sweeps 64-query slices: Q, dO, nlse2 and ndel arrive
// by LDS-DMA into a double-buffered stage, one barrier per slice.  S and dP are produced with the
// key on the lane and the query on the accumulator row; their chains start from nlse2 / ndel
// (4 ds_read_b128 each), so p = exp2(acc) and dS = p * acc with no other VALU, and P, dS are
// directly the B operands of dV^T += dO^T P and dK^T += Q^T dS (A operands: ds_read_tr16_b64).
// The Q/dO images use swz_rt, an XOR swizzle that is conflict-free for BOTH the row reads
// (ds_read_b128) and the transposed reads (rows r..r+3 land in distinct bank quarters); the
// previous (r >> 1) & 7 swizzle put rows r and r+2 of every tr read on the same banks.
__device__ __forceinline__ int swz_rt(int r) {
  const int u = (r >> 1) & 7;
  return ((u & 1) << 2) | (u >> 1);
}
__device__ __forceinline__ int off_rtswz(int r, int c) { return r * 128 + (((c >> 3) ^ swz_rt(r)) << 4) + (c & 7) * 2; }

constexpr int kBwdQT = 64 * 128;           // one 64-row x 64-dh bf16 image
constexpr int kBwdStage = 2 * kBwdQT + 512;  // dK/dV stage: Q, dO, nlse2[64], ndel[64]; dQ stage: K, V

__device__ __forceinline__ void attn_bwd_dkdv_body(char* __restrict__ stg0, char* __restrict__ stg1, int blk,
                                                   const bf16_t* __restrict__ qkv, int64_t ldq,
                                                   const bf16_t* __restrict__ dout, int64_t lddo,
                                                   const float* __restrict__ nlse2, const float* __restrict__ ndel,
                                                   bf16_t* __restrict__ dqkv, int64_t ldd, int N, int H, int Npad,
                                                   float scale) {
  constexpr int QT = kBwdQT;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int nb128 = (N + 127) / 128, kb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const bf16_t* Vp = Qp + 2 * D;
  const bf16_t* Dp = dout + row0 * lddo + h * 64;
  const float* NL = nlse2 + ((int64_t)b * H + h) * Npad;
  const float* ND = ndel + ((int64_t)b * H + h) * Npad;
  const int ki = kb * 128 + wid * 32 + (lane & 31);
  const float c2 = scale * kLog2e;

  bf16x8 kf[4], vf[4];
  {
    const int kr = ki < N ? ki : N - 1;  // rows past N: finite data, their dK/dV are not stored
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 k = *(const bf16x8*)(Kp + (int64_t)kr * ldq + 16 * s + 8 * hh);
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)k[j] * c2;
      kf[s] = __builtin_convertvector(v, bf16x8);
      vf[s] = *(const bf16x8*)(Vp + (int64_t)kr * ldq + 16 * s + 8 * hh);
    }
  }
  f32x16 dkacc[2], dvacc[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dkacc[0][r] = 0.f;
    dkacc[1][r] = 0.f;
    dvacc[0][r] = 0.f;
    dvacc[1][r] = 0.f;
  }

  // LDS-DMA: wave w fills Q pieces 2w, 2w+1 and dO pieces 2w, 2w+1 (8 rows x 128 B each); lane L
  // loads the source chunk that belongs at position L & 7 of its row; waves 0 / 1 fill nlse2 / ndel.
  // per-lane DMA source offsets of rows prow / prow + 8 of a Q / dO slice, computed once (SGPR-base +
  // 32-bit-offset asm DMA: the per-slice 64-bit address arithmetic cost ~40 VALU per slice)
  const int prow = wid * 16 + (lane >> 3), ppos = lane & 7;
  const uint32_t cq0 = (uint32_t)((ppos ^ swz_rt(prow)) << 4), cq1 = (uint32_t)((ppos ^ swz_rt(prow + 8)) << 4);
  const uint32_t gq0 = (uint32_t)(prow * 2 * ldq) + cq0, gq1 = (uint32_t)((prow + 8) * 2 * ldq) + cq1;
  const uint32_t gd0 = (uint32_t)(prow * 2 * lddo) + cq0, gd1 = (uint32_t)((prow + 8) * 2 * lddo) + cq1;
  auto load_stage = [&](int it, char* dst) {
    const int q0 = it * 64;
    const char* qs = (const char*)(Qp + (int64_t)q0 * ldq);
    const char* ds = (const char*)(Dp + (int64_t)q0 * lddo);
    char* dq_ = dst + wid * 2048;
    char* dd_ = dst + QT + wid * 2048;
    if (q0 + 64 <= N) {
      glds16_asm_so(qs, gq0, dq_);
      glds16_asm_so(qs, gq1, dq_ + 1024);
      glds16_asm_so(ds, gd0, dd_);
      glds16_asm_so(ds, gd1, dd_ + 1024);
    } else {  // partial last slice: rows past N re-read row N-1 (their nlse2 = -inf zeroes them)
      const int r0 = q0 + prow < N ? prow : N - 1 - q0, r1 = q0 + prow + 8 < N ? prow + 8 : N - 1 - q0;
      glds16_asm_so(qs, (uint32_t)(r0 * 2 * ldq) + cq0, dq_);
      glds16_asm_so(qs, (uint32_t)(r1 * 2 * ldq) + cq1, dq_ + 1024);
      glds16_asm_so(ds, (uint32_t)(r0 * 2 * lddo) + cq0, dd_);
      glds16_asm_so(ds, (uint32_t)(r1 * 2 * lddo) + cq1, dd_ + 1024);
    }
    // every DMA of the stage in the asm form: a compiler-visible one in flight makes hipcc wait
    // vmcnt(0) before the next LDS read, draining the prefetch of slice it + 1 under slice it
    if (wid == 0) glds4_asm_so(NL + q0, 4 * lane, dst + 2 * QT);
    else if (wid == 1) glds4_asm_so(ND + q0, 4 * lane, dst + 2 * QT + 256);
  };

  // per-lane LDS offsets: row reads of query qrow (+32 per sub-slice), chunk 2s+hh; transposed
  // reads of rows qt and qt+8 (qt = 4hh + q4, +16 per s2, +32 per sub-slice: immediates)
  const int qrow = lane & 31;
  int roff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) roff[s] = qrow * 128 + (((2 * s + hh) ^ swz_rt(qrow)) << 4);
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = ((lane >> 4) & 1) * 16, qt = 4 * hh + q4;
  int toff[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    toff[dt][0] = off_rtswz(qt, dt * 32 + g16 + p4);
    toff[dt][1] = off_rtswz(qt + 8, dt * 32 + g16 + p4);
  }

  // Phased so that S and dP are never live together (fits 3 waves/SIMD): S -> P -> dV += dO^T P,
  // then dP -> dS = P * dP -> dK += Q^T dS.  sched_barriers keep the scheduler from merging the
  // phases back (it hoists the second chain's LDS reads and MFMAs otherwise: 212 VGPRs).
  auto slice = [&](const char* st, int sub) {
    const char* sQ = st;
    const char* sD = st + QT;
    const float* sL = (const float*)(st + 2 * QT) + sub * 32 + 4 * hh;
    const float* sE = (const float*)(st + 2 * QT + 256) + sub * 32 + 4 * hh;
    // dP first, then S: both accumulators live together (the 158-VGPR body has the room since the
    // DMA offsets were hoisted), so dS = P * dP takes P in f32 straight from the exp2 instead of
    // unpacking the bf16 P of the dV product (16 fewer VALU per 32 x 32 unit)
    f32x16 dpa, acc;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 e4 = *(const float4*)(sE + 8 * g);
      dpa[4 * g] = e4.x; dpa[4 * g + 1] = e4.y; dpa[4 * g + 2] = e4.z; dpa[4 * g + 3] = e4.w;
      const float4 l4 = *(const float4*)(sL + 8 * g);
      acc[4 * g] = l4.x; acc[4 * g + 1] = l4.y; acc[4 * g + 2] = l4.z; acc[4 * g + 3] = l4.w;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
      dpa = mfma32p(*(const bf16x8*)(sD + sub * 4096 + roff[s]), vf[s], dpa);
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = mfma32p(*(const bf16x8*)(sQ + sub * 4096 + roff[s]), kf[s], acc);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float p[8], ds[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        p[r] = __builtin_amdgcn_exp2f(acc[8 * s2 + r]);
        ds[r] = p[r] * dpa[8 * s2 + r];  // dS = P * (dP - delta)
      }
      const bf16x8 pb = pack8f(p), db = pack8f(ds);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int o0 = sub * 4096 + s2 * 2048 + toff[dt][0], o1 = sub * 4096 + s2 * 2048 + toff[dt][1];
        dvacc[dt] = mfma32p(tr_pair(sD, o0, o1), pb, dvacc[dt]);
      }
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int o0 = sub * 4096 + s2 * 2048 + toff[dt][0], o1 = sub * 4096 + s2 * 2048 + toff[dt][1];
        dkacc[dt] = mfma32p(tr_pair(sQ, o0, o1), db, dkacc[dt]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nit = (N + 63) / 64;
  load_stage(0, stg0);
  auto iter = [&](int it, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces of slice it landed
    __syncthreads();                                  // ... and every wave's; buffer BUF^1 is free
    if (it + 1 < nit && !((VS_ATTN_DIAG & 2) && it >= 1)) load_stage(it + 1, BUF ? stg0 : stg1);
    const char* st = BUF ? stg1 : stg0;
    slice(st, 0);
    __builtin_amdgcn_sched_barrier(0);  // keep the two slices' S/dP accumulators from overlapping
    if (it * 64 + 32 < N) slice(st, 1);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int it = 0; it < nit; it += 2) {
    iter(it, IC<0>{});
    if (it + 1 < nit) iter(it + 1, IC<1>{});
  }

  if (ki < N) {
    bf16_t* krow = dqkv + (row0 + ki) * ldd + D + h * 64;
    bf16_t* vrow = krow + D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        *(uint2*)(krow + d) = pack4(dkacc[dt][4 * g] * scale, dkacc[dt][4 * g + 1] * scale,
                                    dkacc[dt][4 * g + 2] * scale, dkacc[dt][4 * g + 3] * scale);
        *(uint2*)(vrow + d) = pack4(dvacc[dt][4 * g], dvacc[dt][4 * g + 1], dvacc[dt][4 * g + 2], dvacc[dt][4 * g + 3]);
      }
  }
}

// ------------------------------------------------------------------ backward: dQ
// Query-major, the forward's structure: workgroup = 4 waves x 32 queries, K/V tiles of 64 keys
// arrive by LDS-DMA into double-buffered images (swz_rt: conflict-free row AND transposed reads
// of K).  Q is pre-scaled by c = scale * log2 e exactly as in the forward (same bf16 rounding, so
// P is the forward's P).  S^T = K Q^T and dP^T = V dO^T put the QUERY on the lane; their chains
// start from per-lane splats of nlse2 and ndel, so p = exp2(acc) and dS^T = p * acc, which is
// directly the B operand of dQ^T += K^T dS^T (K^T via ds_read_tr16_b64).  No atomics.
__device__ __forceinline__ void attn_bwd_dq_body(char* __restrict__ kv0, char* __restrict__ kv1, int blk,
                                                 const bf16_t* __restrict__ qkv, int64_t ldq,
                                                 const bf16_t* __restrict__ dout, int64_t lddo,
                                                 const float* __restrict__ nlse2, const float* __restrict__ ndel,
                                                 bf16_t* __restrict__ dqkv, int64_t ldd, int N, int H, int Npad,
                                                 float scale) {
  constexpr int TILE = 64 * 128;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int nb128 = (N + 127) / 128, qb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const bf16_t* Dp = dout + row0 * lddo + h * 64;
  const int qi = qb * 128 + wid * 32 + (lane & 31);
  const float c2 = scale * kLog2e;

  bf16x8 qf[4], df[4];
  {
    const int qr = qi < N ? qi : N - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 q = *(const bf16x8*)(Qp + (int64_t)qr * ldq + 16 * s + 8 * hh);
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)q[j] * c2;
      qf[s] = __builtin_convertvector(v, bf16x8);
      df[s] = *(const bf16x8*)(Dp + (int64_t)qr * lddo + 16 * s + 8 * hh);
    }
  }
  f32x16 sinit, dinit, dqacc[2];
  {
    const int64_t w = ((int64_t)b * H + h) * Npad + qi;
    const float nl = qi < N ? nlse2[w] : -INFINITY;  // a padded query: p = 0
    const float nd = qi < N ? ndel[w] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sinit[r] = nl;
      dinit[r] = nd;
      dqacc[0][r] = 0.f;
      dqacc[1][r] = 0.f;
    }
  }

  // per-lane LDS offsets: row reads of key (lane & 31) (+32 rows per kb: immediate), transposed
  // reads of K rows kt and kt+8 (kt = 4hh + q4; +16 per s2, +32 per kb: immediates)
  int roff[4];
  {
    const int key = lane & 31;
#pragma unroll
    for (int s = 0; s < 4; ++s) roff[s] = key * 128 + (((2 * s + hh) ^ swz_rt(key)) << 4);
  }
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = ((lane >> 4) & 1) * 16, kt0 = 4 * hh + q4;
  int toff[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    toff[dt][0] = off_rtswz(kt0, dt * 32 + g16 + p4);
    toff[dt][1] = off_rtswz(kt0 + 8, dt * 32 + g16 + p4);
  }

  const int64_t tile_bytes = 64 * 2 * ldq, vdelta = 2 * (int64_t)D;
  // per-lane DMA source offsets of rows prow / prow + 8 of a K (or V: base + vdelta) tile, computed
  // once: the DMA is the SGPR-base + 32-bit-offset asm form (the per-tile 64-bit address arithmetic
  // and the rows-past-N selects cost ~45 VALU per tile); the partial last tile clamps separately
  const int prow = wid * 16 + (lane >> 3), ppos = lane & 7;
  const uint32_t ko0 = (uint32_t)(prow * 2 * ldq + ((ppos ^ swz_rt(prow)) << 4));
  const uint32_t ko1 = (uint32_t)((prow + 8) * 2 * ldq + ((ppos ^ swz_rt(prow + 8)) << 4));
  auto load_tile = [&](int kt, char* buf) {
    const char* kb_ = (const char*)Kp + kt * tile_bytes;
    char* dk = buf + wid * 2048;
    char* dv = buf + TILE + wid * 2048;
    if ((kt + 1) * 64 <= N) {
      glds16_asm_so(kb_, ko0, dk);
      glds16_asm_so(kb_, ko1, dk + 1024);
      glds16_asm_so(kb_ + vdelta, ko0, dv);
      glds16_asm_so(kb_ + vdelta, ko1, dv + 1024);
    } else {  // partial last tile: rows past N re-read row N-1 (masked below)
      const int r0 = kt * 64 + prow < N ? prow : N - 1 - kt * 64;
      const int r1 = kt * 64 + prow + 8 < N ? prow + 8 : N - 1 - kt * 64;
      const uint32_t c0 = (uint32_t)(r0 * 2 * ldq + ((ppos ^ swz_rt(prow)) << 4));
      const uint32_t c1 = (uint32_t)(r1 * 2 * ldq + ((ppos ^ swz_rt(prow + 8)) << 4));
      glds16_asm_so(kb_, c0, dk);
      glds16_asm_so(kb_, c1, dk + 1024);
      glds16_asm_so(kb_ + vdelta, c0, dv);
      glds16_asm_so(kb_ + vdelta, c1, dv + 1024);
    }
  };

  auto sub = [&](const char* sK, int kb, int key0) {
    const char* sV = sK + TILE;
    f32x16 sacc = sinit, dpacc = dinit;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 ka = *(const bf16x8*)(sK + kb * 4096 + roff[s]);
      const bf16x8 va = *(const bf16x8*)(sV + kb * 4096 + roff[s]);
      sacc = mfma32p(ka, qf[s], sacc);
      dpacc = mfma32p(va, df[s], dpacc);
    }
    if (key0 + 32 > N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key0 + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) sacc[r] = -INFINITY;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float ds[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) ds[r] = __builtin_amdgcn_exp2f(sacc[8 * s2 + r]) * dpacc[8 * s2 + r];
      const bf16x8 db = pack8f(ds);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int o = kb * 4096 + s2 * 2048;
        const bf16x8 ka = tr_pair(sK, o + toff[dt][0], o + toff[dt][1]);
        dqacc[dt] = mfma32p(ka, db, dqacc[dt]);
      }
    }
  };

  const int nkt = (N + 63) / 64;
  load_tile(0, kv0);
  auto iter = [&](int kt, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nkt && !((VS_ATTN_DIAG & 2) && kt >= 1)) load_tile(kt + 1, BUF ? kv0 : kv1);
    const char* cur = BUF ? kv1 : kv0;
    sub(cur, 0, kt * 64);
    if (kt * 64 + 32 < N) sub(cur, 1, kt * 64 + 32);
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    iter(kt, IC<0>{});
    if (kt + 1 < nkt) iter(kt + 1, IC<1>{});
  }
  if (qi < N) {
    bf16_t* qrow = dqkv + (row0 + qi) * ldd + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        *(uint2*)(qrow + d) = pack4(dqacc[dt][4 * g] * scale, dqacc[dt][4 * g + 1] * scale,
                                    dqacc[dt][4 * g + 2] * scale, dqacc[dt][4 * g + 3] * scale);
      }
  }
}

// ------------------------------------------------------------------ backward, software-pipelined pairs
// The 3-wave bodies above rely on the other waves of the SIMD to fill the gap between a chain's
// MFMAs and the VALU that consumes them (exp after S, dS after dP).  These bodies pipeline two
// independent 32-row units inside the wave instead (2 waves per SIMD: the register file of two
// units): the dK/dV body runs a 64-query slice as S(a), S(b) (interleaved chains) -> P(a) under
// S(b)'s MFMAs -> dV(a), dP(a) -> P(b) under them -> dV(b), dP(b) -> dS(a) under them -> dK(a) ->
// dS(b) under dK(a) -> dK(b); the dQ body runs a 64-key tile as S, dP of keys a and b (interleaved
// chains) -> dS(a) under b's MFMAs -> dQ(a) -> dS(b) under dQ(a) -> dQ(b).  P stays f32 between the
// dV and dK products (no bf16 unpack).  Same LDS images, DMA and numerics as the 3-wave bodies.
__device__ __forceinline__ void attn_bwd_dkdv_pp(char* __restrict__ stg0, char* __restrict__ stg1, int blk,
                                                 const bf16_t* __restrict__ qkv, int64_t ldq,
                                                 const bf16_t* __restrict__ dout, int64_t lddo,
                                                 const float* __restrict__ nlse2, const float* __restrict__ ndel,
                                                 bf16_t* __restrict__ dqkv, int64_t ldd, int N, int H, int Npad,
                                                 float scale) {
  constexpr int QT = kBwdQT;
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb128 = (N + 127) / 128, kb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const bf16_t* Vp = Qp + 2 * D;
  const bf16_t* Dp = dout + row0 * lddo + h * 64;
  const float* NL = nlse2 + ((int64_t)b * H + h) * Npad;
  const float* ND = ndel + ((int64_t)b * H + h) * Npad;
  const int ki = kb * 128 + wid * 32 + (lane & 31);
  const float c2 = scale * kLog2e;

  bf16x8 kf[4], vf[4];
  {
    const int kr = ki < N ? ki : N - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 k = *(const bf16x8*)(Kp + (int64_t)kr * ldq + 16 * s + 8 * hh);
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)k[j] * c2;
      kf[s] = __builtin_convertvector(v, bf16x8);
      vf[s] = *(const bf16x8*)(Vp + (int64_t)kr * ldq + 16 * s + 8 * hh);
    }
  }
  f32x16 dkacc[2], dvacc[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dkacc[0][r] = 0.f;
    dkacc[1][r] = 0.f;
    dvacc[0][r] = 0.f;
    dvacc[1][r] = 0.f;
  }
  auto load_stage = [&](int it, char* dst) {
    const int prow = wid * 16 + (lane >> 3), ppos = lane & 7;
    const uint32_t cq0 = (uint32_t)((ppos ^ swz_rt(prow)) << 4), cq1 = (uint32_t)((ppos ^ swz_rt(prow + 8)) << 4);
    const int q0 = it * 64;
    int r0 = prow, r1 = prow + 8;
    if (q0 + 64 > N) {
      r0 = q0 + r0 < N ? r0 : N - 1 - q0;
      r1 = q0 + r1 < N ? r1 : N - 1 - q0;
    }
    const char* qs = (const char*)(Qp + (int64_t)q0 * ldq);
    const char* ds = (const char*)(Dp + (int64_t)q0 * lddo);
    glds16_asm_so(qs, (uint32_t)r0 * (uint32_t)(2 * ldq) + cq0, dst + wid * 2048);
    glds16_asm_so(qs, (uint32_t)r1 * (uint32_t)(2 * ldq) + cq1, dst + wid * 2048 + 1024);
    glds16_asm_so(ds, (uint32_t)r0 * (uint32_t)(2 * lddo) + cq0, dst + QT + wid * 2048);
    glds16_asm_so(ds, (uint32_t)r1 * (uint32_t)(2 * lddo) + cq1, dst + QT + wid * 2048 + 1024);
    const float* src = (wid < 2 ? NL : ND) + q0 + (wid & 1) * 32;
    if (lane < 32) glds4_asm_so(src, (uint32_t)(lane & 31) * 4, dst + 2 * QT + (wid >> 1) * 256 + (wid & 1) * 128);
  };
  const int qrow = lane & 31;
  int roff[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) roff[s] = qrow * 128 + (((2 * s + hh) ^ swz_rt(qrow)) << 4);
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = ((lane >> 4) & 1) * 16, qt = 4 * hh + q4;
  int toff[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    toff[dt][0] = off_rtswz(qt, dt * 32 + g16 + p4);
    toff[dt][1] = off_rtswz(qt + 8, dt * 32 + g16 + p4);
  }
  auto rowc = [&](const float* base, int sub, f32x16& acc) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 l4 = *(const float4*)(base + sub * 32 + 4 * hh + 8 * g);
      acc[4 * g] = l4.x; acc[4 * g + 1] = l4.y; acc[4 * g + 2] = l4.z; acc[4 * g + 3] = l4.w;
    }
  };
  // one 64-query slice: sub-slices a (queries 0..31) and b (32..63).  A sub-slice past N runs on
  // padded rows (nlse2 = -inf: P = 0, dS = 0), so every slice is branch-free.  Each phase's LDS
  // operand reads are issued ahead of its MFMAs (pinned by sched_barriers; the compiler otherwise
  // sinks every read next to its MFMA behind an lgkmcnt(0)).
  auto rows4 = [&](const char* img, int sub, bf16x8 (&f)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) f[s] = *(const bf16x8*)(img + sub * 4096 + roff[s]);
  };
  auto tr4 = [&](const char* img, int sub, bf16x8 (&f)[4]) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int o = sub * 4096 + s2 * 2048;
        f[2 * s2 + dt] = tr_pair(img, o + toff[dt][0], o + toff[dt][1]);
      }
  };
  auto mma_p = [&](const bf16x8 (&f)[4], const float (&pv)[16], f32x16 (&acc)[2]) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = pack8f(pv + 8 * s2);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) acc[dt] = mfma32p(f[2 * s2 + dt], pb, acc[dt]);
    }
  };
  auto slice = [&](const char* st) {
    const char* sQ = st;
    const char* sD = st + QT;
    const float* sL = (const float*)(st + 2 * QT);
    const float* sE = (const float*)(st + 2 * QT + 256);
    f32x16 xa, xb;
    bf16x8 fa[4], fb[4];
    rowc(sL, 0, xa);
    rows4(sQ, 0, fa);
    rowc(sL, 1, xb);
    rows4(sQ, 1, fb);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // S(a), S(b): two independent chains, interleaved
      xa = mfma32p(fa[s], kf[s], xa);
      xb = mfma32p(fb[s], kf[s], xb);
    }
    __builtin_amdgcn_sched_barrier(0);
    tr4(sD, 0, fa);  // dO(a)^T for dV(a)
    rows4(sD, 0, fb);  // dO(a) rows for dP(a)
    __builtin_amdgcn_sched_barrier(0);
    float pa[16], pb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) pa[r] = __builtin_amdgcn_exp2f(xa[r]);
    rowc(sE, 0, xa);
    mma_p(fa, pa, dvacc);
#pragma unroll
    for (int s = 0; s < 4; ++s) xa = mfma32p(fb[s], vf[s], xa);
    __builtin_amdgcn_sched_barrier(0);
    tr4(sD, 1, fa);  // dO(b)^T
    rows4(sD, 1, fb);  // dO(b) rows
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 16; ++r) pb[r] = __builtin_amdgcn_exp2f(xb[r]);
    rowc(sE, 1, xb);
    mma_p(fa, pb, dvacc);
#pragma unroll
    for (int s = 0; s < 4; ++s) xb = mfma32p(fb[s], vf[s], xb);
    __builtin_amdgcn_sched_barrier(0);
    tr4(sQ, 0, fa);  // Q(a)^T, Q(b)^T for dK
    tr4(sQ, 1, fb);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 16; ++r) pa[r] *= xa[r];
    mma_p(fa, pa, dkacc);
#pragma unroll
    for (int r = 0; r < 16; ++r) pb[r] *= xb[r];
    mma_p(fb, pb, dkacc);
    __builtin_amdgcn_sched_barrier(0);
  };
  const int nit = (N + 63) / 64;
  load_stage(0, stg0);
  auto iter = [&](int it, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (it + 1 < nit) load_stage(it + 1, BUF ? stg0 : stg1);
    slice(BUF ? stg1 : stg0);
  };
  for (int it = 0; it < nit; it += 2) {
    iter(it, IC<0>{});
    if (it + 1 < nit) iter(it + 1, IC<1>{});
  }
  if (ki < N) {
    bf16_t* krow = dqkv + (row0 + ki) * ldd + D + h * 64;
    bf16_t* vrow = krow + D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        *(uint2*)(krow + d) = pack4(dkacc[dt][4 * g] * scale, dkacc[dt][4 * g + 1] * scale,
                                    dkacc[dt][4 * g + 2] * scale, dkacc[dt][4 * g + 3] * scale);
        *(uint2*)(vrow + d) = pack4(dvacc[dt][4 * g], dvacc[dt][4 * g + 1], dvacc[dt][4 * g + 2], dvacc[dt][4 * g + 3]);
      }
  }
}

__device__ __forceinline__ void attn_bwd_dq_pp(char* __restrict__ kv0, char* __restrict__ kv1, int blk,
                                               const bf16_t* __restrict__ qkv, int64_t ldq,
                                               const bf16_t* __restrict__ dout, int64_t lddo,
                                               const float* __restrict__ nlse2, const float* __restrict__ ndel,
                                               bf16_t* __restrict__ dqkv, int64_t ldd, int N, int H, int Npad,
                                               float scale) {
  constexpr int TILE = 64 * 128;
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb128 = (N + 127) / 128, qb = blk % nb128;
  const int h = (blk / nb128) % H, b = blk / nb128 / H, D = H * 64;
  const int64_t row0 = (int64_t)b * N;
  const bf16_t* Qp = qkv + row0 * ldq + h * 64;
  const bf16_t* Kp = Qp + D;
  const bf16_t* Dp = dout + row0 * lddo + h * 64;
  const int qi = qb * 128 + wid * 32 + (lane & 31);
  const float c2 = scale * kLog2e;
  bf16x8 qf[4], df[4];
  {
    const int qr = qi < N ? qi : N - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 q = *(const bf16x8*)(Qp + (int64_t)qr * ldq + 16 * s + 8 * hh);
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)q[j] * c2;
      qf[s] = __builtin_convertvector(v, bf16x8);
      df[s] = *(const bf16x8*)(Dp + (int64_t)qr * lddo + 16 * s + 8 * hh);
    }
  }
  f32x16 sinit, dinit, dqacc[2];
  {
    const int64_t w = ((int64_t)b * H + h) * Npad + qi;
    const float nl = qi < N ? nlse2[w] : -INFINITY;  // a padded query: p = 0
    const float nd = qi < N ? ndel[w] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sinit[r] = nl;
      dinit[r] = nd;
      dqacc[0][r] = 0.f;
      dqacc[1][r] = 0.f;
    }
  }
  int roff[4];
  {
    const int key = lane & 31;
#pragma unroll
    for (int s = 0; s < 4; ++s) roff[s] = key * 128 + (((2 * s + hh) ^ swz_rt(key)) << 4);
  }
  const int q4 = (lane & 15) >> 2, p4 = (lane & 3) * 4, g16 = ((lane >> 4) & 1) * 16, kt0 = 4 * hh + q4;
  int toff[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    toff[dt][0] = off_rtswz(kt0, dt * 32 + g16 + p4);
    toff[dt][1] = off_rtswz(kt0 + 8, dt * 32 + g16 + p4);
  }
  const int64_t tile_bytes = 64 * 2 * ldq, vdelta = 2 * (int64_t)D;
  auto load_tile = [&](int kt, char* buf) {
    const int prow = wid * 16 + (lane >> 3), ppos = lane & 7;
    const uint32_t cc0 = (uint32_t)((ppos ^ swz_rt(prow)) << 4), cc1 = (uint32_t)((ppos ^ swz_rt(prow + 8)) << 4);
    const char* kb_ = (const char*)Kp + kt * tile_bytes;
    int r0 = prow, r1 = prow + 8;
    if ((kt + 1) * 64 > N) {
      r0 = kt * 64 + r0 < N ? r0 : N - 1 - kt * 64;
      r1 = kt * 64 + r1 < N ? r1 : N - 1 - kt * 64;
    }
    const uint32_t o0 = (uint32_t)r0 * (uint32_t)(2 * ldq) + cc0, o1 = (uint32_t)r1 * (uint32_t)(2 * ldq) + cc1;
    glds16_asm_so(kb_, o0, buf + wid * 2048);
    glds16_asm_so(kb_, o1, buf + wid * 2048 + 1024);
    glds16_asm_so(kb_ + vdelta, o0, buf + TILE + wid * 2048);
    glds16_asm_so(kb_ + vdelta, o1, buf + TILE + wid * 2048 + 1024);
  };
  auto mask = [&](f32x16& acc, int key0) {
    if (key0 + 32 > N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key0 + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) acc[r] = -INFINITY;
    }
  };
  auto ktr4 = [&](const char* sK, int kb, bf16x8 (&f)[4]) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int o = kb * 4096 + s2 * 2048;
        f[2 * s2 + dt] = tr_pair(sK, o + toff[dt][0], o + toff[dt][1]);
      }
  };
  auto dq_mma = [&](const bf16x8 (&f)[4], const f32x16& sacc, const f32x16& dpacc) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float ds[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) ds[r] = __builtin_amdgcn_exp2f(sacc[8 * s2 + r]) * dpacc[8 * s2 + r];
      const bf16x8 db = pack8f(ds);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) dqacc[dt] = mfma32p(f[2 * s2 + dt], db, dqacc[dt]);
    }
  };
  // one 64-key tile: key blocks a (0..31) and b (32..63; keys past N masked to p = 0, so every tile
  // is branch-free but the last one's mask).  Operand reads one phase ahead of their MFMAs.
  auto tile = [&](const char* sK, int key0) {
    const char* sV = sK + TILE;
    f32x16 sa, da, sb, db;
    bf16x8 ka[4], va[4], kb_[4], vb[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ka[s] = *(const bf16x8*)(sK + roff[s]);
      va[s] = *(const bf16x8*)(sV + roff[s]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kb_[s] = *(const bf16x8*)(sK + 4096 + roff[s]);
      vb[s] = *(const bf16x8*)(sV + 4096 + roff[s]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sa = mfma32p(ka[s], qf[s], s == 0 ? sinit : sa);
      da = mfma32p(va[s], df[s], s == 0 ? dinit : da);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sb = mfma32p(kb_[s], qf[s], s == 0 ? sinit : sb);
      db = mfma32p(vb[s], df[s], s == 0 ? dinit : db);
    }
    __builtin_amdgcn_sched_barrier(0);
    ktr4(sK, 0, ka);
    ktr4(sK, 1, kb_);
    __builtin_amdgcn_sched_barrier(0);
    if (key0 + 64 > N) {
      mask(sa, key0);
      mask(sb, key0 + 32);
    }
    dq_mma(ka, sa, da);
    dq_mma(kb_, sb, db);
    __builtin_amdgcn_sched_barrier(0);
  };
  const int nkt = (N + 63) / 64;
  load_tile(0, kv0);
  auto iter = [&](int kt, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nkt) load_tile(kt + 1, BUF ? kv0 : kv1);
    tile(BUF ? kv1 : kv0, kt * 64);
  };
  for (int kt = 0; kt < nkt; kt += 2) {
    iter(kt, IC<0>{});
    if (kt + 1 < nkt) iter(kt + 1, IC<1>{});
  }
  if (qi < N) {
    bf16_t* qrow = dqkv + (row0 + qi) * ldd + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        *(uint2*)(qrow + d) = pack4(dqacc[dt][4 * g] * scale, dqacc[dt][4 * g + 1] * scale,
                                    dqacc[dt][4 * g + 2] * scale, dqacc[dt][4 * g + 3] * scale);
      }
  }
}

// PKV / PQ: the pipelined pair (true) or the 3-wave (false) dK/dV / dQ body
template <int WPS, bool PKV, bool PQ>
__global__ __launch_bounds__(256, WPS) void attn_bwd_bf16_pp_kernel(const bf16_t* __restrict__ qkv, int64_t ldq,
                                                                    const bf16_t* __restrict__ dout, int64_t lddo,
                                                                    const float* __restrict__ nlse2,
                                                                    const float* __restrict__ ndel,
                                                                    bf16_t* __restrict__ dqkv, int64_t ldd, int N,
                                                                    int H, int Npad, float scale, int nblk, int skip) {
  __shared__ __attribute__((aligned(16))) char st0[kBwdStage];
  __shared__ __attribute__((aligned(16))) char st1[kBwdStage];
  const int id = blockIdx.x;
  if (skip & (id < nblk ? 1 : 2)) return;
  if (id < nblk) {
    if constexpr (PKV)
      attn_bwd_dkdv_pp(st0, st1, xcd_remap(id, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad, scale);
    else
      attn_bwd_dkdv_body(st0, st1, xcd_remap(id, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad, scale);
  } else {
    if constexpr (PQ)
      attn_bwd_dq_pp(st0, st1, xcd_remap(id - nblk, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad,
                     scale);
    else
      attn_bwd_dq_body(st0, st1, xcd_remap(id - nblk, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad,
                       scale);
  }
}

// ------------------------------------------------------------------ backward: one launch
// The dK/dV and dQ passes run as ONE grid: blocks [0, nblk) are dK/dV workgroups, [nblk, 2 nblk)
// dQ workgroups, sharing the same two LDS stages.  Each pass alone puts 2496 waves on 3072 wave
// slots (B = 16, N = 1568, H = 3), so a third of the SIMDs carry 3 waves and the rest 2 and the
// launch lasts as long as the 3-wave SIMDs; one grid of both lets the dispatcher backfill slots
// freed by the (longer, dispatched first) dK/dV workgroups with dQ workgroups.
__global__ __launch_bounds__(256, 3) void attn_bwd_bf16_kernel(const bf16_t* __restrict__ qkv, int64_t ldq,
                                                               const bf16_t* __restrict__ dout, int64_t lddo,
                                                               const float* __restrict__ nlse2,
                                                               const float* __restrict__ ndel,
                                                               bf16_t* __restrict__ dqkv, int64_t ldd, int N, int H,
                                                               int Npad, float scale, int nblk, int skip) {
  __shared__ __attribute__((aligned(16))) char st0[kBwdStage];  // two objects: see attn_fwd_bf16_kernel
  __shared__ __attribute__((aligned(16))) char st1[kBwdStage];
  const int id = blockIdx.x;
  if (skip & (id < nblk ? 1 : 2)) return;  // diagnostic builds only: one pass timed alone (VS_DEBUG_KNOBS)
  if (id < nblk)
    attn_bwd_dkdv_body(st0, st1, xcd_remap(id, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad, scale);
  else
    attn_bwd_dq_body(st0, st1, xcd_remap(id - nblk, nblk), qkv, ldq, dout, lddo, nlse2, ndel, dqkv, ldd, N, H, Npad,
                     scale);
}

}  // namespace vs

using namespace vs;

static int attn_check(int64_t B, int64_t N, int64_t H, int64_t Dh) {
  VS_REQUIRE(Dh == 64, "vs_attn: head dim must be 64");
  VS_REQUIRE(B > 0 && N > 0 && H > 0, "vs_attn: empty problem");
  VS_REQUIRE(B <= 65535 && H <= 65535 && N < (1 << 30), "vs_attn: extents out of range");
  return VS_OK;
}

extern "C" int vs_attn_fwd(int32_t dtype, int64_t B, int64_t N, int64_t H, int64_t Dh, const void* qkv, int64_t ld_qkv,
                           void* o, int64_t ld_o, float* lse, float scale, void* stream) {
  VS_CALL(attn_check(B, N, H, Dh));
  VS_REQUIRE(qkv && o && lse, "vs_attn_fwd: null pointer");
  VS_REQUIRE(ld_qkv >= 3 * H * 64 && ld_o >= H * 64, "vs_attn_fwd: leading dims too small");
  hipStream_t s = (hipStream_t)stream;
  const double es = dtype == VS_BF16 ? 2.0 : 4.0;
  ScopedTimer timer(VS_TIMER_ATTN_FWD, s, (double)(B * N * H * 64) * 4.0 * es + (double)(B * H * N) * 4.0);
  if (dtype == VS_BF16) {
    VS_REQUIRE(ld_qkv % 8 == 0 && ld_o % 4 == 0 && aligned16(qkv) && (((uintptr_t)o) & 7) == 0,
               "vs_attn_fwd: bf16 rows must be 16-byte aligned");
    count_path(VS_PATH_ATTN_FWD);
    // VS_KNOB_ATTN_VARIANT low nibble: 0 the default kernel (QK(b) issued ahead of PV(a): 299 -> 252 us
    // back to back at 128 clips, neutral inside the step); 6: the round-2 order (PV(a) before QK(b)),
    // the one experimental slot kept.  The one-wave-per-SIMD kernels of round 3 (slower: DESIGN.md
    // section 5) were removed.
    const int fv = knob(VS_KNOB_ATTN_VARIANT) & 15;
    dim3 grid((unsigned)(cdiv(N, 128) * H * B));  // 1D: xcd_remap groups a (b, h)'s blocks on one XCD
    // 7: the cross-tile software pipeline (ORD 2, round 6)
    // (round-6 A/B, profiles/r06_attn_ab_c2.json: 283.6 vs 260.7 us at C2, 1,100 vs 1,019 at C3 -- slower)
    // 8: the 16x16x32-MFMA forward (round 6)
    auto kern = fv == 6   ? attn_fwd_bf16_kernel<0>
                : fv == 7 ? attn_fwd_bf16_kernel<2>
                : fv == 8 ? attn_fwd16_bf16_kernel
                          : attn_fwd_bf16_kernel<1>;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, (const bf16_t*)qkv, ld_qkv, (bf16_t*)o, ld_o, lse, (int)N, (int)H,
                       scale * kLog2e);
  } else if (dtype == VS_F32) {
    dim3 grid((unsigned)cdiv(N, 64), (unsigned)H, (unsigned)B);
    count_path(VS_PATH_ATTN_F32);
    hipLaunchKernelGGL(attn_fwd_f32_kernel, grid, dim3(256), 0, s, (const float*)qkv, ld_qkv, (float*)o, ld_o, lse,
                       (int)N, (int)H, scale);
  } else {
    VS_REQUIRE(false, "vs_attn_fwd: bad dtype");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_attn_redo_count(int64_t* out, int32_t reset) {
  VS_REQUIRE(out, "vs_attn_redo_count: null pointer");
  unsigned long long v = 0;
  // synchronising (as the header says): forward launches on any stream (torch's side streams are
  // not ordered against the null-stream symbol copies) have finished their atomicAdd before the
  // read, and none is in flight when the counter is reset
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(vs::g_attn_redo), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return (int)e;
  *out = (int64_t)v;
  if (reset) {
    const unsigned long long z = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(vs::g_attn_redo), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    if (e != hipSuccess) return (int)e;
  }
  return VS_OK;
}

static inline int64_t attn_npad(int64_t N) { return (N + 63) / 64 * 64; }

extern "C" size_t vs_attn_bwd_workspace_bytes(int64_t B, int64_t N, int64_t H, int64_t Dh) {
  (void)Dh;
  // bf16: nlse2 and ndel [B*H][Npad] f32; f32: delta [B,H,N] (smaller); 256-B padded
  return ((size_t)(2 * B * H * attn_npad(N)) * 4 + 255) / 256 * 256;
}

extern "C" int vs_attn_bwd(int32_t dtype, int64_t B, int64_t N, int64_t H, int64_t Dh, const void* qkv, int64_t ld_qkv,
                           const void* o, int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, void* dqkv,
                           int64_t ld_dqkv, void* workspace, float scale, void* stream) {
  VS_CALL(attn_check(B, N, H, Dh));
  VS_REQUIRE(qkv && o && dout && lse && dqkv && workspace, "vs_attn_bwd: null pointer");
  VS_REQUIRE(ld_qkv >= 3 * H * 64 && ld_dqkv >= 3 * H * 64 && ld_o >= H * 64 && ld_do >= H * 64,
             "vs_attn_bwd: leading dims too small");
  hipStream_t s = (hipStream_t)stream;
  const double es = dtype == VS_BF16 ? 2.0 : 4.0;
  ScopedTimer timer(VS_TIMER_ATTN_BWD, s, (double)(B * N * H * 64) * 8.0 * es + (double)(B * H * N) * 4.0);
  float* delta = (float*)workspace;
  const int64_t rows = B * N;
  const unsigned dgrid = (unsigned)cdiv(rows * H, 4);
  if (dtype == VS_BF16) {
    VS_REQUIRE(ld_qkv % 8 == 0 && ld_dqkv % 4 == 0 && ld_do % 8 == 0 && aligned16(qkv) && aligned16(dout) &&
                   (((uintptr_t)dqkv) & 7) == 0,
               "vs_attn_bwd: bf16 rows must be 16-byte aligned");
    VS_REQUIRE(ld_o % 8 == 0 && aligned16(o) && aligned16(workspace), "vs_attn_bwd: o / workspace alignment");
    const int64_t npad = attn_npad(N);
    float* nlse2 = (float*)workspace;
    float* ndel = nlse2 + B * H * npad;
    count_path(VS_PATH_ATTN_BWD);
    hipLaunchKernelGGL(attn_rowprep_kernel, dim3((unsigned)cdiv(rows * H * 4, 256)), dim3(256), 0, s, (const bf16_t*)o,
                       ld_o, (const bf16_t*)dout, ld_do, lse, nlse2, ndel, B, (int)N, (int)H, (int)npad);
    // VS_KNOB_ATTN_VARIANT bits 4..7: 0 (default) picks 6 or 9 by grid size; 6 the software-pipelined
    // pair kernel (2 waves per SIMD), 9 the 3-wave kernel (3 waves per SIMD, one 32-row unit per wave)
    int bv = (knob(VS_KNOB_ATTN_VARIANT) >> 4) & 15;
    if (bv == 0) {
      // default by grid size: the pipelined pairs (2 waves/SIMD) when both passes fit in about two
      // rounds of the 3-wave kernel's slots (C2 at 16 clips: 624 + 624 workgroups, 122.3 -> 116.6 us),
      // the 3-wave kernel beyond (128 clips: 4,992 + 4,992 workgroups, 1,026 vs 924 us in
      // profiles/r03_v5_microbench_b128.txt)
      static const int slots = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return 3 * cus;
      }();
      bv = cdiv(N, 128) * H * B <= slots ? 6 : 9;
    }
#ifdef VS_DEBUG_KNOBS
    // diagnostic builds only (build.build(variant=..., defines=["VS_DEBUG_KNOBS"])): bits 8, 9 skip the
    // dK/dV or the dQ pass, so one pass can be timed alone -- the gradients are then WRONG
    const int skip = (knob(VS_KNOB_ATTN_VARIANT) >> 8) & 3;
#else
    const int skip = 0;
#endif
    const unsigned g = (unsigned)(cdiv(N, 128) * H * B);  // 1D: xcd_remap groups a (b, h)'s blocks on one XCD
    if (bv == 6) {
      hipLaunchKernelGGL((attn_bwd_bf16_pp_kernel<2, true, true>), dim3(2 * g), dim3(256), 0, s, (const bf16_t*)qkv,
                         ld_qkv, (const bf16_t*)dout, ld_do, nlse2, ndel, (bf16_t*)dqkv, ld_dqkv, (int)N, (int)H,
                         (int)npad, scale, (int)g, skip);
    } else {  // 9: the 3-wave kernel (round-2 default)
      hipLaunchKernelGGL(attn_bwd_bf16_kernel, dim3(2 * g), dim3(256), 0, s, (const bf16_t*)qkv, ld_qkv,
                         (const bf16_t*)dout, ld_do, nlse2, ndel, (bf16_t*)dqkv, ld_dqkv, (int)N, (int)H, (int)npad,
                         scale, (int)g, skip);
    }
  } else if (dtype == VS_F32) {
    count_path(VS_PATH_ATTN_F32);
    hipLaunchKernelGGL(attn_delta_kernel<float>, dim3(dgrid), dim3(256), 0, s, (const float*)o, ld_o,
                       (const float*)dout, ld_do, delta, rows, (int)N, (int)H);
    dim3 grid((unsigned)cdiv(N, 64), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL(attn_bwd_dkdv_f32_kernel, grid, dim3(256), 0, s, (const float*)qkv, ld_qkv, (const float*)dout,
                       ld_do, lse, delta, (float*)dqkv, ld_dqkv, (int)N, (int)H, scale);
    hipLaunchKernelGGL(attn_bwd_dq_f32_kernel, grid, dim3(256), 0, s, (const float*)qkv, ld_qkv, (const float*)dout,
                       ld_do, lse, delta, (float*)dqkv, ld_dqkv, (int)N, (int)H, scale);
  } else {
    VS_REQUIRE(false, "vs_attn_bwd: bad dtype");
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

#ifdef VS_STAMP
extern "C" int vs_dbg_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vs::g_stamp), (size_t)n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
