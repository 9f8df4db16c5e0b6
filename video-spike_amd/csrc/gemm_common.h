// gemm_common.h — the GEMM epilogue machinery shared by gemm.hip and fp8.hip: epilogue parameters,
// the per-element / 8-column epilogues (bias, position table, GELU and its gradient, residual, ...)
// and the XCD-aware tile map.
#pragma once

#include "common.h"

namespace vs {

struct EpiParams {
  int64_t M, N;
  void* c;
  int64_t ldc;
  int out_bf16;
  int op_bf16;
  uint32_t flags;
  float alpha;
  const float* bias;
  const float* residual;
  int64_t ldr;
  const float* pos;
  int64_t pos_rows;
  const void* aux_in;
  int64_t ld_aux_in;
  void* aux_out;
  int64_t ld_aux_out;
  int vec_ok;  // all leading dims / pointers allow 16-B vectors on 8-column groups
  float* a_rowsum;  // optional: += sum_k A(m, k) (fused bias gradient of dW = dY^T X)
  float* part;      // split-K partials [split][M][N] (ATOMIC with workspace), else null
};

// Row sums of the A fragments a wave consumed (lane holds row (lane & 15) of 16-row fragment i):
// reduce the 4 lane groups and add once per row.
template <int TM>
__device__ __forceinline__ void flush_rowsum(float* out, float (&rs)[TM], int64_t row_base, int64_t M, int lane) {
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float v = rs[i];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const int64_t m = row_base + i * 16 + lane;
    if (lane < 16 && m < M) unsafeAtomicAdd(out + m, v);
  }
}

struct GridMap {
  int tiles_n, tiles_m, splits;
  int64_t k_per_split;
};

__device__ __forceinline__ void map_block(const GridMap& g, int& nt, int& mt, int& split) {
  // bijective XCD-aware remap: blocks b, b+8, b+16 ... (one XCD under round-robin dispatch) get
  // consecutive tile indices
  const int nwg = g.tiles_n * g.tiles_m * g.splits;
  const int b = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
  const int tiles = g.tiles_n * g.tiles_m;
  split = t / tiles;
  const int rem = t % tiles;
  mt = rem / g.tiles_n;
  nt = rem % g.tiles_n;
}

__device__ __forceinline__ float ld_any(const void* p, int64_t i, int bf) {
  return bf ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
__device__ __forceinline__ void st_any(void* p, int64_t i, float v, int bf) {
  if (bf) ((bf16_t*)p)[i] = f2bf(v);
  else ((float*)p)[i] = v;
}

__device__ __forceinline__ void ld8(const void* p, int64_t i, int bf, float (&v)[8]) {
  if (bf) {
    const uint4 u = *(const uint4*)((const bf16_t*)p + i);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    const float4 a = *(const float4*)((const float*)p + i);
    const float4 b = *(const float4*)((const float*)p + i + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
__device__ __forceinline__ void st8(void* p, int64_t i, int bf, const float (&v)[8]) {
  if (bf) {
    uint4 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    u.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    u.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    *(uint4*)((bf16_t*)p + i) = u;
  } else {
    *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)((float*)p + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// Epilogue flags are a template parameter EF for the combinations the ViT block launches (dead
// branches vanish: the all-runtime epilogue of a 4-pass unrolled tile is ~9k instructions of
// mostly-unused GELU/erf/atomic code); kEpiRuntime reads e.flags.
constexpr uint32_t kEpiRuntime = 0xFFFFFFFFu;
template <uint32_t EF>
__device__ __forceinline__ uint32_t epi_flags(const EpiParams& e) {
  return EF == kEpiRuntime ? e.flags : EF;
}

// elementwise part of the epilogue for one value (scalar path)
template <uint32_t EF>
__device__ __forceinline__ void epi_one(const EpiParams& e, int64_t m, int64_t n, float v) {
  const uint32_t f = epi_flags<EF>(e);
  if (f & VS_EPI_BIAS) v += e.bias[n];
  if (f & VS_EPI_POS) v += e.pos[(m % e.pos_rows) * e.N + n];
  if (f & VS_EPI_GELU_BWD) v *= gelu_erf_grad(ld_any(e.aux_in, m * e.ld_aux_in + n, e.op_bf16));
  if (f & VS_EPI_RELU_BWD) v = ld_any(e.aux_in, m * e.ld_aux_in + n, e.op_bf16) > 0.f ? v : 0.f;
  if (f & VS_EPI_MUL_AUX) v *= ld_any(e.aux_in, m * e.ld_aux_in + n, e.op_bf16);
  if (f & VS_EPI_GELU) {
    if (f & VS_EPI_GELU_GRAD) {  // store gelu'(x) for the backward, x = the value it would have seen
      const float x = e.op_bf16 ? bf2f(f2bf(v)) : v;
      st_any(e.aux_out, m * e.ld_aux_out + n, gelu_erf_grad(x), e.op_bf16);
      v = gelu_erf(x);
    } else {
      st_any(e.aux_out, m * e.ld_aux_out + n, v, e.op_bf16);
      v = gelu_erf(e.op_bf16 ? bf2f(f2bf(v)) : v);  // GELU of the value the backward will see
    }
  }
  if (f & VS_EPI_RELU) v = fmaxf(v, 0.f);
  if (f & VS_EPI_RESIDUAL) v += e.residual[m * e.ldr + n];
  if (f & VS_EPI_ACCUM) v += ((const float*)e.c)[m * e.ldc + n];
  st_any(e.c, m * e.ldc + n, v, e.out_bf16);
}

// the same for 8 consecutive columns with 16-B vector accesses, in two halves: fetch (every operand
// load) and finish (arithmetic + stores).  CDNA4's vmcnt counts stores as well as loads and retires
// them in order, so a load issued after a store waits for that store's round trip too: an epilogue
// that runs several 8-column groups per thread fetches all of them before the first finish (one
// store round trip per tile, not one per group).
struct EpiOps8 {
  float bias[8], pos[8], aux[8], res[8], acc[8];
};
template <uint32_t EF>
__device__ __forceinline__ void epi_eight_fetch(const EpiParams& e, int64_t m, int64_t n, EpiOps8& o, bool skip_bias) {
  const uint32_t f = epi_flags<EF>(e) & (skip_bias ? ~(uint32_t)VS_EPI_BIAS : 0xFFFFFFFFu);
  if (f & VS_EPI_BIAS) ld8(e.bias, n, 0, o.bias);
  if (f & VS_EPI_POS) ld8(e.pos, (m % e.pos_rows) * e.N + n, 0, o.pos);
  if (f & (VS_EPI_GELU_BWD | VS_EPI_RELU_BWD | VS_EPI_MUL_AUX)) ld8(e.aux_in, m * e.ld_aux_in + n, e.op_bf16, o.aux);
  if (f & VS_EPI_RESIDUAL) ld8(e.residual, m * e.ldr + n, 0, o.res);
  if (f & VS_EPI_ACCUM) ld8(e.c, m * e.ldc + n, 0, o.acc);
}
template <uint32_t EF>
__device__ __forceinline__ void epi_eight_finish(const EpiParams& e, int64_t m, int64_t n, float (&v)[8], const EpiOps8& o,
                                                 bool skip_bias) {
  const uint32_t f = epi_flags<EF>(e) & (skip_bias ? ~(uint32_t)VS_EPI_BIAS : 0xFFFFFFFFu);
  float t[8];
  if (f & VS_EPI_BIAS) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o.bias[k];
  }
  if (f & VS_EPI_POS) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o.pos[k];
  }
  if (f & VS_EPI_GELU_BWD) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= e.op_bf16 ? gelu_fast_grad(o.aux[k]) : gelu_erf_grad(o.aux[k]);
  } else if (f & VS_EPI_RELU_BWD) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = o.aux[k] > 0.f ? v[k] : 0.f;
  }
  if (f & VS_EPI_MUL_AUX) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= o.aux[k];
  }
  if (f & VS_EPI_GELU) {
    if (f & VS_EPI_GELU_GRAD) {  // store gelu'(x) for the backward, x = the value it would have seen
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float x = e.op_bf16 ? bf2f(f2bf(v[k])) : v[k];
        if (e.op_bf16) v[k] = gelu_fast_both(x, t[k]);
        else {
          t[k] = gelu_erf_grad(x);
          v[k] = gelu_erf(x);
        }
      }
      st8(e.aux_out, m * e.ld_aux_out + n, e.op_bf16, t);
    } else {
      st8(e.aux_out, m * e.ld_aux_out + n, e.op_bf16, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = e.op_bf16 ? gelu_fast(bf2f(f2bf(v[k]))) : gelu_erf(v[k]);
    }
  }
  if (f & VS_EPI_RELU) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (f & VS_EPI_RESIDUAL) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o.res[k];
  }
  if (f & VS_EPI_ACCUM) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o.acc[k];
  }
  st8(e.c, m * e.ldc + n, e.out_bf16, v);
}
template <uint32_t EF>
__device__ __forceinline__ void epi_eight(const EpiParams& e, int64_t m, int64_t n, float (&v)[8], bool skip_bias) {
  EpiOps8 o;
  epi_eight_fetch<EF>(e, m, n, o, skip_bias);
  epi_eight_finish<EF>(e, m, n, v, o, skip_bias);
}

// 4 consecutive columns (n % 4 == 0) of one row, as a lane of the transposed (C^T) MFMA layout holds
// them: 8-B bf16 / 16-B f32 vector accesses for every operand
__device__ __forceinline__ void ld4(const void* p, int64_t i, int bf, float (&v)[4]) {
  if (bf) {
    const uint2 u = *(const uint2*)((const bf16_t*)p + i);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    const float4 a = *(const float4*)((const float*)p + i);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}
__device__ __forceinline__ void st4(void* p, int64_t i, int bf, const float (&v)[4]) {
  if (bf) {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)((bf16_t*)p + i) = u;
  } else {
    *(float4*)((float*)p + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

}  // namespace vs
