// gemm_dw.hip — the weight-gradient products of the backward: C[M,N] += A^T B over the token axis.
//
// Replaces the dW half of autograd for every nn.Linear / Conv3d-as-GEMM of the encoder
// (accelerator.backward, src/trainer/base.py:150): dW2 = dx'^T a (mv:390-397), dW1 = da^T h2
// (mv:373-383), dWproj = dy^T o (mv:312-319), dWqkv = dqkv^T h1 (mv:233-236), the patch-embed
// dW = dx^T cols (mv:176-181), each with the bias gradient (column sums of the dY operand) fused.
//
// Shape: K = B*N tokens (25,088 at the bench) >> M, N (192..1536).  Both operands are token-major
// ([K, features] rows), so the product is a reduction over K and its output is small (0.04-1.2 MB):
// the only parallelism is splitting K.  Design (MI355X):
//   * tile = BM x 64 outputs with BM up to 192 = the WHOLE narrow operand (the host swaps A and B so
//     that A is the narrow one, storing C transposed), so the wide operand is streamed exactly once
//     per token slab and only the narrow one is re-read (from L2: the tiles of one token slab are
//     consecutive logical blocks, which the XCD remap puts on one XCD);
//   * one token slab (split) per workgroup, 4-deep LDS-DMA ring of 64-token steps (asm
//     global_load_lds, counted vmcnt across raw s_barriers, as gemm_bf16_ring_kernel);
//   * the f32 partial tile is written in MFMA FRAGMENT order (each wave-instruction a contiguous
//     1 KiB: no LDS staging), and gemm_dw_reduce adds the splits IN SPLIT ORDER and scatters into C
//     (C += sum): bitwise reproducible, no atomics — also for the fused bias gradient, whose
//     per-split sums go through the same workspace;
//   * the split count comes from a small cost model (plan_dw): enough workgroups to stream at the
//     chip's rate, few enough that the partial tiles (#workgroups x tile bytes) stay a small
//     fraction of the operand bytes.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_dw.h"

namespace vs {

// [64 k][64 rows] bf16 LDS image of an M/N-contiguous operand: the 8-KiB image of OperandBf16<64,
// KC=false> in gemm.hip (16-B chunk XOR on k, read back transposed by ds_read_tr16_b64).
__device__ __forceinline__ int dw_swz(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

// LDS-DMA of one 8-KiB image: 8 pieces of 8 k-rows x 128 B; with NW waves, wave `wid` issues
// pieces wid * (8 / NW) ...  Columns past `cols` re-read the last 8 valid columns, token rows past
// `k_valid` re-read row k_valid - 1 (finite data; those rows are zeroed in LDS before use, those
// columns never stored).
template <int NW>
__device__ __forceinline__ void dw_dma(char* img, const bf16_t* __restrict__ p, int64_t ld, int64_t c0, int64_t cols,
                                       int64_t k0, int k_valid, int wid, int lane) {
#pragma unroll
  for (int j = 0; j < 8 / NW; ++j) {
    const int pi = wid * (8 / NW) + j;
    const int k = pi * 8 + (lane >> 3);
    const int c = (lane & 7) ^ dw_swz(k);
    const int64_t gc = c0 + c * 8 <= cols - 8 ? c0 + c * 8 : cols - 8;
    const int kk = k < k_valid ? k : k_valid - 1;
    glds16_asm(p + (k0 + kk) * ld + gc, img + pi * 1024);
  }
}

// fragment of rows [rb, rb+16) (rb within the image), 32-deep k step kk: lane holds row
// rb + (lane & 15), k = 32 kk + 8 (lane >> 4) + 0..7 (the MFMA 16x16x32 A / B operand layout)
__device__ __forceinline__ bf16x8 dw_frag(const char* img, int rb, int kk, int lane) {
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
  const int col = rb + p4;
  const int k0 = kk * 32 + 8 * (lane >> 4) + q;
  const int k1 = k0 + 4;
  const int off0 = k0 * 128 + (((col >> 3) ^ dw_swz(k0)) << 4) + (col & 7) * 2;
  const int off1 = k1 * 128 + (((col >> 3) ^ dw_swz(k1)) << 4) + (col & 7) * 2;
  short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(img + off0));
  short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(img + off1));
  typedef __attribute__((ext_vector_type(8))) short short8v;
  short8v s = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, s);
}

// SUMS: 0 none; 1 row sums of A (the bias gradient when A is the dY operand), written by the
// nt == 0 tiles; 2 column sums of B (when the host swapped the operands), by the mt == 0 tiles.
// NW = 8 waves (two per SIMD: one wave's DMA issue and LDS reads overlap its partner's MFMAs) in a
// 4 x 2 grid of (BM/4) x 32 wave tiles, or NW = 4 in a 4 x 1 grid of (BM/4) x 64.
// Partial tiles are stored in tile-fragment order: float4 ((rowfrag * 4 + colfrag) * 64 + lane),
// rowfrag / colfrag = the 16-row / 16-column block within the BM x 64 tile.
template <int BM, int SUMS, int NW, int NSTG = 4>
__global__ __launch_bounds__(NW * 64, 1) void gemm_dw_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t M,
                                                             const bf16_t* __restrict__ B, int64_t ldb, int64_t N,
                                                             int64_t K, DwGrid g, float* __restrict__ part,
                                                             float* __restrict__ sums) {
  constexpr int NA = BM / 64;             // 64-row A images per stage
  constexpr int IMG = 8192;
  constexpr int STAGE = (NA + 1) * IMG;   // A images then the B image
  constexpr int PER = (NA + 1) * (8 / NW);  // DMA wave-instructions per stage
  constexpr int WM = BM / 4, FI = WM / 16, FJ = NW == 8 ? 2 : 4;
  static_assert(NSTG == 3 || NSTG == 4, "3- or 4-stage ring");
  __shared__ __attribute__((aligned(16))) char st0[STAGE];
  __shared__ __attribute__((aligned(16))) char st1[STAGE];
  __shared__ __attribute__((aligned(16))) char st2[STAGE];
  __shared__ __attribute__((aligned(16))) char st3[NSTG == 4 ? STAGE : 16];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wid & 3, cw = wid >> 2;  // wave tile: rows rw*WM.., columns cw*FJ*16..
  const int tiles = g.tiles_m * g.tiles_n;
  const int t = xcd_remap(blockIdx.x, gridDim.x);   // one token slab's tiles are consecutive: one XCD
  const int split = t / tiles, rem = t % tiles, mt = rem / g.tiles_n, nt = rem % g.tiles_n;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * 64;
  const int nk_all = (int)((K + 63) / 64);
  const int ks0 = split * g.ksteps, ks1 = ks0 + g.ksteps < nk_all ? ks0 + g.ksteps : nk_all;
  const int nk = ks1 - ks0;

  f32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool sum_on = (SUMS == 1 && nt == 0 && cw == 0) || (SUMS == 2 && mt == 0 && rw == 0);
  float sacc[SUMS == 2 ? FJ : FI];
#pragma unroll
  for (int i = 0; i < (SUMS == 2 ? FJ : FI); ++i) sacc[i] = 0.f;

  auto issue = [&](int s, char* stg) {
    const int64_t k0 = (int64_t)(ks0 + s) * 64;
    const int kv = K - k0 < 64 ? (int)(K - k0) : 64;
#pragma unroll
    for (int a = 0; a < NA; ++a) dw_dma<NW>(stg + a * IMG, A, lda, m0 + a * 64, M, k0, kv, wid, lane);
    dw_dma<NW>(stg + NA * IMG, B, ldb, n0, N, k0, kv, wid, lane);
  };
  auto compute = [&](const char* stg) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FI], bfr[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int r = rw * WM + i * 16;  // r and r+15 lie in the same 64-row image (WM % 16 == 0)
        af[i] = dw_frag(stg + (r >> 6) * IMG, r & 63, kk, lane);
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j) bfr[j] = dw_frag(stg + NA * IMG, (cw * FJ + j) * 16, kk, lane);
      if (sum_on) {
        if constexpr (SUMS == 1) {
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) sacc[i] += (float)af[i][q];
        } else if constexpr (SUMS == 2) {
#pragma unroll
          for (int j = 0; j < FJ; ++j)
#pragma unroll
            for (int q = 0; q < 8; ++q) sacc[j] += (float)bfr[j][q];
        }
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // rows k >= k_valid of a partial last step hold re-read data: zero them in every image
  auto zero_tail = [&](char* stg, int kv) {
    const int bytes = (64 - kv) * 128;
    for (int a = 0; a <= NA; ++a)
      for (int o = tid * 16; o < bytes; o += NW * 64 * 16) *(uint4*)(stg + a * IMG + kv * 128 + o) = make_uint4(0, 0, 0, 0);
  };
  auto step = [&](int s, auto sc) {
    constexpr int S = decltype(sc)::value;
    char* cur = S == 0 ? st0 : S == 1 ? st1 : S == 2 ? st2 : st3;
    // stage of step s + NSTG - 1 (the one step s - 1 used)
    char* far = NSTG == 4 ? (S == 0 ? st3 : S == 1 ? st0 : S == 2 ? st1 : st2) : (S == 0 ? st2 : S == 1 ? st0 : st1);
    // steps s+1 .. s+NSTG-2 may stay in flight
    if (NSTG == 4 && s + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (s + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's step-s pieces landed; step s-1's stage is free
    asm volatile("" ::: "memory");
    const int64_t k0 = (int64_t)(ks0 + s) * 64;
    if (K - k0 < 64) {  // block-uniform: only the very last token step of the whole reduction
      zero_tail(cur, (int)(K - k0));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (s + NSTG - 1 < nk) issue(s + NSTG - 1, far);
    compute(cur);
  };
  if (nk > 0) issue(0, st0);
  if (nk > 1) issue(1, st1);
  if (NSTG == 4 && nk > 2) issue(2, st2);
  for (int s = 0; s < nk; s += NSTG) {
    step(s, IC<0>{});
    if (s + 1 < nk) step(s + 1, IC<1>{});
    if (s + 2 < nk) step(s + 2, IC<2>{});
    if (NSTG == 4 && s + 3 < nk) step(s + 3, IC<3>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float4* pt = (float4*)(part + ((int64_t)rem * g.splits + split) * (BM * 64));
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const f32x4 v = acc[i][j];
      pt[((rw * FI + i) * 4 + cw * FJ + j) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
    }
  if (sum_on) {
    // lane groups g = lane >> 4 hold disjoint k; rows / columns (lane & 15)
    constexpr int NS = SUMS == 2 ? FJ : FI;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      float v = sacc[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      sacc[i] = v;
    }
    if (lane < 16) {
      if constexpr (SUMS == 1) {
        float* so = sums + ((int64_t)mt * g.splits + split) * BM;
#pragma unroll
        for (int i = 0; i < FI; ++i) so[rw * WM + i * 16 + lane] = sacc[i];
      } else if constexpr (SUMS == 2) {
        float* so = sums + ((int64_t)nt * g.splits + split) * 64;
#pragma unroll
        for (int j = 0; j < FJ; ++j) so[(cw * FJ + j) * 16 + lane] = sacc[j];
      }
    }
  }
}

// The same product with REGISTER-staged operands: per 64-token step each thread loads (NA+1)*2
// 16-B chunks with global_load_dwordx4 (a few issue cycles each, against ~60-180 for an LDS-DMA
// piece, which made the DMA ring above issue-bound at ~26 GB/s per CU with one wave per SIMD),
// two steps in flight in two register sets, written into a double-buffered LDS image one step
// ahead of the MFMAs (guide T14: issue early, write late).  64 KB of LDS at BM = 192: two
// workgroups per CU, 8 waves to hide the load latency.  Token rows past K load zeros.
template <int BM, int SUMS>
__global__ __launch_bounds__(256, 2) void gemm_dw_reg_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t M,
                                                             const bf16_t* __restrict__ B, int64_t ldb, int64_t N,
                                                             int64_t K, DwGrid g, float* __restrict__ part,
                                                             float* __restrict__ sums) {
  constexpr int NA = BM / 64;
  constexpr int IMG = 8192;
  constexpr int STAGE = (NA + 1) * IMG;
  constexpr int CPT = (NA + 1) * 2;       // 16-B chunks per thread per step
  constexpr int WM = BM / 4, FI = WM / 16, FJ = 4;
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles = g.tiles_m * g.tiles_n;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int split = t / tiles, rem = t % tiles, mt = rem / g.tiles_n, nt = rem % g.tiles_n;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * 64;
  const int nk_all = (int)((K + 63) / 64);
  const int ks0 = split * g.ksteps, ks1 = ks0 + g.ksteps < nk_all ? ks0 + g.ksteps : nk_all;
  const int nk = ks1 - ks0;

  // chunk c of this thread: image im = c / 2 (im == NA: B), index i = tid + 256 (c & 1):
  // k = i / 8, 16-B column chunk q = i % 8 (one 128-B segment per 8 lanes)
  const int kq0 = tid >> 3, q = tid & 7;  // i = tid (+256 -> k + 32)
  auto load = [&](uint4 (&r)[CPT], int s) {
    const int64_t k0 = (int64_t)(ks0 + s) * 64;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int im = c >> 1, k = kq0 + 32 * (c & 1);
      const bf16_t* p = im < NA ? A : B;
      const int64_t ld = im < NA ? lda : ldb;
      const int64_t col = (im < NA ? m0 + im * 64 : n0) + q * 8;
      const int64_t lim = im < NA ? M : N;
      const bool ok = k0 + k < K && col < lim;
      r[c] = ok ? *(const uint4*)(p + (k0 + k) * ld + col) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](const uint4 (&r)[CPT], char* stg) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int im = c >> 1, k = kq0 + 32 * (c & 1);
      *(uint4*)(stg + im * IMG + k * 128 + ((q ^ dw_swz(k)) << 4)) = r[c];
    }
  };

  f32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool sum_on = (SUMS == 1 && nt == 0) || (SUMS == 2 && mt == 0 && wid == 0);
  float sacc[SUMS == 2 ? FJ : FI];
#pragma unroll
  for (int i = 0; i < (SUMS == 2 ? FJ : FI); ++i) sacc[i] = 0.f;

  auto compute = [&](const char* stg) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FI], bfr[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int r = wid * WM + i * 16;
        af[i] = dw_frag(stg + (r >> 6) * IMG, r & 63, kk, lane);
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j) bfr[j] = dw_frag(stg + NA * IMG, j * 16, kk, lane);
      if (sum_on) {
        if constexpr (SUMS == 1) {
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int qq = 0; qq < 8; ++qq) sacc[i] += (float)af[i][qq];
        } else if constexpr (SUMS == 2) {
#pragma unroll
          for (int j = 0; j < FJ; ++j)
#pragma unroll
            for (int qq = 0; qq < 8; ++qq) sacc[j] += (float)bfr[j][qq];
        }
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  uint4 ra[CPT], rb[CPT];
  if (nk > 0) load(ra, 0);
  if (nk > 1) load(rb, 1);
  if (nk > 0) store(ra, lds);                 // waits for step 0's loads only (compiler-counted)
  if (nk > 2) load(ra, 2);
  __syncthreads();
  // step s computes from lds[s & 1]; meanwhile step s+1 (regs) is stored into the other half and
  // step s+3 is loaded into the freed register set
  auto step = [&](int s, uint4 (&cur)[CPT], uint4 (&nxt)[CPT]) {
    compute(lds + (s & 1) * STAGE);
    if (s + 1 < nk) store(cur, lds + ((s + 1) & 1) * STAGE);
    if (s + 3 < nk) load(cur, s + 3);
    __syncthreads();
    (void)nxt;
  };
  for (int s = 0; s < nk; s += 2) {
    step(s, rb, ra);
    if (s + 1 < nk) step(s + 1, ra, rb);
  }

  float4* pt = (float4*)(part + ((int64_t)rem * g.splits + split) * (BM * 64));
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const f32x4 v = acc[i][j];
      pt[((wid * FI + i) * FJ + j) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
    }
  if (sum_on) {
    constexpr int NS = SUMS == 2 ? FJ : FI;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      float v = sacc[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      sacc[i] = v;
    }
    if (lane < 16) {
      if constexpr (SUMS == 1) {
        float* so = sums + ((int64_t)mt * g.splits + split) * BM;
#pragma unroll
        for (int i = 0; i < FI; ++i) so[wid * WM + i * 16 + lane] = sacc[i];
      } else if constexpr (SUMS == 2) {
        float* so = sums + ((int64_t)nt * g.splits + split) * 64;
#pragma unroll
        for (int j = 0; j < FJ; ++j) so[j * 16 + lane] = sacc[j];
      }
    }
  }
}

// C (+)= sum over splits of the fragment-order partial tiles.  A workgroup owns 64 float4 of one
// tile (one per lane); wave w sums splits w, w+4, ... (all loads of its share issued before the
// adds), then the four wave sums are added in wave order through LDS — a fixed order that depends
// only on the split count (bitwise reproducible).  Blocks after the tile blocks reduce the bias
// sums.  TRANS: the kernel ran on swapped operands, so its tile element (m, n) is C[n][m].
template <int BM, bool TRANS>
__global__ __launch_bounds__(1024) void gemm_dw_reduce(const float* __restrict__ part, const float* __restrict__ sums,
                                                       DwGrid g, int64_t M, int64_t N, float* __restrict__ c,
                                                       int64_t ldc, float* __restrict__ bias_out, int64_t sum_len,
                                                       int sum_tiles, int sum_w) {
  constexpr int Q = BM * 16;  // float4 per tile
  constexpr int NWR = 16;     // waves per block: wave w sums splits w, w + 16, ... (<= 4 loads in flight each)
  const int tiles = g.tiles_m * g.tiles_n;
  const int64_t blk = blockIdx.x;
  const int64_t tile_blocks = (int64_t)tiles * (Q / 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (blk < tile_blocks) {
    __shared__ float4 red[NWR][64];
    const int tile = (int)(blk / (Q / 64));
    const int q = (int)(blk % (Q / 64)) * 64 + lane;
    const float4* p = (const float4*)(part + (int64_t)tile * g.splits * (BM * 64)) + q;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sp0 = w; sp0 < g.splits; sp0 += NWR * 4) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int sp = sp0 + NWR * u;
        v[u] = sp < g.splits ? p[(int64_t)sp * Q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
      }
    }
    red[w][lane] = s;
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int k = 1; k < NWR; ++k) {  // fixed wave order
      const float4 o = red[k][lane];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    const int f = q >> 6, rf = f >> 2, cf = f & 3;
    const int mt = tile / g.tiles_n, nt = tile % g.tiles_n;
    const int64_t n = (int64_t)nt * 64 + cf * 16 + (lane & 15);
    const int64_t mb = (int64_t)mt * BM + rf * 16 + (lane >> 4) * 4;
    const float vv[4] = {s.x, s.y, s.z, s.w};
    if (n < N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = mb + r;
        if (m < M) {
          float* dst = TRANS ? c + n * ldc + m : c + m * ldc + n;
          *dst += vv[r];
        }
      }
    }
    return;
  }
  const int64_t e = (blk - tile_blocks) * 1024 + threadIdx.x;  // element of the bias vector
  if (e >= sum_len) return;
  const int64_t st = e / sum_w, off = e % sum_w;
  if (st >= sum_tiles) return;
  const float* p = sums + st * (int64_t)g.splits * sum_w + off;
  float s = 0.f;
  int sp = 0;
  for (; sp + 8 <= g.splits; sp += 8) {  // 8 loads in flight (a serial chain of 50 loads took ~10 us)
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(sp + u) * sum_w];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; sp < g.splits; ++sp) s += p[(int64_t)sp * sum_w];
  bias_out[e] += s;
}

// The same reduction for few splits (S <= 8: the ViT-Base products, whose many output tiles leave
// one or two splits): one float4 of a tile per thread in 256-thread blocks, the splits added in
// split order (the 16-wave layout above left 15 of 16 waves idle there and ran latency-bound,
// 363 us for a 9.4 MB dW at S = 1).  TRANS stores the 4 consecutive m of a lane as one float4.
template <int BM, bool TRANS>
__global__ __launch_bounds__(256) void gemm_dw_reduce_few(const float* __restrict__ part, const float* __restrict__ sums,
                                                          DwGrid g, int64_t M, int64_t N, float* __restrict__ c,
                                                          int64_t ldc, float* __restrict__ bias_out, int64_t sum_len,
                                                          int sum_tiles, int sum_w) {
  constexpr int Q = BM * 16;  // float4 per tile
  const int tiles = g.tiles_m * g.tiles_n;
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile_items = (int64_t)tiles * Q;
  if (item < tile_items) {
    const int tile = (int)(item / Q), q = (int)(item % Q), lane = q & 63;
    const float4* p = (const float4*)(part + (int64_t)tile * g.splits * (BM * 64)) + q;
    float4 sum = p[0];
    for (int sp = 1; sp < g.splits; ++sp) {
      const float4 o = p[(int64_t)sp * Q];
      sum.x += o.x; sum.y += o.y; sum.z += o.z; sum.w += o.w;
    }
    const int f = q >> 6, rf = f >> 2, cf = f & 3;
    const int mt = tile / g.tiles_n, nt = tile % g.tiles_n;
    const int64_t n = (int64_t)nt * 64 + cf * 16 + (lane & 15);
    const int64_t mb = (int64_t)mt * BM + rf * 16 + (lane >> 4) * 4;
    if (n >= N) return;
    const float vv[4] = {sum.x, sum.y, sum.z, sum.w};
    if (TRANS && mb + 4 <= M && ldc % 4 == 0) {
      float4* dst = (float4*)(c + n * ldc + mb);
      float4 o = *dst;
      o.x += vv[0]; o.y += vv[1]; o.z += vv[2]; o.w += vv[3];
      *dst = o;
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mb + r;
      if (m < M) {
        float* dst = TRANS ? c + n * ldc + m : c + m * ldc + n;
        *dst += vv[r];
      }
    }
    return;
  }
  const int64_t e = item - tile_items;  // element of the bias vector
  if (e >= sum_len) return;
  const int64_t st = e / sum_w, off = e % sum_w;
  if (st >= sum_tiles) return;
  const float* ps = sums + st * (int64_t)g.splits * sum_w + off;
  float acc = 0.f;
  for (int sp = 0; sp < g.splits; ++sp) acc += ps[(int64_t)sp * sum_w];
  bias_out[e] += acc;
}

// ---------------------------------------------------------------------------------------------
// Skinny split-K product with both operands K-contiguous: C[M,N] (+)= A[M,K] B[N,K]^T (+ bias),
// M <= 64, N <= 256, K huge — the head's Linear(N*D -> 64) forward (src/model/videomae.py:13,29:
// M = batch, K = 301,056 at the bench, 1.2 M at ViT-Base) and the Linear plugin's first layer
// (src/model/linear.py:26: K = 120*128*128 = 1,966,080, a 503 M-parameter f32 weight), both
// HBM-bound on the weight.  Each operand element is used by ONE wave, so the MFMA fragments are
// loaded straight from global memory, no LDS: per 16-B load a lane holds
//   bf16: 8 consecutive k of row (lane & 15) at k0 + 8 (lane >> 4)  (the 16x16x32 operand layout);
//   f32:  4 consecutive k at k0 + 4 (lane >> 4), consumed by 4 exact-f32 16x16x4 MFMAs, MFMA j
//         taking element j (a fixed permutation of the k order inside each 16-deep step, the same
//         for A and B: it changes only the f32 summation order).
// Wave w of a workgroup takes steps w, w+4, ... of the workgroup's K slice with U steps of loads in
// flight; the four wave tiles are added through LDS in wave order and the workgroup's f32 partial
// [M][N] goes to the split-K workspace, summed in split order by gemm_splitk_reduce_wide (gemm.hip).
template <typename T, int FI, int FJ>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const T* __restrict__ A, int64_t lda, int64_t M,
                                                          const T* __restrict__ B, int64_t ldb, int64_t N,
                                                          int64_t K, int steps_per_split, float* __restrict__ part) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int KS = BF ? 32 : 16;               // k per step
  constexpr int U = FJ <= 4 ? 4 : 2;             // steps of loads in flight per wave
  typedef __attribute__((ext_vector_type(4))) float f32v4;
  typedef typename std::conditional<BF, bf16x8, f32v4>::type Frag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t nsteps = K / KS;
  const int64_t s0 = (int64_t)blockIdx.x * steps_per_split;
  const int64_t s1 = s0 + steps_per_split < nsteps ? s0 + steps_per_split : nsteps;
  const int r = lane & 15, kq = (BF ? 8 : 4) * (lane >> 4);
  const T* ap[FI];
  const T* bp[FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i) {
    const int64_t row = i * 16 + r < M ? i * 16 + r : M - 1;  // rows past M: finite, never stored
    ap[i] = A + row * lda + kq;
  }
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int64_t row = j * 16 + r < N ? j * 16 + r : N - 1;
    bp[j] = B + row * ldb + kq;
  }
  f32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t st = s0 + w; st < s1; st += 4 * U) {
    Frag a[U][FI], b[U][FJ];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = (st + 4 * u < s1 ? st + 4 * u : st) * KS;   // past the slice: re-read, not used
#pragma unroll
      for (int i = 0; i < FI; ++i) a[u][i] = *(const Frag*)(ap[i] + k);
#pragma unroll
      for (int j = 0; j < FJ; ++j) b[u][j] = *(const Frag*)(bp[j] + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (st + 4 * u < s1) {
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int j = 0; j < FJ; ++j) {
            if constexpr (BF) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][i][e], b[u][j][e], acc[i][j], 0, 0, 0);
            }
          }
      }
    }
  }
  // wave tiles -> LDS -> summed in wave order; C layout 16x16: acc[r4] at row 4 (lane >> 4) + r4, col lane & 15
  __shared__ float red[4][FI * 16][FJ * 16 + 1];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) red[w][i * 16 + 4 * (lane >> 4) + r4][j * 16 + (lane & 15)] = acc[i][j][r4];
  __syncthreads();
  float* pt = part + (int64_t)blockIdx.x * M * N;
  for (int e = tid; e < M * N; e += 256) {
    const int m = (int)(e / N), n = (int)(e % N);
    pt[e] = ((red[0][m][n] + red[1][m][n]) + red[2][m][n]) + red[3][m][n];
  }
}

static int skinny_ks(int dtype) { return dtype == VS_BF16 ? 32 : 16; }

bool skinny_ok(const vs_gemm_desc* d) {
  const uint32_t f = d->epilogue;
  const int ks = skinny_ks(d->dtype);
  const int vec = d->dtype == VS_BF16 ? 8 : 4;
  const int max_fj = d->M <= 16 ? 16 : 4;     // LDS / register budget: FI * FJ <= 16
  return (d->dtype == VS_BF16 || d->dtype == VS_F32) && d->out_dtype == VS_F32 && d->a_kcontig && d->b_kcontig &&
         d->M >= 1 && d->M <= 64 && d->N >= 16 && d->N <= 16 * max_fj && d->N % 16 == 0 && d->K % ks == 0 &&
         d->lda % vec == 0 && d->ldb % vec == 0 && (f & VS_EPI_ATOMIC) &&
         !(f & ~(uint32_t)(VS_EPI_ATOMIC | VS_EPI_BIAS | VS_EPI_RELU)) && !d->a_rowsum && d->split_k <= 0 &&
         d->K / ks >= 64;
}

static int skinny_splits(int64_t K, int ks, int64_t* steps_per_split) {
  const int64_t nsteps = K / ks;
  int64_t S = nsteps / 32;               // >= 8 steps per wave
  if (S > 1024) S = 1024;
  if (S < 1) S = 1;
  const int64_t sps = (nsteps + S - 1) / S;
  *steps_per_split = sps;
  return (int)((nsteps + sps - 1) / sps);
}

size_t skinny_workspace_bytes(int32_t dtype, int64_t M, int64_t N, int64_t K) {
  const int ks = skinny_ks(dtype);
  if (M < 1 || M > 64 || N > 256 || K % ks != 0 || K / ks < 64) return 0;
  int64_t sps;
  const int S = skinny_splits(K, ks, &sps);
  return (size_t)S * (size_t)(M * N) * 4;
}

template <typename T>
static void launch_skinny_t(const vs_gemm_desc* d, int FI, int FJ, int S, int64_t sps, float* part, hipStream_t s) {
  const T* a = (const T*)d->a;
  const T* b = (const T*)d->b;
#define SK_(I, J)                                                                                                   \
  hipLaunchKernelGGL((gemm_skinny_kernel<T, I, J>), dim3((unsigned)S), dim3(256), 0, s, a, d->lda, d->M, b, d->ldb, \
                     d->N, d->K, (int)sps, part)
  if (FI == 1) {
    switch (FJ) {
      case 1: SK_(1, 1); break;
      case 2: SK_(1, 2); break;
      case 3: SK_(1, 3); break;
      case 4: SK_(1, 4); break;
      case 8: SK_(1, 8); break;
      default: SK_(1, 16); break;   // N <= 256: columns past N re-read row N-1 and are not stored
    }
  } else {
    const int fj = FJ <= 1 ? 1 : FJ <= 2 ? 2 : FJ <= 3 ? 3 : 4;
#define SK_J(I)                      \
  do {                               \
    if (fj == 1) SK_(I, 1);          \
    else if (fj == 2) SK_(I, 2);     \
    else if (fj == 3) SK_(I, 3);     \
    else SK_(I, 4);                  \
  } while (0)
    if (FI == 2) SK_J(2);
    else if (FI == 3) SK_J(3);
    else SK_J(4);
#undef SK_J
  }
#undef SK_
}

int launch_skinny(const vs_gemm_desc* d, hipStream_t s, int* splits_out) {
  int64_t sps;
  const int S = skinny_splits(d->K, skinny_ks(d->dtype), &sps);
  VS_REQUIRE((size_t)d->workspace_bytes >= (size_t)S * (size_t)(d->M * d->N) * 4, "vs_gemm: skinny workspace too small");
  const int FI = (int)((d->M + 15) / 16);
  int FJ = (int)(d->N / 16);
  if (FI == 1 && FJ > 4) FJ = FJ <= 8 ? 8 : 16;
  if (d->dtype == VS_BF16) launch_skinny_t<bf16_t>(d, FI, FJ, S, sps, (float*)d->workspace, s);
  else launch_skinny_t<float>(d, FI, FJ, S, sps, (float*)d->workspace, s);
  *splits_out = S;
  return VS_OK;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && v[0] ? atoi(v) : dflt;
}

// Cost model (microseconds): the workgroups stream their token slab of both operands (L2/HBM ->
// LDS at ~80 GB/s per CU), then the partial tiles are written and re-read by the reduce (at ~5 TB/s
// each way), plus the reduce launch.  Splits keep >= 8 token steps each.
DwPlan plan_dw(int64_t M, int64_t N, int64_t K) {
  DwPlan best = {};
  best.valid = false;
  const bool swap = M > N;
  const int64_t Ma = swap ? N : M, Nb = swap ? M : N;
  const int64_t nk = (K + 63) / 64;
  const int force_bm = env_int("VSPIKE_DW_BM", 0);
  const bool dma = env_int("VSPIKE_DW_MODE", 1) == 1;   // 1: 8-wave LDS-DMA ring (default), 0: register-staged
  double best_t = 1e30;
  for (int BM : {64, 128, 192}) {
    if (force_bm && BM != force_bm) continue;
    const int64_t tm = (Ma + BM - 1) / BM, tn = (Nb + 63) / 64, tiles = tm * tn;
    const int slots = (BM == 64 || !dma) ? 512 : 256;
    int64_t S = slots / tiles;
    const int force_s = env_int("VSPIKE_DW_SPLITS", 0);
    if (force_s > 0) S = force_s;
    if (S < 1) S = 1;
    const int64_t smax = nk / 8 > 0 ? nk / 8 : 1;
    if (S > smax) S = smax;
    int64_t kps = (nk + S - 1) / S;
    S = (nk + kps - 1) / kps;
    const int64_t wgs = tiles * S;
    const double per_wg = (double)kps * 64.0 * (BM + 64) * 2.0;
    const double rate = slots == 512 ? 40e3 : 80e3;  // bytes / us per workgroup (2 or 1 per CU)
    const double rounds = (double)((wgs + slots - 1) / slots);
    const double part = (double)wgs * BM * 64 * 4.0;
    const double t = rounds * per_wg / rate + 2.0 * part / 5e6 + 3.0 + (BM - Ma > 0 ? 0.0 : 0.0);
    // wasted rows of the last A tile cost their share of the stream
    const double waste = (double)(tm * BM - Ma) / (double)(tm * BM);
    const double tt = t * (1.0 + 0.5 * waste);
    if (tt < best_t) {
      best_t = tt;
      best.valid = true;
      best.dma = dma;
      best.swap = swap;
      best.BM = BM;
      best.g.tiles_m = (int)tm;
      best.g.tiles_n = (int)tn;
      best.g.splits = (int)S;
      best.g.ksteps = (int)kps;
      best.part_floats = (int64_t)wgs * BM * 64;
      best.sum_floats = (int64_t)S * (tm * BM > tn * 64 ? tm * BM : tn * 64);
    }
  }
  return best;
}

size_t dw_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const DwPlan p = plan_dw(M, N, K);
  if (!p.valid) return 0;
  return (size_t)(p.part_floats + p.sum_floats + 64) * 4;
}

template <int BM, int SUMS, bool TRANS>
static void launch_dw_t(const bf16_t* a, int64_t lda, int64_t Ma, const bf16_t* b, int64_t ldb, int64_t Nb, int64_t K,
                        const DwPlan& p, float* part, float* sums, float* c, int64_t ldc, float* bias, hipStream_t s) {
  const unsigned nwg = (unsigned)(p.g.tiles_m * p.g.tiles_n * p.g.splits);
  static const int stages = env_int("VSPIKE_DW_STAGES", 4);
  if (p.dma && stages == 3)
    hipLaunchKernelGGL((gemm_dw_kernel<BM, SUMS, 8, 3>), dim3(nwg), dim3(512), 0, s, a, lda, Ma, b, ldb, Nb, K, p.g,
                       part, sums);
  else if (p.dma)
    hipLaunchKernelGGL((gemm_dw_kernel<BM, SUMS, 8>), dim3(nwg), dim3(512), 0, s, a, lda, Ma, b, ldb, Nb, K, p.g, part,
                       sums);
  else
    hipLaunchKernelGGL((gemm_dw_reg_kernel<BM, SUMS>), dim3(nwg), dim3(256), 0, s, a, lda, Ma, b, ldb, Nb, K, p.g, part,
                       sums);
  const int tiles = p.g.tiles_m * p.g.tiles_n;
  const int64_t tile_blocks = (int64_t)tiles * (BM * 16 / 64);
  int64_t sum_len = 0, sum_w = 1;
  int sum_tiles = 0;
  if (SUMS == 1) {
    sum_w = BM;
    sum_tiles = p.g.tiles_m;
    sum_len = Ma;
  } else if (SUMS == 2) {
    sum_w = 64;
    sum_tiles = p.g.tiles_n;
    sum_len = Nb;
  }
  // C is [M][N] of the ORIGINAL product: with TRANS the kernel's (m, n) = (original n, original m)
  if (p.g.splits <= 8) {
    const int64_t items = (int64_t)tiles * (BM * 16) + sum_len;
    hipLaunchKernelGGL((gemm_dw_reduce_few<BM, TRANS>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, part,
                       sums, p.g, Ma, Nb, c, ldc, bias, sum_len, sum_tiles, (int)sum_w);
    return;
  }
  const int64_t blocks = tile_blocks + (sum_len + 1023) / 1024;
  hipLaunchKernelGGL((gemm_dw_reduce<BM, TRANS>), dim3((unsigned)blocks), dim3(1024), 0, s, part, sums, p.g, Ma, Nb, c,
                     ldc, bias, sum_len, sum_tiles, (int)sum_w);
}

int launch_dw(const vs_gemm_desc* d, hipStream_t s) {
  const DwPlan p = plan_dw(d->M, d->N, d->K);
  VS_REQUIRE(p.valid, "vs_gemm: no dW plan");
  VS_REQUIRE((size_t)d->workspace_bytes >= dw_workspace_bytes(d->M, d->N, d->K), "vs_gemm: dW workspace too small");
  float* part = (float*)d->workspace;
  float* sums = part + p.part_floats;
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  float* c = (float*)d->c;
  float* bias = d->a_rowsum;
  // swap: A' = B (the narrow operand), B' = A; the bias (row sums of the ORIGINAL A) = column sums of B'
  const bf16_t* aa = p.swap ? b : a;
  const bf16_t* bb = p.swap ? a : b;
  const int64_t la = p.swap ? d->ldb : d->lda, lb = p.swap ? d->lda : d->ldb;
  const int64_t Ma = p.swap ? d->N : d->M, Nb = p.swap ? d->M : d->N;
  const int sm = !bias ? 0 : (p.swap ? 2 : 1);
#define DW_(BM_, S_, T_) launch_dw_t<BM_, S_, T_>(aa, la, Ma, bb, lb, Nb, d->K, p, part, sums, c, d->ldc, bias, s)
#define DW_BM(BM_)                                  \
  do {                                              \
    if (p.swap) {                                   \
      if (sm == 2) DW_(BM_, 2, true);               \
      else DW_(BM_, 0, true);                       \
    } else {                                        \
      if (sm == 1) DW_(BM_, 1, false);              \
      else DW_(BM_, 0, false);                      \
    }                                               \
  } while (0)
  if (p.BM == 64) DW_BM(64);
  else if (p.BM == 128) DW_BM(128);
  else DW_BM(192);
#undef DW_BM
#undef DW_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

}  // namespace vs
