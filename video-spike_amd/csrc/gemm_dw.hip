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
//   * tile = BM x BN outputs, BM up to 192 = the WHOLE narrow operand (the host swaps A and B so
//     that A is the narrow one, storing C transposed), BN = 64 or 128 columns of the wide one, so the
//     wide operand is streamed exactly once per token slab and only the narrow one is re-read (from
//     L2: the tiles of one token slab are consecutive logical blocks, which the XCD remap puts on
//     one XCD).  BN = 128 halves the narrow re-reads and doubles the MFMAs per LDS-DMA byte;
//   * one token slab (split) per workgroup, 3- or 4-deep LDS-DMA ring of 64-token steps (asm
//     global_load_lds with step-invariant per-lane offsets from one SGPR base per operand, counted
//     vmcnt across raw s_barriers, as gemm_bf16_ring_kernel);
//   * the f32 partial tile is written in MFMA FRAGMENT order (each wave-instruction a contiguous
//     1 KiB: no LDS staging), and gemm_dw_reduce adds the splits IN SPLIT ORDER and scatters into C
//     (C += sum): bitwise reproducible, no atomics — also for the fused bias gradient, whose
//     per-split sums go through the same workspace;
//   * tile shape and split count come from a small cost model (plan_dw): enough workgroups to
//     stream at the chip's rate, few enough that the partial tiles (#workgroups x tile bytes) stay a
//     small fraction of the operand bytes.
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
// Tile BM x BN (BM, BN multiples of 64: NA + NB 64-column LDS images per token step), 8 waves
// (two per SIMD: one wave's DMA issue and LDS reads overlap its partner's MFMAs) in a 4 x 2 grid
// of (BM/4) x (BN/2) wave tiles.  Per 64-token step each wave issues piece `wid` (8 token rows x
// 128 B) of every image; its per-lane source offsets are step-invariant (column clamps included)
// and computed once, so a step's DMA is one SGPR base per operand + NA + NB instructions.
// Partial tiles are stored in tile-fragment order: float4 ((rowfrag * BN/16 + colfrag) * 64 + lane),
// rowfrag / colfrag = the 16-row / 16-column block within the tile.
//
// PX (the patch embedding's dW, mv:176-181): B is not a tensor but the tubelet gather of the f32
// pixels — column n = (c, t, i, j) of token m = (b, f', hp, wp) is px[b][2f'+t][c][16hp+i][16wp+j].
// A lane's 16-B piece of a B image (token row krow, 8 columns n..n+7 = 8 adjacent pixels of one
// image row) is two 16-B global loads at a step-invariant column offset plus the token's base,
// converted to bf16 (RNE, as im2col) and written to the LDS position the DMA would fill: the MFMA
// side and the reduction are the plain kernel's, so the result is bitwise im2col + dW.  The loads of
// step s + 1 are issued (asm, counted waits) before step s's MFMAs and written to LDS after them;
// the A operand (dx) keeps the LDS-DMA, two steps ahead.  NSTG = 3.
template <int BM, int BN, int SUMS, int NSTG, bool PX = false>
__global__ __launch_bounds__(512, 1) void gemm_dw_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t M,
                                                         const bf16_t* __restrict__ B, int64_t ldb, int64_t N,
                                                         int64_t K, DwGrid g, float* __restrict__ part,
                                                         float* __restrict__ sums, const float* __restrict__ px,
                                                         PatchDwGeo pg) {
  constexpr int NA = BM / 64, NB = BN / 64, NI = NA + NB;  // 64-column LDS images per stage
  constexpr int IMG = 8192;
  constexpr int STAGE = NI * IMG;
  constexpr int PER = PX ? NA : NI;       // DMA wave-instructions per wave per stage
  static_assert(!PX || NSTG == 3, "the gather variant runs the 3-stage ring");
  constexpr int WM = BM / 4, FI = WM / 16, WN = BN / 2, FJ = WN / 16, CF = BN / 16;
  static_assert(NSTG >= 2 && NSTG <= 4, "2- to 4-stage ring");
  __shared__ __attribute__((aligned(16))) char st0[STAGE];
  __shared__ __attribute__((aligned(16))) char st1[STAGE];
  __shared__ __attribute__((aligned(16))) char st2[NSTG >= 3 ? STAGE : 16];
  __shared__ __attribute__((aligned(16))) char st3[NSTG == 4 ? STAGE : 16];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wid & 3, cw = wid >> 2;  // wave tile: rows rw*WM.., columns cw*WN..
  const int tiles = g.tiles_m * g.tiles_n;
  const int t = xcd_remap(blockIdx.x, gridDim.x);   // one token slab's tiles are consecutive: one XCD
  const int split = t / tiles, rem = t % tiles, mt = rem / g.tiles_n, nt = rem % g.tiles_n;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * BN;
  const int nk_all = (int)((K + 63) / 64);
  const int ks0 = split * g.ksteps, ks1 = ks0 + g.ksteps < nk_all ? ks0 + g.ksteps : nk_all;
  const int nk = ks1 - ks0;

  // this lane's DMA position: token row krow of the step, 16-B chunk cch of its image row; columns
  // past the operand re-read its last 8 (finite data, never stored)
  const int krow = wid * 8 + (lane >> 3);
  const int cch = (lane & 7) ^ dw_swz(krow);
  auto col_of = [&](int j) -> int64_t {
    const int64_t c0 = j < NA ? m0 + j * 64 : n0 + (j - NA) * 64;
    const int64_t cols = j < NA ? M : N;
    return c0 + cch * 8 <= cols - 8 ? c0 + cch * 8 : cols - 8;
  };
  uint32_t off[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) off[j] = (uint32_t)(((int64_t)krow * (j < NA ? lda : ldb) + col_of(j)) * 2);

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
    const char* ba = (const char*)(A + k0 * lda);
    const char* bb = PX ? ba : (const char*)(B + k0 * ldb);
    if (K - k0 >= 64) {
#pragma unroll
      for (int j = 0; j < PER; ++j) glds16_asm_so(j < NA ? ba : bb, off[j], stg + j * IMG + wid * 1024);
    } else {  // the reduction's last, partial step: token rows past K re-read row K-1 (zeroed in LDS)
      const int kv = (int)(K - k0);
      const int kk = krow < kv ? krow : kv - 1;
#pragma unroll
      for (int j = 0; j < PER; ++j)
        glds16_asm_so(j < NA ? ba : bb, (uint32_t)(((int64_t)kk * (j < NA ? lda : ldb) + col_of(j)) * 2),
                      stg + j * IMG + wid * 1024);
    }
  };
  // PX: this lane's pixel offset of its 8 columns in B image jb (step-invariant), and the token base
  typedef __attribute__((ext_vector_type(4))) float f4v;
  const int64_t plane = (int64_t)pg.H * pg.W;
  uint32_t coff[NB];
#pragma unroll
  for (int jb = 0; jb < NB; ++jb) {
    const int n = (int)n0 + jb * 64 + cch * 8;   // columns n .. n + 7: pixels j = n & 15 .. + 7 of one image row
    coff[jb] = PX ? (uint32_t)((((n >> 8) & 1) * pg.C + (n >> 9)) * plane + ((n >> 4) & 15) * pg.W + (n & 15)) : 0u;
  }
  auto tok_base = [&](int64_t m) -> int64_t {
    const int mi = (int)m;
    int b = (int)((float)mi * pg.inv_ntok);
    b -= b * pg.n_tok > mi;
    b += (b + 1) * pg.n_tok <= mi;
    const int n = mi - b * pg.n_tok;
    int fp = (int)((float)n * pg.inv_hpwp);
    fp -= fp * pg.HpWp > n;
    fp += (fp + 1) * pg.HpWp <= n;
    const int r = n - fp * pg.HpWp;
    int hp = (int)((float)r * pg.inv_wp);
    hp -= hp * pg.Wp > r;
    hp += (hp + 1) * pg.Wp <= r;
    const int wp = r - hp * pg.Wp;
    return ((int64_t)b * pg.F + 2 * fp) * pg.C * plane + (int64_t)(16 * hp) * pg.W + 16 * wp;
  };
  auto gather = [&](int s, f4v (&r)[2 * NB]) {
    const int64_t k0 = (int64_t)(ks0 + s) * 64;
    const int64_t m = k0 + krow < K ? k0 + krow : K - 1;   // rows past K: finite re-reads, zeroed in LDS
    const float* tb = px + tok_base(m);
#pragma unroll
    for (int jb = 0; jb < NB; ++jb) {
      const float* p = tb + coff[jb];
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[2 * jb]) : "v"(p) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(r[2 * jb + 1]) : "v"(p) : "memory");
    }
  };
  // after the counted wait: tie the registers to it (no use is scheduled above the wait), convert, store
  auto bwrite = [&](char* stg, f4v (&r)[2 * NB]) {
#pragma unroll
    for (int q = 0; q < 2 * NB; ++q) asm volatile("" : "+v"(r[q]));
#pragma unroll
    for (int jb = 0; jb < NB; ++jb) {
      uint4 u;
      u.x = (uint32_t)f2bf(r[2 * jb][0]) | ((uint32_t)f2bf(r[2 * jb][1]) << 16);
      u.y = (uint32_t)f2bf(r[2 * jb][2]) | ((uint32_t)f2bf(r[2 * jb][3]) << 16);
      u.z = (uint32_t)f2bf(r[2 * jb + 1][0]) | ((uint32_t)f2bf(r[2 * jb + 1][1]) << 16);
      u.w = (uint32_t)f2bf(r[2 * jb + 1][2]) | ((uint32_t)f2bf(r[2 * jb + 1][3]) << 16);
      *(uint4*)(stg + (NA + jb) * IMG + wid * 1024 + lane * 16) = u;
    }
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
      for (int j = 0; j < FJ; ++j) {
        const int cidx = cw * WN + j * 16;
        bfr[j] = dw_frag(stg + (NA + (cidx >> 6)) * IMG, cidx & 63, kk, lane);
      }
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
    for (int a = 0; a < NI; ++a)
      for (int o = tid * 16; o < bytes; o += 512 * 16) *(uint4*)(stg + a * IMG + kv * 128 + o) = make_uint4(0, 0, 0, 0);
  };
  auto stage_ptr = [&](int i) -> char* { return i == 0 ? st0 : i == 1 ? st1 : i == 2 ? st2 : st3; };
  auto step = [&](int s, auto sc) {
    constexpr int S = decltype(sc)::value;
    char* cur = stage_ptr(S);
    char* far = stage_ptr((S + NSTG - 1) % NSTG);  // the stage step s - 1 used
    if constexpr (PX) {
      // A of step s landed at the previous step's gather wait; only A of s + 1 may be in flight
      if (s + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // step s's images complete (B written last step); step s-1's stage free
      asm volatile("" ::: "memory");
      const int64_t k0 = (int64_t)(ks0 + s) * 64;
      if (K - k0 < 64) {
        zero_tail(cur, (int)(K - k0));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      f4v r[2 * NB];
      if (s + 1 < nk) gather(s + 1, r);
      if (s + 2 < nk) issue(s + 2, far);
      compute(cur);
      if (s + 1 < nk) {  // B of step s + 1: its loads, then (maybe) A of s + 2 are outstanding
        if (s + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bwrite(stage_ptr((S + 1) % NSTG), r);
      }
      return;
    }
    // steps s+1 .. s+NSTG-2 may stay in flight
    const int ahead = nk - 1 - s;
    if (NSTG >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (NSTG >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
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
  if constexpr (PX) {  // prologue: B of step 0 gathered and written, A of steps 0, 1 in flight
    f4v r[2 * NB];
    gather(0, r);
    issue(0, st0);
    if (nk > 1) {
      issue(1, st1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NA) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA) : "memory");
    }
    bwrite(st0, r);
  } else {
#pragma unroll
    for (int i = 0; i < NSTG - 1; ++i)
      if (i < nk) issue(i, stage_ptr(i));
  }
  for (int s = 0; s < nk; s += NSTG) {
    step(s, IC<0>{});
    if (s + 1 < nk) step(s + 1, IC<1 % NSTG>{});
    if (NSTG >= 3 && s + 2 < nk) step(s + 2, IC<2 % NSTG>{});
    if (NSTG >= 4 && s + 3 < nk) step(s + 3, IC<3 % NSTG>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float4* pt = (float4*)(part + ((int64_t)rem * g.splits + split) * (BM * BN));
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const f32x4 v = acc[i][j];
      pt[((rw * FI + i) * CF + cw * FJ + j) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
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
        float* so = sums + ((int64_t)nt * g.splits + split) * BN;
#pragma unroll
        for (int j = 0; j < FJ; ++j) so[cw * WN + j * 16 + lane] = sacc[j];
      }
    }
  }
}

// C (+)= sum over splits of the fragment-order partial tiles, many splits (the C2 shapes: 21-49).
// A workgroup owns 64 float4 of one tile (one per lane); wave w sums splits w, w+16, ... (four loads
// in flight each), then the 16 wave sums are added in wave order through LDS — a fixed order that
// depends only on the split count (bitwise reproducible).  Blocks after the tile blocks reduce the
// bias sums (8 loads in flight per thread).
template <int BM, int BN, bool TRANS>
__global__ __launch_bounds__(1024) void gemm_dw_reduce(const float* __restrict__ part, const float* __restrict__ sums,
                                                       DwGrid g, int64_t M, int64_t N, float* __restrict__ c,
                                                       int64_t ldc, float* __restrict__ bias_out, int64_t sum_len,
                                                       int sum_tiles, int sum_w) {
  constexpr int Q = BM * BN / 4;  // float4 per tile
  constexpr int CF = BN / 16;
  constexpr int NWR = 16;
  const int tiles = g.tiles_m * g.tiles_n;
  const int64_t blk = blockIdx.x;
  const int64_t tile_blocks = (int64_t)tiles * (Q / 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (blk < tile_blocks) {
    __shared__ float4 red[NWR][64];
    const int tile = (int)(blk / (Q / 64));
    const int q = (int)(blk % (Q / 64)) * 64 + lane;
    const float4* p = (const float4*)(part + (int64_t)tile * g.splits * (BM * BN)) + q;
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
    const int f = q >> 6, rf = f / CF, cf = f % CF;
    const int mt = tile / g.tiles_n, nt = tile % g.tiles_n;
    const int64_t n = (int64_t)nt * BN + cf * 16 + (lane & 15);
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
  for (; sp + 8 <= g.splits; sp += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(sp + u) * sum_w];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; sp < g.splits; ++sp) s += p[(int64_t)sp * sum_w];
  bias_out[e] += s;
}

// Few splits (S <= 8: ViT-Base's many output tiles leave one to three): one float4 of a tile per
// thread, the splits added in split order (a fixed order: bitwise reproducible).  Threads after the
// tile items reduce the bias sums.  TRANS: the kernel ran on swapped operands, so its tile element
// (m, n) is C[n][m] (the 4 consecutive m of a lane are then one float4 of C).
template <int BM, int BN, bool TRANS>
__global__ __launch_bounds__(256) void gemm_dw_reduce_few(const float* __restrict__ part, const float* __restrict__ sums,
                                                      DwGrid g, int64_t M, int64_t N, float* __restrict__ c,
                                                      int64_t ldc, float* __restrict__ bias_out, int64_t sum_len,
                                                      int sum_tiles, int sum_w) {
  constexpr int Q = BM * BN / 4;  // float4 per tile
  constexpr int CF = BN / 16;
  const int tiles = g.tiles_m * g.tiles_n;
  const int64_t item = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tile_items = (int64_t)tiles * Q;
  const int S = g.splits;
  if (item < tile_items) {
    const int tile = (int)(item / Q), q = (int)(item % Q), lane = q & 63;
    const float4* p = (const float4*)(part + (int64_t)tile * S * (BM * BN)) + q;
    float4 sum = p[0];
    int sp = 1;
    for (; sp + 8 <= S; sp += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(sp + u) * Q];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        sum.x += v[u].x; sum.y += v[u].y; sum.z += v[u].z; sum.w += v[u].w;
      }
    }
    for (; sp < S; ++sp) {
      const float4 o = p[(int64_t)sp * Q];
      sum.x += o.x; sum.y += o.y; sum.z += o.z; sum.w += o.w;
    }
    const int f = q >> 6, rf = f / CF, cf = f % CF;
    const int mt = tile / g.tiles_n, nt = tile % g.tiles_n;
    const int64_t n = (int64_t)nt * BN + cf * 16 + (lane & 15);
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
  const float* ps = sums + st * (int64_t)S * sum_w + off;
  float acc = 0.f;
  int sp = 0;
  for (; sp + 8 <= S; sp += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ps[(int64_t)(sp + u) * sum_w];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; sp < S; ++sp) acc += ps[(int64_t)sp * sum_w];
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
// Cost model (microseconds), fitted to rocprof durations of the C2 shapes: a launch pays ~10 us of
// fixed cost (dispatch, the prologue burst of every workgroup's first stages, the partial-tile store
// burst at the end, the reduce launch); a 64-token step costs ~0.25 us + 0.02 us per MFMA of a wave
// (0.49 us at 192 x 64, 0.73 us at 192 x 128), and the partial tiles cost ~0.3 us per MB (stored,
// then re-read by the reduce).  Splits keep >= 8 token steps each.  VS_KNOB_DW_BM / _BN / _SPLITS /
// _STAGES force a choice (A/B runs, tests).
DwPlan plan_dw(int64_t M, int64_t N, int64_t K) {
  DwPlan best = {};
  best.valid = false;
  const bool swap = M > N;
  const int64_t Ma = swap ? N : M, Nb = swap ? M : N;
  const int64_t nk = (K + 63) / 64;
  const int force_bm = knob(VS_KNOB_DW_BM), force_bn = knob(VS_KNOB_DW_BN);
  const int force_s = knob(VS_KNOB_DW_SPLITS), force_stg = knob(VS_KNOB_DW_STAGES);
  double best_t = 1e30;
  for (int BN : {64, 128}) {
    if (force_bn && BN != force_bn) continue;
    if (!force_bn && BN > 64 && Nb <= 64) continue;
    for (int BM : {64, 128, 192}) {
      if (force_bm && BM != force_bm) continue;
      const int stage = (BM + BN) / 64 * 8192;
      int nstg = 4 * stage <= 131072 ? 4 : 3;
      if (force_stg == 3 || (force_stg == 4 && 4 * stage <= 131072)) nstg = force_stg;
      const int per_cu = nstg * stage <= 81920 ? 2 : 1;
      const int slots = 256 * per_cu;
      const int64_t tm = (Ma + BM - 1) / BM, tn = (Nb + BN - 1) / BN, tiles = tm * tn;
      int64_t S = force_s > 0 ? force_s : slots / tiles;
      if (S < 1) S = 1;
      const int64_t smax = nk / 8 > 0 ? nk / 8 : 1;
      if (S > smax) S = smax;
      int64_t kps = (nk + S - 1) / S;
      S = (nk + kps - 1) / kps;
      const int64_t wgs = tiles * S;
      const double rounds = (double)((wgs + slots - 1) / slots);
      const double t_step = (0.25 + 0.02 * (BM * BN / 1024)) * per_cu;
      const double part = (double)wgs * BM * BN * 4.0;
      double t = 10.0 + rounds * (double)kps * t_step + 0.3 * part / 1e6;
      // rows / columns of the last tiles past the operands cost their share of the stream
      const double waste = 1.0 - (double)(Ma * Nb) / (double)(tm * BM * tn * BN);
      t *= 1.0 + 0.5 * waste;
      if (t < best_t) {
        best_t = t;
        best.valid = true;
        best.swap = swap;
        best.BM = BM;
        best.BN = BN;
        best.stages = nstg;
        best.g.tiles_m = (int)tm;
        best.g.tiles_n = (int)tn;
        best.g.splits = (int)S;
        best.g.ksteps = (int)kps;
        best.part_floats = wgs * BM * BN;
        best.sum_floats = S * (tm * BM > tn * BN ? tm * BM : tn * BN);
      }
    }
  }
  return best;
}

size_t dw_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const DwPlan p = plan_dw(M, N, K);
  if (!p.valid) return 0;
  return (size_t)(p.part_floats + p.sum_floats + 64) * 4;
}

template <int BM, int BN, int SUMS, bool TRANS, bool PX = false>
static void launch_dw_t(const bf16_t* a, int64_t lda, int64_t Ma, const bf16_t* b, int64_t ldb, int64_t Nb, int64_t K,
                        const DwPlan& p, float* part, float* sums, float* c, int64_t ldc, float* bias, hipStream_t s,
                        const float* px = nullptr, const PatchDwGeo& pg = PatchDwGeo{}) {
  const unsigned nwg = (unsigned)(p.g.tiles_m * p.g.tiles_n * p.g.splits);
  if constexpr ((BM + BN) / 64 * 8192 * 4 <= 131072) {
    if (!PX && p.stages == 4) {
      hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, SUMS, 4>), dim3(nwg), dim3(512), 0, s, a, lda, Ma, b, ldb, Nb, K, p.g,
                         part, sums, px, pg);
    } else {
      hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, SUMS, 3, PX>), dim3(nwg), dim3(512), 0, s, a, lda, Ma, b, ldb, Nb, K,
                         p.g, part, sums, px, pg);
    }
  } else {
    hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, SUMS, 3, PX>), dim3(nwg), dim3(512), 0, s, a, lda, Ma, b, ldb, Nb, K, p.g,
                       part, sums, px, pg);
  }
  const int tiles = p.g.tiles_m * p.g.tiles_n;
  int64_t sum_len = 0, sum_w = 1;
  int sum_tiles = 0;
  if (SUMS == 1) {
    sum_w = BM;
    sum_tiles = p.g.tiles_m;
    sum_len = Ma;
  } else if (SUMS == 2) {
    sum_w = BN;
    sum_tiles = p.g.tiles_n;
    sum_len = Nb;
  }
  // C is [M][N] of the ORIGINAL product: with TRANS the kernel's (m, n) = (original n, original m)
  if (p.g.splits <= 8) {
    const int64_t items = (int64_t)tiles * (BM * BN / 4) + sum_len;
    hipLaunchKernelGGL((gemm_dw_reduce_few<BM, BN, TRANS>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s,
                       part, sums, p.g, Ma, Nb, c, ldc, bias, sum_len, sum_tiles, (int)sum_w);
    return;
  }
  const int64_t blocks = (int64_t)tiles * (BM * BN / 256) + (sum_len + 1023) / 1024;
  hipLaunchKernelGGL((gemm_dw_reduce<BM, BN, TRANS>), dim3((unsigned)blocks), dim3(1024), 0, s, part, sums, p.g, Ma, Nb,
                     c, ldc, bias, sum_len, sum_tiles, (int)sum_w);
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
#define DW_(BM_, BN_, S_, T_) launch_dw_t<BM_, BN_, S_, T_>(aa, la, Ma, bb, lb, Nb, d->K, p, part, sums, c, d->ldc, bias, s)
#define DW_BM(BM_, BN_)                             \
  do {                                              \
    if (p.swap) {                                   \
      if (sm == 2) DW_(BM_, BN_, 2, true);          \
      else DW_(BM_, BN_, 0, true);                  \
    } else {                                        \
      if (sm == 1) DW_(BM_, BN_, 1, false);         \
      else DW_(BM_, BN_, 0, false);                 \
    }                                               \
  } while (0)
#define DW_BN(BM_)                   \
  do {                               \
    if (p.BN == 128) DW_BM(BM_, 128); \
    else DW_BM(BM_, 64);             \
  } while (0)
  if (p.BM == 64) DW_BN(64);
  else if (p.BM == 128) DW_BN(128);
  else DW_BN(192);
#undef DW_BN
#undef DW_BM
#undef DW_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

int launch_patch_dw(const bf16_t* dx, int64_t lddx, int64_t D, const float* px, const PatchDwGeo& pg, int64_t tokens,
                    int64_t K, float* dw, int64_t ldw, float* db, float* ws, hipStream_t s) {
  const DwPlan p = plan_dw(D, K, tokens);
  VS_REQUIRE(p.valid && !p.swap && K % p.BN == 0, "vs_patch_embed_dw: no gather dW plan for this shape");
  float* part = ws;
  float* sums = part + p.part_floats;
#define PD_(BM_, BN_)                                                                                               \
  do {                                                                                                            \
    if (db) launch_dw_t<BM_, BN_, 1, false, true>(dx, lddx, D, nullptr, 0, K, tokens, p, part, sums, dw, ldw, db, s, \
                                                  px, pg);                                                        \
    else launch_dw_t<BM_, BN_, 0, false, true>(dx, lddx, D, nullptr, 0, K, tokens, p, part, sums, dw, ldw, db, s,    \
                                               px, pg);                                                           \
  } while (0)
  if (p.BM == 64) { if (p.BN == 128) PD_(64, 128); else PD_(64, 64); }
  else if (p.BM == 128) { if (p.BN == 128) PD_(128, 128); else PD_(128, 64); }
  else { if (p.BN == 128) PD_(192, 128); else PD_(192, 64); }
#undef PD_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

}  // namespace vs
