// gemm.hip — MFMA GEMM with fused epilogues (vs_gemm).
//
// Replaces the nn.Linear / F.linear / Conv3d(as im2col) kernels of the reference hot path and
// their autograd backward (see include/vspike.h for the per-call-site citations).
//
// bf16 operands: v_mfma_f32_16x16x32_bf16, block tile BM x BN x 64, 4 waves in 2x2, each wave
//   (BM/2) x (BN/2).  Operands are staged global -> registers -> LDS (double-buffered, loads for
//   tile t+1 issued before the MFMAs of tile t).  LDS images:
//     K-contiguous operand:  [rows][64 k] 128-B rows, 16-B chunk XOR (row>>1)&7  -> ds_read_b128
//     M/N-contiguous operand: [64 k][rows] rows, chunk XOR f(k)                 -> ds_read_tr16_b64
//   so the transposed products of the backward (dW = dY^T X, dX = dY W) need no transpose pass.
// f32 operands: v_mfma_f32_16x16x4_f32 (exact f32 fma chain), tile 64x64x32, [k][rows] images.
// Epilogue: the accumulator tile is staged through LDS (f32, padded rows) and written back in
//   row order, 8 consecutive columns per thread: every bias/pos/residual/aux read and every output
//   store is a 16-B vector access (the shapes here — M = 25,088 tokens, K = 192..768 — are
//   HBM-bound on their outputs; the first version's 2-4 B scattered stores were 5-9x off that
//   bound, profiles/r01_v0_kernel_stats.csv).  Split-K (VS_EPI_ATOMIC) adds whole 256-B rows.
// Grid: 1-D, tiles remapped so that consecutive tiles of one XCD (blockIdx % 8 group) share the
//   A row-panel / the same K slice (bijective remap, cdna_hip_programming.md §5 T1).
#include <cstdlib>

#include "common.h"
#include "gemm_common.h"
#include "gemm_dw.h"

namespace vs {

// Stage a BM x BN f32 tile (16x16-MFMA C layout in `acc`) through LDS and apply the epilogue in
// row order.  PARTS = 2 stages the two 64-row halves one after the other (the waves of row block
// wr write in pass wr), halving the staging LDS; `lds` must hold (BM/PARTS)*(BN+4) floats.
template <int BM, int BN, int TM, int TN, uint32_t EF, int PARTS = 1>
__device__ __forceinline__ void store_tile(const EpiParams& e, float* lds, const f32x4 (&acc)[TM][TN], int64_t m0,
                                           int64_t n0, int split) {
  static_assert(PARTS == 1 || (PARTS == 2 && BM / 2 == BM / 2 / 16 * 16), "row halves");
  const bool first_split = split == 0;
  const uint32_t F = epi_flags<EF>(e);
  constexpr int LDT = BN + 4;  // +4 floats: 16-B aligned rows, conflict-free scalar writes
  constexpr int WM = BM / 2, WN = BN / 2, RB = BM / PARTS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  constexpr int CPR = BN / 8;        // 8-column groups per row
  constexpr int RPP = 256 / CPR;     // rows per pass
  const int cg = tid % CPR;
  const int64_t n = n0 + cg * 8;     // a thread keeps its column group in every pass
  const bool vec = e.vec_ok && n + 8 <= e.N;
  float bias8[8];
  if ((F & VS_EPI_BIAS) && vec && !(F & VS_EPI_ATOMIC) && !e.part) ld8(e.bias, n, 0, bias8);
#pragma unroll
  for (int part = 0; part < PARTS; ++part) {
    const int64_t mp = m0 + part * RB;  // first output row of this pass
    __syncthreads();
    if (PARTS == 1 || wr == part) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            lds[(wr * WM - part * RB + i * 16 + (lane >> 4) * 4 + r) * LDT + wc * WN + j * 16 + (lane & 15)] =
                acc[i][j][r] * e.alpha;
    }
    __syncthreads();
    if (e.part) {
      // split-K partial: plain 16-B stores of this split's tile (gemm_splitk_reduce adds the splits)
      float* pbase = e.part + (int64_t)split * e.M * e.N;
      constexpr int C4 = BN / 4;
      for (int idx = tid; idx < RB * C4; idx += 256) {
        const int rr = idx / C4, c4 = idx % C4;
        const int64_t m = mp + rr, nn = n0 + 4 * c4;
        if (m < e.M && nn < e.N) {
          const float* src = lds + rr * LDT + 4 * c4;
          if (nn + 4 <= e.N && (e.N & 3) == 0) {
            *(float4*)(pbase + m * e.N + nn) = *(const float4*)src;
          } else {
            for (int k = 0; k < 4 && nn + k < e.N; ++k) pbase[m * e.N + nn + k] = src[k];
          }
        }
      }
      continue;
    }
    if (F & VS_EPI_ATOMIC) {
      // one column per lane: a wave adds 64 consecutive floats (256 B) of a row per instruction
      for (int idx = tid; idx < RB * BN; idx += 256) {
        const int rr = idx / BN, cc = idx % BN;
        const int64_t m = mp + rr, nn = n0 + cc;
        if (m < e.M && nn < e.N) {
          float v = lds[rr * LDT + cc];
          if ((F & VS_EPI_BIAS) && first_split) v += e.bias[nn];
          unsafeAtomicAdd((float*)e.c + m * e.ldc + nn, v);
        }
      }
      continue;
    }
    if (n >= e.N) continue;
    if (vec) {
      // per-column constants loaded once, all row passes unrolled: their LDS reads, operand loads
      // and stores overlap (the rolled loop paid one global-load latency per pass: ~5.5k of a
      // ~10k-cycle K = 192 tile, scripts/stamp_gemm.py)
#pragma unroll
      for (int p = 0; p < RB / RPP; ++p) {
        const int rr = tid / CPR + p * RPP;
        const int64_t m = mp + rr;
        if (m < e.M) {
          const float* src = lds + rr * LDT + cg * 8;
          float v[8];
          const float4 a = *(const float4*)src;
          const float4 b = *(const float4*)(src + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
          if (F & VS_EPI_BIAS) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += bias8[k];
          }
          epi_eight<EF>(e, m, n, v, true);
        }
      }
    } else {
      for (int rr = tid / CPR; rr < RB; rr += RPP) {
        const int64_t m = mp + rr;
        if (m >= e.M) break;
        const float* src = lds + rr * LDT + cg * 8;
        for (int k = 0; k < 8 && n + k < e.N; ++k) epi_one<EF>(e, m, n + k, src[k]);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// bf16 kernel
// ----------------------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ int swz_mc(int k) {  // chunk XOR for [k][R] images (R = 128 or 64)
  if constexpr (R == 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}
__device__ __forceinline__ int swz_kc(int r) { return (r >> 1) & 7; }

template <int R, bool KC>
struct OperandBf16 {
  static constexpr int BK = 64;
  static constexpr int BYTES = R * BK * 2;
  static constexpr int CHUNKS = R * BK / 8 / 256;  // 16-B chunks per thread per tile

  __device__ __forceinline__ static void load(uint4 (&reg)[CHUNKS], const bf16_t* __restrict__ p, int64_t ld,
                                              int64_t r0, int64_t rows, int64_t k0, int64_t k_end, int tid) {
#pragma unroll
    for (int s = 0; s < CHUNKS; ++s) {
      const int i = tid + 256 * s;
      int64_t gr, gk;
      if constexpr (KC) {
        gr = r0 + (i >> 3);
        gk = k0 + (i & 7) * 8;
      } else {
        gk = k0 + i / (R / 8);
        gr = r0 + (i % (R / 8)) * 8;
      }
      const bool ok = gr < rows && gk < k_end;
      const bf16_t* src = KC ? p + gr * ld + gk : p + gk * ld + gr;
      reg[s] = ok ? *(const uint4*)src : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ static void store(char* lds, const uint4 (&reg)[CHUNKS], int tid) {
#pragma unroll
    for (int s = 0; s < CHUNKS; ++s) {
      const int i = tid + 256 * s;
      int off;
      if constexpr (KC) {
        const int r = i >> 3, c = i & 7;
        off = r * 128 + ((c ^ swz_kc(r)) << 4);
      } else {
        const int k = i / (R / 8), c = i % (R / 8);
        off = k * (R * 2) + ((c ^ swz_mc<R>(k)) << 4);
      }
      *(uint4*)(lds + off) = reg[s];
    }
  }
  // LDS-DMA fill of the same image (global_load_lds_dwordx4, 1-KiB pieces, the XOR swizzle moved
  // to the per-lane source chunk): wave `wid` issues pieces wid*PPW .. +PPW.  Rows / columns past
  // `rows` re-read the last valid ones (their outputs are never stored); k must be in range.
  static constexpr int PIECES = BYTES / 1024, PPW = PIECES / 4;
  template <bool ASM = false>
  __device__ __forceinline__ static void dma(char* lds, const bf16_t* __restrict__ p, int64_t ld, int64_t r0,
                                             int64_t rows, int64_t k0, int wid, int lane) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pi = wid * PPW + j;
      const bf16_t* src;
      if constexpr (KC) {
        const int r = pi * 8 + (lane >> 3), c = (lane & 7) ^ swz_kc(r);
        const int64_t gr = r0 + r < rows ? r0 + r : rows - 1;
        src = p + gr * ld + k0 + c * 8;
      } else if constexpr (R == 128) {
        const int k = pi * 4 + (lane >> 4), c = (lane & 15) ^ swz_mc<R>(k);
        const int64_t gc = r0 + c * 8 <= rows - 8 ? r0 + c * 8 : rows - 8;
        src = p + (k0 + k) * ld + gc;
      } else {
        const int k = pi * 8 + (lane >> 3), c = (lane & 7) ^ swz_mc<R>(k);
        const int64_t gc = r0 + c * 8 <= rows - 8 ? r0 + c * 8 : rows - 8;
        src = p + (k0 + k) * ld + gc;
      }
      if constexpr (ASM) glds16_asm(src, lds + pi * 1024);
      else glds16(src, lds + pi * 1024);
    }
  }
  // the same fill issued by NW waves (8-wave kernels)
  template <int NW>
  __device__ __forceinline__ static void dma_nw(char* lds, const bf16_t* __restrict__ p, int64_t ld, int64_t r0,
                                                int64_t rows, int64_t k0, int wid, int lane) {
    static_assert(PIECES % NW == 0, "whole pieces per wave");
#pragma unroll
    for (int j = 0; j < PIECES / NW; ++j) {
      const int pi = wid * (PIECES / NW) + j;
      const bf16_t* src;
      if constexpr (KC) {
        const int r = pi * 8 + (lane >> 3), c = (lane & 7) ^ swz_kc(r);
        const int64_t gr = r0 + r < rows ? r0 + r : rows - 1;
        src = p + gr * ld + k0 + c * 8;
      } else if constexpr (R == 128) {
        const int k = pi * 4 + (lane >> 4), c = (lane & 15) ^ swz_mc<R>(k);
        const int64_t gc = r0 + c * 8 <= rows - 8 ? r0 + c * 8 : rows - 8;
        src = p + (k0 + k) * ld + gc;
      } else {
        const int k = pi * 8 + (lane >> 3), c = (lane & 7) ^ swz_mc<R>(k);
        const int64_t gc = r0 + c * 8 <= rows - 8 ? r0 + c * 8 : rows - 8;
        src = p + (k0 + k) * ld + gc;
      }
      glds16_asm(src, lds + pi * 1024);
    }
  }
  // fragment of rows [rb, rb+16) for the 32-deep k step kk (0/1): lane holds rows rb+(lane&15),
  // k = 32kk + 8(lane>>4) + 0..7.
  __device__ __forceinline__ static bf16x8 frag(const char* lds, int rb, int kk, int lane) {
    if constexpr (KC) {
      const int r = rb + (lane & 15);
      const int c = kk * 4 + (lane >> 4);
      return *(const bf16x8*)(lds + r * 128 + ((c ^ swz_kc(r)) << 4));
    } else {
      const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
      const int col = rb + p4;
      const int k0 = kk * 32 + 8 * (lane >> 4) + q;
      const int k1 = k0 + 4;
      const int off0 = k0 * (R * 2) + (((col >> 3) ^ swz_mc<R>(k0)) << 4) + (col & 7) * 2;
      const int off1 = k1 * (R * 2) + (((col >> 3) ^ swz_mc<R>(k1)) << 4) + (col & 7) * 2;
      short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(lds + off0));
      short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(lds + off1));
      typedef __attribute__((ext_vector_type(8))) short short8v;
      short8v s = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
      return __builtin_bit_cast(bf16x8, s);
    }
  }
};

template <int A, int B>
struct CMax {
  static constexpr int v = A > B ? A : B;
};

template <int BM, int BN, bool AKC, bool BKC, uint32_t EF>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb, int64_t K,
                                                           GridMap g, EpiParams e) {
  using OA = OperandBf16<BM, AKC>;
  using OB = OperandBf16<BN, BKC>;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int SMEM = CMax<2 * STAGE, BM*(BN + 4) * 4>::v;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  int nt, mt, split;
  map_block(g, nt, mt, split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * BN;
  const int64_t k_begin = (int64_t)split * g.k_per_split;
  const int64_t k_end = k_begin + g.k_per_split < K ? k_begin + g.k_per_split : K;
  const int nk = (int)((k_end - k_begin + 63) / 64);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused bias gradient: only the first column tile's wc == 0 waves (wave-uniform condition)
  const bool rowsum_on = e.a_rowsum != nullptr && nt == 0 && wc == 0;
  float rs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) rs[i] = 0.f;

  uint4 ra[OA::CHUNKS], rb[OB::CHUNKS];
  if (nk > 0) {
    OA::load(ra, A, lda, m0, e.M, k_begin, k_end, tid);
    OB::load(rb, B, ldb, n0, e.N, k_begin, k_end, tid);
    OA::store(smem, ra, tid);
    OB::store(smem + OA::BYTES, rb, tid);
  }
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const char* sa = smem + (t & 1) * STAGE;
    const char* sb = sa + OA::BYTES;
    const bool more = t + 1 < nk;
    if (more) {
      const int64_t kn = k_begin + (int64_t)(t + 1) * 64;
      OA::load(ra, A, lda, m0, e.M, kn, k_end, tid);
      OB::load(rb, B, ldb, n0, e.N, kn, k_end, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = OA::frag(sa, wr * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = OB::frag(sb, wc * WN + j * 16, kk, lane);
      if (rowsum_on) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q) rs[i] += (float)af[i][q];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* dst = smem + ((t + 1) & 1) * STAGE;
      OA::store(dst, ra, tid);
      OB::store(dst + OA::BYTES, rb, tid);
    }
    __syncthreads();
  }
  if (rowsum_on) flush_rowsum<TM>(e.a_rowsum, rs, m0 + wr * WM, e.M, lane);
  store_tile<BM, BN, TM, TN, EF>(e, (float*)smem, acc, m0, n0, split);
}

// ----------------------------------------------------------------------------------------------
// bf16, whole K in LDS (K = 64 * KT <= 256, no split): the skinny projections of the ViT block
// (K = D = 192, and the N = 192 dX products of the attention/MLP inputs).  With only 3 k-steps the
// register-staged pipeline above pays one global-load latency per k-step; here every k-step of A
// and B is DMA'd into LDS in one burst (global_load_lds, no staging registers), one wait, one
// barrier, then all MFMAs and the epilogue — one latency per tile, and 2 blocks per CU overlap
// one block's loads with the other's MFMAs and stores.
// ----------------------------------------------------------------------------------------------
#ifdef VS_STAMP
// diagnostic build only: per-wave shader-clock phase marks of the whole-K kernel (vs_dbg_gstamps)
__device__ unsigned long long g_gstamp[8 * 8192];
#define VS_GMARK(slot)                                                                        \
  do {                                                                                        \
    const int w_ = blockIdx.x * 4 + (threadIdx.x >> 6);                                       \
    if ((threadIdx.x & 63) == 0 && w_ < 8192) g_gstamp[8 * w_ + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define VS_GMARK(slot)
#endif

template <int BM, int BN, int KT, bool AKC, bool BKC, uint32_t EF>
__global__ __launch_bounds__(256, 2) void gemm_bf16_fullk_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                 const bf16_t* __restrict__ B, int64_t ldb,
                                                                 GridMap g, EpiParams e) {
  using OA = OperandBf16<BM, AKC>;
  using OB = OperandBf16<BN, BKC>;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int SMEM = CMax<KT * (OA::BYTES + OB::BYTES), BM*(BN + 4) * 4>::v;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  VS_GMARK(0);
  int nt, mt, split;
  map_block(g, nt, mt, split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * BN;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    OA::dma(smem + t * OA::BYTES, A, lda, m0, e.M, t * 64, wid, lane);
    OB::dma(smem + KT * OA::BYTES + t * OB::BYTES, B, ldb, n0, e.N, t * 64, wid, lane);
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  VS_GMARK(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  VS_GMARK(2);
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const char* sa = smem + t * OA::BYTES;
    const char* sb = smem + KT * OA::BYTES + t * OB::BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = OA::frag(sa, wr * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = OB::frag(sb, wc * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  (void)split;
  VS_GMARK(3);
  store_tile<BM, BN, TM, TN, EF>(e, (float*)smem, acc, m0, n0, 0);
  VS_GMARK(4);
#ifdef VS_STAMP
  if ((threadIdx.x & 63) == 0) {
    const int w_ = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w_ < 8192) {
      g_gstamp[8 * w_ + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_gstamp[8 * w_ + 6] = __builtin_amdgcn_s_memrealtime();
    }
  }
#endif
}

// ----------------------------------------------------------------------------------------------
// bf16, long K (K % 64 == 0): 3-stage LDS-DMA ring.  Step t+2 is DMA'd while step t computes, and
// a counted vmcnt keeps step t+1 in flight across each barrier (raw s_barrier: __syncthreads()
// would wait vmcnt(0) and drain it).  The three stages are separate __shared__ objects, the loop
// is unrolled by 3 so every stage index is a constant: alias analysis then keeps hipcc from
// draining the ring before each step's LDS reads.  The register-staged kernel above had one
// global-load latency exposed per 64-deep step.  Epilogue staged in two row halves (72 KB of LDS
// for 128 x 64: 2 blocks per CU).
// ----------------------------------------------------------------------------------------------
template <int BM, int BN, bool AKC, bool BKC, uint32_t EF>
__global__ __launch_bounds__(256, 2) void gemm_bf16_ring_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                const bf16_t* __restrict__ B, int64_t ldb, int64_t K,
                                                                GridMap g, EpiParams e) {
  using OA = OperandBf16<BM, AKC>;
  using OB = OperandBf16<BN, BKC>;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int S0 = CMax<STAGE, (BM / 2) * (BN + 4) * 4>::v;
  constexpr int PER = OA::PPW + OB::PPW;  // DMA wave-instructions per k-step
  __shared__ __attribute__((aligned(16))) char st0[S0];
  __shared__ __attribute__((aligned(16))) char st1[STAGE];
  __shared__ __attribute__((aligned(16))) char st2[STAGE];

  int nt, mt, split;
  map_block(g, nt, mt, split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * BN;
  const int64_t k_begin = (int64_t)split * g.k_per_split;
  const int64_t k_end = k_begin + g.k_per_split < K ? k_begin + g.k_per_split : K;
  const int nk = (int)((k_end - k_begin) / 64);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool rowsum_on = e.a_rowsum != nullptr && nt == 0 && wc == 0;
  float rs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) rs[i] = 0.f;

  auto issue = [&](int t, char* st) {
    const int64_t k0 = k_begin + (int64_t)t * 64;
    OA::template dma<true>(st, A, lda, m0, e.M, k0, wid, lane);
    OB::template dma<true>(st + OA::BYTES, B, ldb, n0, e.N, k0, wid, lane);
  };
  auto compute = [&](const char* sa) {
    const char* sb = sa + OA::BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = OA::frag(sa, wr * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = OB::frag(sb, wc * WN + j * 16, kk, lane);
      if (rowsum_on) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q) rs[i] += (float)af[i][q];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  auto step = [&](int t, auto sc) {
    constexpr int S = decltype(sc)::value;
    const char* cur = S == 0 ? st0 : (S == 1 ? st1 : st2);
    char* far = S == 0 ? st2 : (S == 1 ? st0 : st1);  // stage of step t + 2
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");  // step t landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's step-t pieces landed; step t-1's stage is free
    asm volatile("" ::: "memory");
    if (t + 2 < nk) issue(t + 2, far);
    compute(cur);
  };
  if (nk > 0) issue(0, st0);
  if (nk > 1) issue(1, st1);
  for (int t = 0; t < nk; t += 3) {
    step(t, IC<0>{});
    if (t + 1 < nk) step(t + 1, IC<1>{});
    if (t + 2 < nk) step(t + 2, IC<2>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the asm DMA is invisible to hipcc's own waits)
  if (rowsum_on) flush_rowsum<TM>(e.a_rowsum, rs, m0 + wr * WM, e.M, lane);
  store_tile<BM, BN, TM, TN, EF, 2>(e, (float*)st0, acc, m0, n0, split);
}

// ----------------------------------------------------------------------------------------------
// bf16 row-panel kernel for K <= 192 (the ViT block's K = D projections and dX products:
// qkv, proj, fc1 + GELU, do, da * GELU').  These shapes are HBM-bound on the activations they
// write (M = 25,088 tokens x N = 192..768 columns); the per-tile kernels above re-read the A panel
// once per 64-column tile (12x for fc1) and pay one load latency per tile.  Here a persistent
// workgroup owns a contiguous range of (128-row panel, 64-column chunk) items, panel-major:
//   * A: each wave keeps its 32 rows x K of the panel in registers as MFMA fragments (loaded from
//     global once per panel, 48 VGPRs at K = 192) — A is read from HBM about once;
//   * W: the 64 x K chunk of the weight (L2-resident) is register-staged: its global loads for
//     chunk i+1 are in flight while chunk i computes, then written into one LDS image between two
//     barriers (guide T14);
//   * epilogue: each wave stages its 32 x 64 f32 tile in a wave-private LDS image and writes it
//     in the NEXT item's iteration (after the next chunk's loads are issued), whole 8-column
//     groups per lane with 16-B accesses (bias, GELU, GELU', residual fused as elsewhere).
// Grid = min(items, 2 workgroups x 256 CUs): one round, every CU busy, 2 workgroups per CU
// overlap one's epilogue stores with the other's MFMAs.
// ----------------------------------------------------------------------------------------------
template <int KT, bool BKC, uint32_t EF>
__global__ __launch_bounds__(256, 2) void gemm_bf16_panel_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                 const bf16_t* __restrict__ B, int64_t ldb,
                                                                 int64_t items, EpiParams e) {
  using OB = OperandBf16<64, BKC>;
  constexpr int KS = 2 * KT;           // 32-deep MFMA k-steps
  constexpr int LDT = 64 + 4;          // staging row stride (floats)
  __shared__ __attribute__((aligned(16))) char wimg[KT * OB::BYTES];
  __shared__ __attribute__((aligned(16))) float stage[4][32 * LDT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t chunks = e.N / 64;
  const int64_t G = gridDim.x;
  const int64_t it0 = (int64_t)blockIdx.x * items / G, it1 = ((int64_t)blockIdx.x + 1) * items / G;
  if (it0 >= it1) return;
  VS_GMARK(0);
#ifdef VS_STAMP
  if ((threadIdx.x & 63) == 0 && blockIdx.x * 4 + (threadIdx.x >> 6) < 8192)
    g_gstamp[8 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 7] = __builtin_amdgcn_s_memrealtime();
#endif

  bf16x8 af[2][KS];
  auto load_a = [&](int64_t panel) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int64_t r = panel * 128 + wid * 32 + i * 16 + (lane & 15);
      r = r < e.M ? r : e.M - 1;  // rows past M: finite data, never stored
      const bf16_t* p = A + r * lda + 8 * (lane >> 4);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[i][ks] = *(const bf16x8*)(p + 32 * ks);
    }
  };
  uint4 wreg[KT][OB::CHUNKS];
  auto load_w = [&](int64_t chunk) {
#pragma unroll
    for (int t = 0; t < KT; ++t) OB::load(wreg[t], B, ldb, chunk * 64, e.N, t * 64, KT * 64, tid);
  };
  float* st = stage[wid];
  auto stage_acc = [&](const f32x4 (&acc)[2][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[(i * 16 + (lane >> 4) * 4 + r) * LDT + j * 16 + (lane & 15)] = acc[i][j][r] * e.alpha;
  };
  // epilogue of a staged item: lane -> rows (lane >> 3) + 8p, 8-column group lane & 7
  auto epilogue = [&](int64_t item) {
    const int64_t m0 = (item / chunks) * 128 + wid * 32, n = (item % chunks) * 64 + (lane & 7) * 8;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rr = p * 8 + (lane >> 3);
      const int64_t m = m0 + rr;
      if (m < e.M) {
        const float* src = st + rr * LDT + (lane & 7) * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_eight<EF>(e, m, n, v, false);
      }
    }
  };

  int64_t panel = it0 / chunks;
  load_a(panel);
  load_w(it0 % chunks);
  for (int64_t it = it0; it < it1; ++it) {
    __syncthreads();  // every wave is done reading the W image of the previous item
#pragma unroll
    for (int t = 0; t < KT; ++t) OB::store(wimg + t * OB::BYTES, wreg[t], tid);
    __syncthreads();  // W image of item `it` complete
    if (it == it0) VS_GMARK(1);
    if (it + 1 < it1) load_w((it + 1) % chunks);  // in flight under this item's MFMAs
    if (it > it0) epilogue(it - 1);              // previous item's staged tile (wave-private)
    if (it / chunks != panel) {
      panel = it / chunks;
      load_a(panel);
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = OB::frag(wimg + (ks >> 1) * OB::BYTES, j * 16, ks & 1, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bfr[j], acc[i][j], 0, 0, 0);
    }
    stage_acc(acc);
    if (it == it0) VS_GMARK(2);
  }
  VS_GMARK(3);
  epilogue(it1 - 1);
  VS_GMARK(4);
#ifdef VS_STAMP
  if ((threadIdx.x & 63) == 0) {
    const int w_ = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w_ < 8192) {
      g_gstamp[8 * w_ + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_gstamp[8 * w_ + 6] = __builtin_amdgcn_s_memrealtime();
    }
  }
#endif
}

// ----------------------------------------------------------------------------------------------
// bf16 row-slab kernel for N <= 192 (the ViT block's D-wide outputs: proj + residual, fc2 +
// residual, and the dX products do, dh2, dh1).  With 128 x 64 tiles these shapes make 588 tiles
// for 512 resident slots (2 per CU): two rounds, the second a quarter full.  Here the grid is
// exactly min(512, M/16) workgroups and workgroup g owns the contiguous rows [g M / G, (g+1) M / G)
// (49 at the bench) and ALL N columns, so every CU carries the same work in one round:
//   * one 64-row tile covers the slab (rows past the slab re-read its last row, never stored, so
//     no HBM byte is fetched twice); the W operand (N x 64 per k-step, L2-resident) is re-read by
//     every workgroup from L2;
//   * 2-stage LDS-DMA ring over 64-deep k-steps (asm DMA, counted vmcnt + raw barrier, as the ring
//     kernel): step t+1 is in flight while step t computes; 2 workgroups per CU (64 KB each);
//   * 4 waves in 2 x 2, wave tile 32 x (N / 2);
//   * epilogue: the f32 tile is staged through the ring's LDS, each thread takes 2 NT 8-column
//     groups, every bias / residual load of the thread issued before its first store.
// Slabs longer than 64 rows (M > 32,768) are processed as consecutive 64-row tiles.
// ----------------------------------------------------------------------------------------------
// LayerNorm backward fused into the slab kernel's epilogue (vs_gemm_ln_bwd): the product is dh,
// the gradient w.r.t. the LN output; every workgroup owns whole rows, so the row reductions of
// LN' run on the staged tile and dh never reaches HBM.
struct LnBwdParams {
  const float* x;      // LN input rows
  int64_t ldx;
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* dres;   // residual gradient added to dx (or null)
  int64_t ldr;
  float* dx;
  int64_t lddx;
  bf16_t* dx_lp;       // optional bf16 copy of dx (next GEMM operand)
  float* part;         // [gridDim.x][2][N] dgamma / dbeta partial rows (ln_partsum adds them)
  // LayerNorm FORWARD fused into the epilogue (vs_gemm_ln_fwd): y = v + bias + residual is stored
  // (e.c, f32) and normalised: h = (y - mean) rstd gamma + beta (bf16), mean / rstd per row
  const float* beta;
  float eps;
  bf16_t* h;
  int64_t ldh;
  float* mean_out;
  float* rstd_out;
};

template <int NT, bool BKC, uint32_t EF, bool LNB = false, bool LNF = false, int WV = 4>
__global__ __launch_bounds__(64 * WV, 2) __attribute__((amdgpu_waves_per_eu(WV / 2, WV / 2))) void gemm_bf16_slab_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                const bf16_t* __restrict__ B, int64_t ldb, int64_t K,
                                                                EpiParams e, LnBwdParams ln) {
  // WV = 4: 64-row tiles (2 x 2 waves); WV = 8: 128-row tiles (4 x 2 waves, 2 workgroups = 16 waves
  // per CU): the W slice of a k-step (N x 64, L2) is streamed once per 128 rows instead of per 64
  constexpr int RT = 16 * WV, NTH = 64 * WV, PR = NTH / 16;  // tile rows, threads, LN' rows per pass
  using OA = OperandBf16<RT, true>;
  using OB = OperandBf16<64, BKC>;
  constexpr int N = 64 * NT, TM = 2, TN = NT * 2, WN = N / 2;
  constexpr int STAGE = OA::BYTES + NT * OB::BYTES;
  constexpr int LDT = N + 4;
  static_assert(64 * LDT * 4 <= 2 * STAGE, "epilogue staging (64 rows at a time) fits the ring");
  static_assert(WV == 4 || WV == 8, "4 or 8 waves");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int64_t G = gridDim.x;
  const int64_t r_begin = (int64_t)blockIdx.x * e.M / G, r_end = ((int64_t)blockIdx.x + 1) * e.M / G;
  const int nk = (int)(K / 64);
  // LN': 16 lanes per row (lane gl owns columns 4 (gl + 16 j), j < NT), PR rows per pass
  const int gl = tid & 15, rsub = tid >> 4;
  float4 pg[NT], pb[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    pg[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    pb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  for (int64_t m0 = r_begin; m0 < r_end; m0 += RT) {
    const int64_t m_end = m0 + RT < r_end ? m0 + RT : r_end;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto issue = [&](int t, char* st) {
      const int64_t k0 = (int64_t)t * 64;
      if constexpr (WV == 4) {
        OA::template dma<true>(st, A, lda, m0, m_end, k0, wid, lane);   // rows >= m_end re-read row m_end - 1
#pragma unroll
        for (int j = 0; j < NT; ++j) OB::template dma<true>(st + OA::BYTES + j * OB::BYTES, B, ldb, j * 64, N, k0, wid, lane);
      } else {
        OA::template dma_nw<WV>(st, A, lda, m0, m_end, k0, wid, lane);
#pragma unroll
        for (int j = 0; j < NT; ++j) OB::template dma_nw<WV>(st + OA::BYTES + j * OB::BYTES, B, ldb, j * 64, N, k0, wid, lane);
      }
    };
    auto compute = [&](const char* sa) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = OA::frag(sa, wr * 32 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * WN + j * 16;
          bfr[j] = OB::frag(sa + OA::BYTES + (col >> 6) * OB::BYTES, col & 63, kk, lane);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    auto step = [&](int t, auto sc) {
      constexpr int S = decltype(sc)::value;
      char* cur = smem + S * STAGE;
      char* nxt = smem + (1 - S) * STAGE;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of step t landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                      // every wave's; step t-1's stage is free
      asm volatile("" ::: "memory");
      if (t + 1 < nk) issue(t + 1, nxt);
      compute(cur);
    };
    __syncthreads();  // a previous tile's epilogue reads of the staging area are done
    issue(0, smem);
    for (int t = 0; t < nk; t += 2) {
      step(t, IC<0>{});
      if (t + 1 < nk) step(t + 1, IC<1>{});
    }
    // epilogue, 64 rows at a time (the 128-row tile in two halves): the owning waves stage their f32
    // rows (alpha applied) over the ring, then every thread takes 8-column groups / LN' rows
    for (int hf = 0; hf < RT / 64; ++hf) {
    const int64_t mb = m0 + hf * 64, mbe = mb + 64 < m_end ? mb + 64 : m_end;
    if (mb >= m_end) break;  // workgroup-uniform
    __syncthreads();  // every wave's last MFMA operand reads (or the previous half's reads) are done
    float* stg = (float*)smem;
    if ((wr >> 1) == hf) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[((wr & 1) * 32 + i * 16 + (lane >> 4) * 4 + r) * LDT + wc * WN + j * 16 + (lane & 15)] = acc[i][j][r] * e.alpha;
    }
    __syncthreads();
    if constexpr (LNB) {
      // dx = rstd (g dh - mean(g dh) - xh mean(g dh xh)) + dres, xh = (x - mu) rstd (ln_bwd_vec_kernel)
      constexpr float inv = 1.f / (float)N;
      constexpr int NP = 64 / PR;
      float4 xv[NP][NT], rv[NP][NT];
      float mu[NP], rs[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {  // every operand load of the passes issued first
        int64_t m = mb + p * PR + rsub;
        m = m < mbe ? m : mbe - 1;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int c = 4 * (gl + 16 * j);
          xv[p][j] = *(const float4*)(ln.x + m * ln.ldx + c);
          rv[p][j] = ln.dres ? *(const float4*)(ln.dres + m * ln.ldr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        mu[p] = ln.mean[m];
        rs[p] = ln.rstd[m];
      }
      float4 gam[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) gam[j] = *(const float4*)(ln.gamma + 4 * (gl + 16 * j));
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int rr = p * PR + rsub;
        const int64_t m = mb + rr;
        const bool valid = m < mbe;
        float4 d[NT];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          d[j] = *(const float4*)(stg + rr * LDT + 4 * (gl + 16 * j));
#define VS_LNB(C)                                    \
  {                                                  \
    const float xh = (xv[p][j].C - mu[p]) * rs[p];   \
    const float gy = d[j].C * gam[j].C;              \
    if (valid) {                                     \
      pg[j].C += d[j].C * xh;                        \
      pb[j].C += d[j].C;                             \
    }                                                \
    xv[p][j].C = xh;                                 \
    d[j].C = gy;                                     \
    s1 += gy;                                        \
    s2 += gy * xh;                                   \
  }
          VS_LNB(x) VS_LNB(y) VS_LNB(z) VS_LNB(w)
#undef VS_LNB
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
          s1 += __shfl_xor(s1, o, 64);
          s2 += __shfl_xor(s2, o, 64);
        }
        const float m1 = s1 * inv, m2 = s2 * inv;
        if (valid) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int c = 4 * (gl + 16 * j);
            float4 o;
            o.x = rs[p] * (d[j].x - m1 - xv[p][j].x * m2) + rv[p][j].x;
            o.y = rs[p] * (d[j].y - m1 - xv[p][j].y * m2) + rv[p][j].y;
            o.z = rs[p] * (d[j].z - m1 - xv[p][j].z * m2) + rv[p][j].z;
            o.w = rs[p] * (d[j].w - m1 - xv[p][j].w * m2) + rv[p][j].w;
            *(float4*)(ln.dx + m * ln.lddx + c) = o;
            if (ln.dx_lp) {
              uint2 u;
              u.x = (uint32_t)f2bf(o.x) | ((uint32_t)f2bf(o.y) << 16);
              u.y = (uint32_t)f2bf(o.z) | ((uint32_t)f2bf(o.w) << 16);
              *(uint2*)(ln.dx_lp + m * ln.lddx + c) = u;
            }
          }
        }
      }
      continue;
    }
    if constexpr (LNF) {
      // y = (v + bias) + residual (epi_eight's order), stored f32; then ln_fwd_vec_kernel's LayerNorm
      // on the row held by 16 lanes (same lane layout and reduction order: bitwise the unfused result)
      constexpr float inv = 1.f / (float)N;
      constexpr int NP = 64 / PR;
      float4 rv[NP][NT];
#pragma unroll
      for (int p = 0; p < NP; ++p) {  // every residual load of the passes issued first
        int64_t m = mb + p * PR + rsub;
        m = m < mbe ? m : mbe - 1;
#pragma unroll
        for (int j = 0; j < NT; ++j) rv[p][j] = *(const float4*)(e.residual + m * e.ldr + 4 * (gl + 16 * j));
      }
      float4 bia[NT], gam[NT], bet[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int c = 4 * (gl + 16 * j);
        bia[j] = (EF & VS_EPI_BIAS) ? *(const float4*)(e.bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        gam[j] = *(const float4*)(ln.gamma + c);
        bet[j] = *(const float4*)(ln.beta + c);
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int rr = p * PR + rsub;
        const int64_t m = mb + rr;
        const bool valid = m < mbe;
        float4 v[NT];
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int c = 4 * (gl + 16 * j);
          v[j] = *(const float4*)(stg + rr * LDT + c);
          if constexpr ((EF & VS_EPI_BIAS) != 0) {
            v[j].x += bia[j].x; v[j].y += bia[j].y; v[j].z += bia[j].z; v[j].w += bia[j].w;
          }
          v[j].x += rv[p][j].x; v[j].y += rv[p][j].y; v[j].z += rv[p][j].z; v[j].w += rv[p][j].w;
          if (valid) *(float4*)((float*)e.c + m * e.ldc + c) = v[j];
          sm += (v[j].x + v[j].y) + (v[j].z + v[j].w);
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
        const float mu = sm * inv;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          v[j].x -= mu; v[j].y -= mu; v[j].z -= mu; v[j].w -= mu;
          q += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        const float rs = rsqrtf(q * inv + ln.eps);
        if (valid) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            float4 o;
            o.x = v[j].x * rs * gam[j].x + bet[j].x;
            o.y = v[j].y * rs * gam[j].y + bet[j].y;
            o.z = v[j].z * rs * gam[j].z + bet[j].z;
            o.w = v[j].w * rs * gam[j].w + bet[j].w;
            uint2 u;
            u.x = (uint32_t)f2bf(o.x) | ((uint32_t)f2bf(o.y) << 16);
            u.y = (uint32_t)f2bf(o.z) | ((uint32_t)f2bf(o.w) << 16);
            *(uint2*)(ln.h + m * ln.ldh + 4 * (gl + 16 * j)) = u;
          }
          if (gl == 0) {
            ln.mean_out[m] = mu;
            ln.rstd_out[m] = rs;
          }
        }
      }
      continue;
    }
    constexpr int CPR = N / 8, ITEMS = 64 * CPR / NTH;
    static_assert(64 * CPR % NTH == 0, "whole items per thread");
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int idx = tid + NTH * it, rr = idx / CPR, cg = idx % CPR;
      const int64_t m = mb + rr;
      if (m < mbe) {
        const float* src = stg + rr * LDT + cg * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_eight<EF>(e, m, (int64_t)cg * 8, v, false);
      }
    }
    }  // halves
  }
  if constexpr (LNB) {
    // dgamma / dbeta partial row of this workgroup: the 4 row groups of a wave (lanes of equal gl),
    // then the 4 waves in wave order through LDS (fixed order: bitwise reproducible)
    float* red = (float*)smem;  // [2][WV][N]
    __syncthreads();            // the last tile's staging reads are done
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#define VS_RED(V)                               \
  {                                             \
    _Pragma("unroll") for (int o = 16; o < 64; o <<= 1) { \
      V.x += __shfl_xor(V.x, o, 64);            \
      V.y += __shfl_xor(V.y, o, 64);            \
      V.z += __shfl_xor(V.z, o, 64);            \
      V.w += __shfl_xor(V.w, o, 64);            \
    }                                           \
  }
      VS_RED(pg[j]) VS_RED(pb[j])
#undef VS_RED
      if (lane < 16) {
        *(float4*)&red[(0 * WV + wid) * N + 4 * (gl + 16 * j)] = pg[j];
        *(float4*)&red[(1 * WV + wid) * N + 4 * (gl + 16 * j)] = pb[j];
      }
    }
    __syncthreads();
    for (int c = tid; c < N; c += NTH) {
      float a = (red[0 * N + c] + red[1 * N + c]) + (red[2 * N + c] + red[3 * N + c]);
      float b = (red[WV * N + c] + red[(WV + 1) * N + c]) + (red[(WV + 2) * N + c] + red[(WV + 3) * N + c]);
      if constexpr (WV == 8) {  // waves 4..7, added in the same fixed order
        a += (red[4 * N + c] + red[5 * N + c]) + (red[6 * N + c] + red[7 * N + c]);
        b += (red[12 * N + c] + red[13 * N + c]) + (red[14 * N + c] + red[15 * N + c]);
      }
      ln.part[(int64_t)blockIdx.x * 2 * N + c] = a;
      ln.part[(int64_t)blockIdx.x * 2 * N + N + c] = b;
    }
  }
}

// ----------------------------------------------------------------------------------------------
// Patch embedding with the tubelet gather in the A-operand load (mv:176-181, 194-195 + the sinusoid
// table, mv:135): x0[m, n] = sum_k X[m, k] W[n, k] + bias[n] + pos[m % n_tok, n], where X[m, k] is the
// pixel of token m = (b, f', hp, wp) at k = (c, t, i, j) — no im2col tensor.  The row-slab structure
// of gemm_bf16_slab_kernel (workgroup = contiguous token rows, all N <= 192 columns, 64-deep k
// steps, W tiles by LDS-DMA into a 2-stage ring); the A tile of a k step (64 tokens x (c, t, 4 image
// rows, 16 pixels)) is read from the f32 NCHW pixels — a wave's load instruction covers 4 adjacent
// tokens x 4 image rows, i.e. 4 contiguous 256-B row segments — NR steps ahead into registers,
// converted to bf16 and written into the same swizzled LDS image the MFMA fragments read.  Optionally
// the bf16 gathered rows are also stored (cols, the operand the weight gradient reads).
// Geometry compile-time: tubelet 2, patch 16 (the VideoMAE tubelet), K = C * 512.
// ----------------------------------------------------------------------------------------------
struct PatchGeo {
  int F, C, H, W;       // pixels (B, F, C, H, W)
  int n_tok, HpWp, Wp;  // tokens per clip, per frame pair, per patch row
};

template <int NT, bool COLS>
__global__ __launch_bounds__(256, 2) void patch_embed_fwd_kernel(const float* __restrict__ px, PatchGeo g,
                                                                 const bf16_t* __restrict__ B, int64_t K,
                                                                 EpiParams e, bf16_t* __restrict__ cols) {
  using OA = OperandBf16<64, true>;
  using OB = OperandBf16<64, true>;
  constexpr int N = 64 * NT, TM = 2, TN = NT * 2, WN = N / 2, NR = 3;
  constexpr int STAGE = OA::BYTES + NT * OB::BYTES;
  constexpr int LDT = N + 4;
  static_assert(64 * LDT * 4 <= 2 * STAGE, "epilogue staging fits the ring");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int64_t G = gridDim.x;
  const int64_t r_begin = (int64_t)blockIdx.x * e.M / G, r_end = ((int64_t)blockIdx.x + 1) * e.M / G;
  const int nk = (int)(K / 64);  // 8 steps per channel: (t, 4-row group of the patch)
  // this thread's part of every A tile: image row ii of the 4, pixels 4 jq .. 4 jq + 3 of the 16, for
  // the tokens rows (tid >> 4) + 16 s, s < 4
  const int ii = (tid >> 2) & 3, jq = tid & 3;
  const int64_t plane = (int64_t)g.H * g.W;

  for (int64_t m0 = r_begin; m0 < r_end; m0 += 64) {
    const int64_t m_end = m0 + 64 < r_end ? m0 + 64 : r_end;
    int64_t base[4];  // pixel index of (token, c = 0, t = 0, i = ii, j = 4 jq)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      int64_t m = m0 + (tid >> 4) + 16 * s;
      m = m < m_end ? m : m_end - 1;
      const int64_t b = m / g.n_tok;
      const int n = (int)(m - b * g.n_tok);
      const int fp = n / g.HpWp, r = n - fp * g.HpWp, hp = r / g.Wp, wp = r - hp * g.Wp;
      base[s] = ((b * g.F + 2 * fp) * g.C) * plane + (int64_t)(hp * 16 + ii) * g.W + wp * 16 + 4 * jq;
    }
    auto step_off = [&](int t) {  // k step t = (c, tt, i0): c = t / 8, tt = (t / 4) & 1, i0 = 4 (t & 3)
      return ((int64_t)((t >> 2) & 1) * g.C + (t >> 3)) * plane + (int64_t)(4 * (t & 3)) * g.W;
    };
    float4 ra[NR][4];
    auto gload = [&](int t, float4 (&r)[4]) {
      const int64_t o = step_off(t);
#pragma unroll
      for (int s = 0; s < 4; ++s) r[s] = *(const float4*)(px + base[s] + o);
    };
    // bf16 of this thread's 4 pixels -> A image row (token) rr, k = 16 ii + 4 jq: 8-B half of chunk 2 ii + jq / 2
    auto awrite = [&](char* st, const float4 (&r)[4], int t) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int rr = (tid >> 4) + 16 * s;
        uint2 u;
        u.x = (uint32_t)f2bf(r[s].x) | ((uint32_t)f2bf(r[s].y) << 16);
        u.y = (uint32_t)f2bf(r[s].z) | ((uint32_t)f2bf(r[s].w) << 16);
        const int c8 = 2 * ii + (jq >> 1);
        *(uint2*)(st + rr * 128 + ((c8 ^ swz_kc(rr)) << 4) + (jq & 1) * 8) = u;
      }
      (void)t;
    };
    // the bf16 rows of a completed A image as whole 128-B segments of cols (8 lanes per token row)
    auto cols_store = [&](const char* st, int t) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ci = tid + 256 * q, rr = ci >> 3, c = ci & 7;
        const int64_t m = m0 + rr;
        const uint4 v = *(const uint4*)(st + rr * 128 + ((c ^ swz_kc(rr)) << 4));
        if (m < m_end) *(uint4*)(cols + m * K + (int64_t)t * 64 + c * 8) = v;
      }
    };
    auto bdma = [&](int t, char* st) {
#pragma unroll
      for (int j = 0; j < NT; ++j) OB::template dma<true>(st + OA::BYTES + j * OB::BYTES, B, K, j * 64, N, (int64_t)t * 64, wid, lane);
    };
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const char* sa) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = OA::frag(sa, wr * 32 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * WN + j * 16;
          bfr[j] = OB::frag(sa + OA::BYTES + (col >> 6) * OB::BYTES, col & 63, kk, lane);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    __syncthreads();  // a previous tile's epilogue reads of the staging area are done
    // prologue: A of steps 0 .. NR-1 in flight, step 0 staged
#pragma unroll
    for (int t = 0; t < NR; ++t)
      if (t < nk) gload(t, ra[t]);
    bdma(0, smem);
    awrite(smem, ra[0], 0);
    if (NR < nk) gload(NR, ra[0]);
    // step t: [B DMA of t+1 into the other stage] compute(t) [A of t+1 -> LDS, loads of t+1+NR] barrier
    auto step = [&](int t, auto rc) {
      constexpr int R = decltype(rc)::value;  // register set of step t+1 = (t + 1) % NR
      char* cur = smem + (t & 1) * STAGE;
      char* nxt = smem + ((t + 1) & 1) * STAGE;
      // this wave's B pieces of step t landed; the 4 A loads of step t + NR (issued after them) may
      // stay in flight (vmcnt counts in issue order)
      if (t + NR < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // stage t complete (A written, B landed); every wave is done with stage t-1
      if (t + 1 < nk) bdma(t + 1, nxt);
      if constexpr (COLS) cols_store(cur, t);
      compute(cur);
      if (t + 1 < nk) {
        awrite(nxt, ra[R], t + 1);
        if (t + 1 + NR < nk) gload(t + 1 + NR, ra[R]);
      }
    };
    int t = 0;
    for (; t + NR <= nk; t += NR) {
      step(t, IC<1 % NR>{});
      step(t + 1, IC<2 % NR>{});
      step(t + 2, IC<3 % NR>{});
    }
    static_assert(NR == 3, "the unrolled step sequence assumes NR = 3");
    if (t < nk) step(t, IC<1 % NR>{});
    if (t + 1 < nk) step(t + 1, IC<2 % NR>{});
    // epilogue: stage the f32 tile over the ring, then 8-column groups per thread (bias + position)
    __syncthreads();
    float* stg = (float*)smem;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          stg[(wr * 32 + i * 16 + (lane >> 4) * 4 + r) * LDT + wc * WN + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    constexpr int CPR = N / 8, ITEMS = 64 * CPR / 256;
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int idx = tid + 256 * it, rr = idx / CPR, cg = idx % CPR;
      const int64_t m = m0 + rr;
      if (m < m_end) {
        const float* src = stg + rr * LDT + cg * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_eight<(uint32_t)(VS_EPI_BIAS | VS_EPI_POS)>(e, m, (int64_t)cg * 8, v, false);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// bf16 W-resident kernel for the wide K = 192 products of the ViT block: qkv (N = 576), fc1 + GELU
// (N = 768, two bf16 outputs) and the GELU' dX product da = (dx' W2) * gelu'(a_pre) (N = 768).
// Outputs are 3-4x the input, so the bound is the output stream; the per-tile kernels re-read
// their A tile once per 64-column tile and spend a barrier per tile.  Here:
//   * the N columns are cut in parts of 192; a workgroup copies its part of W (192 x 192 bf16,
//     76.8 KB with padded rows) into LDS ONCE and keeps it for its whole row range (2 workgroups
//     per CU, persistent: grid = 512, workgroup = (row range, part), XCD-grouped so the parts of
//     a range share an L2);
//   * no barrier after the fill: each wave walks its own (16-token block, 64-column chunk) units;
//     the token block's operand rows come straight from HBM as MFMA B fragments (8 consecutive k of
//     one token per lane: the K-contiguous layout), loaded once per block;
//   * the product is computed transposed, C^T = W X^T (W rows as the MFMA A operand), with the W
//     rows permuted in LDS so that a lane's two accumulator quads are 8 CONSECUTIVE output columns
//     of one token: the epilogue (bias, GELU / GELU', bf16 casts) runs on registers and writes
//     16-B vectors, no staging.  The GELU' operand of a chunk is loaded before its MFMAs.
// ----------------------------------------------------------------------------------------------
constexpr int kWresNH = 192;                  // columns per part
// LDS bytes per W row: K = 192 plus 32 B.  A ds_read_b128 of the MFMA A fragment (row = lane & 15,
// 16-B chunk 4 ks + lane / 16) is serviced in four 16-lane groups; a row stride of 104 dwords puts the
// 16 chunks of every group on distinct 4-bank quads (the 400-B stride collided in half of them:
// SQ_LDS_BANK_CONFLICT 46 % of the LDS cycles at 128 clips).  2 x (192 x 416 + 768) B fits 160 KiB.
constexpr int kWresRow = 192 * 2 + 32;

// LDS row of part-local column n: chunk ch = n / 64; within it MFMA tile jj = 2 (r / 32) + (r % 8) / 4
// and tile row i = 4 ((r % 32) / 8) + r % 4 (r = n % 64), so that accumulator rows 4g..4g+3 of
// tiles 2p and 2p+1 are the columns 32p + 8g .. 32p + 8g + 7 of the chunk.
__device__ __forceinline__ int wres_lds_row(int n) {
  const int ch = n >> 6, r = n & 63, p = r >> 5, q = r & 31;
  return ch * 64 + (2 * p + ((q >> 2) & 1)) * 16 + 4 * (q >> 3) + (q & 3);
}

template <bool BKC, uint32_t EF, int WV = 4>
__global__ __launch_bounds__(64 * WV, 2) void gemm_bf16_wres_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                const bf16_t* __restrict__ B, int64_t ldb,
                                                                EpiParams e, int dbg) {
  constexpr int K = 192, KS = K / 32, NCH = kWresNH / 64;
  constexpr bool MULA = (EF & VS_EPI_MUL_AUX) != 0;             // v *= aux (the stored gelu')
  constexpr bool GBWD = (EF & VS_EPI_GELU_BWD) != 0 || MULA;    // an aux operand per output
  __shared__ __attribute__((aligned(16))) char wl[kWresNH * kWresRow];
  __shared__ __attribute__((aligned(16))) float bl[kWresNH];
  // wave-uniform work bounds (readfirstlane): the block and chunk loops run on scalar counters
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int parts = (int)(e.N / kWresNH);
  const int G = gridDim.x, ranges = G / parts;
  const int logical = xcd_remap(blockIdx.x, G);
  const int part = logical % parts, range = logical / parts;
  if (range >= ranges) return;  // workgroup-uniform (at most parts - 1 idle workgroups)
  const int64_t r_begin = (int64_t)range * e.M / ranges, r_end = ((int64_t)range + 1) * e.M / ranges;
  const int64_t n_part = (int64_t)part * kWresNH;

  // ---- W part -> LDS (permuted rows), once: every thread issues all 18 of its 16-B loads before
  // its first LDS write (a load -> write chain per chunk serialises 18 HBM latencies)
  constexpr int NTH = 64 * WV;
  constexpr int FILL = kWresNH * K / 8 / NTH;  // 16-B chunks per thread
  static_assert(FILL * NTH * 8 == kWresNH * K, "fill split");
  uint4 fv[FILL];
  if constexpr (BKC) {  // W[n][k]: 24 16-B chunks per row
#pragma unroll
    for (int i = 0; i < FILL; ++i) {
      const int c = tid + NTH * i, n = c / (K / 8), kc = c % (K / 8);
      fv[i] = *(const uint4*)(B + (n_part + n) * ldb + kc * 8);
    }
#pragma unroll
    for (int i = 0; i < FILL; ++i) {
      const int c = tid + NTH * i, n = c / (K / 8), kc = c % (K / 8);
      *(uint4*)(wl + wres_lds_row(n) * kWresRow + kc * 16) = fv[i];
    }
  } else {  // W[k][n] (N-contiguous): 8 columns per 16-B load, scattered into 8 LDS rows
#pragma unroll
    for (int i = 0; i < FILL; ++i) {
      const int c = tid + NTH * i, k = c / (kWresNH / 8), nc = c % (kWresNH / 8);
      fv[i] = *(const uint4*)(B + (int64_t)k * ldb + n_part + nc * 8);
    }
#pragma unroll
    for (int i = 0; i < FILL; ++i) {
      const int c = tid + NTH * i, k = c / (kWresNH / 8), nc = c % (kWresNH / 8);
      const uint32_t w[4] = {fv[i].x, fv[i].y, fv[i].z, fv[i].w};
#pragma unroll
      for (int t = 0; t < 8; ++t)
        *(uint16_t*)(wl + wres_lds_row(nc * 8 + t) * kWresRow + k * 2) = (uint16_t)(w[t >> 1] >> (16 * (t & 1)));
    }
  }
  // the part's bias in LDS: the epilogue then issues no global load behind its own stores (on CDNA4
  // vmcnt counts stores too, so a load after the previous unit's stores would wait for all of them)
  if constexpr ((EF & VS_EPI_BIAS) != 0) {
    if (tid < kWresNH) bl[tid] = e.bias[n_part + tid];
  }
  __syncthreads();

  // ---- this wave's 16-token blocks (all NCH 64-column chunks of each); the next block's operand
  // rows are loaded while this block's chunks run
  const int64_t rows = r_end - r_begin;
  const int tb_n = (int)((rows + 15) / 16);
  const int tb0 = wid * tb_n / WV, tb1 = (wid + 1) * tb_n / WV - 1;
  const int g = lane >> 4, tok = lane & 15;
  const char* wbase = wl + tok * kWresRow + g * 16;  // + (tile row block) * kWresRow, + ks * 64
  if (tb0 > tb1) return;
  // Every global access goes through a buffer descriptor whose base is the token block's first row
  // (wave-uniform: the per-block address arithmetic is scalar) and whose extent ends at r_end: loads
  // of rows past the range return 0 and their stores are dropped by the range check, so no lane
  // predicate or branch remains, and hipcc sees one fixed sequence of loads and stores per block
  // (counted vmcnt waits).  Per lane only constant 32-bit offsets (+ immediates).  The host keeps
  // M x ld x 2 bytes below 2^31 for every operand.
  const uint32_t xoff = (uint32_t)(tok * lda + 8 * g) * 2u;
  const uint32_t coff = (uint32_t)(tok * e.ldc + n_part + 8 * g) * 2u;
  const uint32_t aooff = (uint32_t)(tok * e.ld_aux_out + n_part + 8 * g) * 2u;
  const uint32_t aioff = (uint32_t)(tok * e.ld_aux_in + n_part + 8 * g) * 2u;
  auto rsrc = [&](const void* base, int64_t row0, int64_t ld, bool live = true) {
    // a dead block (or one starting past the range): an empty descriptor, loads give 0, stores dropped
    const int64_t left = live && r_end > row0 ? r_end - row0 : 0;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(left * ld * 2), 0x00020000);
  };
  // x fragments held as 32-bit vectors (bf16 vector copies were re-packed lane half by lane half)
  auto load_x = [&](int tb, u32x4v (&dst)[KS]) {
    const int64_t row0 = r_begin + (int64_t)(dbg & 2 ? 0 : tb) * 16;  // dbg & 2 (timing): L2-resident reads
    const auto rx = rsrc(A + row0 * lda, row0, lda);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) dst[ks] = __builtin_amdgcn_raw_buffer_load_b128(rx, xoff + 64 * ks, 0, 0);
  };
  auto pack8 = [](const float (&v)[8]) {
    u32x4v u;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      u[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2v));
    return u;
  };
  // three fragment sets, prefetch two token blocks ahead (one block of MFMA work, ~0.5 us, hid too
  // little of the loaded HBM latency), the loop unrolled by three blocks: no register copies
  u32x4v xa[KS], xb[KS], xc[KS];
  load_x(tb0, xa);
  load_x(tb0 < tb1 ? tb0 + 1 : tb1, xb);
  auto block = [&](int tb, const u32x4v (&xf)[KS], u32x4v (&xn)[KS], bool live) {
    // compiler barrier: the W fragment reads are loop-invariant, and hoisted out of the block loop
    // they need 288 VGPRs (spills); re-read per block from LDS instead
    asm volatile("" ::: "memory");
    // unconditional (the last block re-loads itself): with a conditional prefetch the path without
    // it made hipcc wait vmcnt(0) for this block's fragments, i.e. for the prefetch just issued too
    load_x(tb + 2 <= tb1 ? tb + 2 : tb1, xn);
    __builtin_amdgcn_sched_barrier(0);  // the prefetch goes out first, ahead of this block's work
    const int64_t row0 = r_begin + (int64_t)tb * 16;
    // dbg & 1 (timing only): every block's stores rewrite the range's first two blocks (L2-resident)
    const int64_t srow0 = dbg & 1 ? r_begin + (int64_t)(tb & 1) * 16 : row0;
    const auto rc = rsrc((const bf16_t*)e.c + srow0 * e.ldc, srow0, e.ldc, live);
    const auto rao = rsrc((const bf16_t*)e.aux_out + srow0 * e.ld_aux_out, srow0, e.ld_aux_out, live);
    const auto rai = rsrc((const bf16_t*)e.aux_in + row0 * e.ld_aux_in, row0, e.ld_aux_in);
    // GELU' operand: chunk c + 1's is loaded before chunk c's stores (a counted wait then skips them)
    u32x4v aux[2][2];
    auto load_aux = [&](int ch, u32x4v (&dst)[2]) {
      if constexpr (GBWD) {
#pragma unroll
        for (int p = 0; p < 2; ++p) dst[p] = __builtin_amdgcn_raw_buffer_load_b128(rai, aioff + 2 * (ch * 64 + 32 * p), 0, 0);
      }
    };
    auto chunk = [&](int ch, u32x4v (&ax)[2], u32x4v (&axn)[2]) {
      if (ch + 1 < NCH) load_aux(ch + 1, axn);
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 wf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) wf[j] = *(const bf16x8*)(wbase + (ch * 64 + j * 16) * kWresRow + ks * 64);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], __builtin_bit_cast(bf16x8, xf[ks]), acc[j], 0, 0, 0);
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        // this lane's 8 columns: n_part + ch * 64 + 32 p + 8 g .. + 7 of token row row0 + tok
        const uint32_t cb = 2 * (ch * 64 + 32 * p);
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[2 * p][r] * e.alpha;
          v[4 + r] = acc[2 * p + 1][r] * e.alpha;
        }
        if constexpr (GBWD) {
          const u32x4v w = ax[p];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = __uint_as_float(w[q] << 16), hi = __uint_as_float(w[q] & 0xffff0000u);
            v[2 * q] *= MULA ? lo : gelu_fast_grad(lo);
            v[2 * q + 1] *= MULA ? hi : gelu_fast_grad(hi);
          }
        } else {
          if constexpr ((EF & VS_EPI_BIAS) != 0) {
            const float4 b0 = *(const float4*)&bl[ch * 64 + 32 * p + 8 * g];
            const float4 b1 = *(const float4*)&bl[ch * 64 + 32 * p + 8 * g + 4];
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
          }
          if constexpr ((EF & VS_EPI_GELU) != 0 && (EF & VS_EPI_GELU_GRAD) != 0) {
            float gr[8];  // gelu' of the bf16-rounded pre-activation: what the backward multiplies by
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = gelu_fast_both(bf2f(f2bf(v[k])), gr[k]);
            __builtin_amdgcn_raw_buffer_store_b128(pack8(gr), rao, aooff + cb, 0, 0);
          } else if constexpr ((EF & VS_EPI_GELU) != 0) {
            __builtin_amdgcn_raw_buffer_store_b128(pack8(v), rao, aooff + cb, 0, 0);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = gelu_fast(bf2f(f2bf(v[k])));  // GELU of the stored value
          }
        }
        __builtin_amdgcn_raw_buffer_store_b128(pack8(v), rc, coff + cb, 0, 0);
      }
    };
    // the chunks unrolled and unconditional (no inner loop: hipcc waits vmcnt(0) before a loop that
    // reads a pending load, i.e. for the next block's prefetch too), so every block issues the same
    // loads and stores and the waits before its MFMAs count past the previous block's stores
    load_aux(0, aux[0]);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) chunk(ch, aux[ch & 1], aux[(ch + 1) & 1]);
  };
  // The first block peeled (every entry into the loop then follows a block's stores), then triples
  // of blocks, all unconditional: a conditional block let hipcc sink the previous blocks' prefetch
  // into it (its only user), i.e. issue it right before its use.  A count that is not a multiple of
  // three ends with dead blocks (their stores dropped by an empty descriptor).
  block(tb0, xa, xc, true);
  for (int tb = tb0 + 1; tb <= tb1; tb += 3) {
    block(tb, xb, xa, true);
    block(tb + 1, xc, xb, tb + 1 <= tb1);
    block(tb + 2, xa, xc, tb + 2 <= tb1);
  }
}

// ----------------------------------------------------------------------------------------------
// bf16 wide row-slab kernel for K <= 192 and N > 192 (the ViT block's qkv, fc1 + GELU and the
// GELU' dX product: outputs 3-4x the size of the input, so they are bound by their stores).  Same
// balanced row ownership as the slab kernel (workgroup g owns rows [g M / G, (g+1) M / G), one
// 64-row tile), walking the N columns in 64-wide chunks:
//   * A: each wave keeps its 32 rows x K as MFMA fragments in registers, loaded once;
//   * W chunk c+1 (64 x K, L2-resident) is register-staged: loads in flight under chunk c's MFMAs,
//     written into the one LDS image between two barriers (guide T14);
//   * the GELU' operand of chunk c+1 is loaded under chunk c too, so the epilogue never waits on
//     HBM; epilogue stores are compiler-visible, so no wait ever drains them;
//   * epilogue per wave from a wave-private LDS staging tile (32 x 32 f32), 16-B accesses.
// 2 workgroups per CU (4 waves each).
// ----------------------------------------------------------------------------------------------
template <int KT, bool BKC, uint32_t EF>
__global__ __launch_bounds__(256, 2) void gemm_bf16_wslab_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                 const bf16_t* __restrict__ B, int64_t ldb,
                                                                 EpiParams e) {
  using OB = OperandBf16<64, BKC>;
  constexpr int KS = 2 * KT;   // 32-deep MFMA k-steps
  constexpr int LDS_T = 68;    // staging row stride (floats)
  constexpr bool MULA = (EF & VS_EPI_MUL_AUX) != 0;           // v *= aux (the stored gelu')
  constexpr bool GBWD = (EF & VS_EPI_GELU_BWD) != 0 || MULA;  // an aux operand per output
  __shared__ __attribute__((aligned(16))) char wimg[KT * OB::BYTES];
  __shared__ __attribute__((aligned(16))) float stage[4][16 * LDS_T];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t G = gridDim.x;
  const int64_t r_begin = (int64_t)blockIdx.x * e.M / G, r_end = ((int64_t)blockIdx.x + 1) * e.M / G;
  const int nch = (int)(e.N / 64);
  float* st = stage[wid];
  // wave w: rows 16w .. 16w+15 of the tile, all 64 columns of a chunk (whole 128-B output rows);
  // epilogue: lane -> rows erow, erow + 8, 8-column group ecg
  const int erow = lane >> 3, ecg = lane & 7;

  for (int64_t m0 = r_begin; m0 < r_end; m0 += 64) {
    const int64_t m_end = m0 + 64 < r_end ? m0 + 64 : r_end;
    bf16x8 af[KS];
    {
      int64_t r = m0 + wid * 16 + (lane & 15);
      r = r < m_end ? r : m_end - 1;  // rows past the slab: its last row again (never stored)
      const bf16_t* p = A + r * lda + 8 * (lane >> 4);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[ks] = *(const bf16x8*)(p + 32 * ks);
    }
    uint4 wreg[KT][OB::CHUNKS];
    auto load_w = [&](int c) {
#pragma unroll
      for (int t = 0; t < KT; ++t) OB::load(wreg[t], B, ldb, (int64_t)c * 64, e.N, t * 64, KT * 64, tid);
    };
    // GELU' operand of this lane's two epilogue rows of chunk c (rows past the slab: clamped), in
    // two named register sets (the chunk loop is unrolled by 2) so no copy waits on a load
    uint4 auxA[2], auxB[2];
    auto load_aux = [&](int c, uint4 (&dst)[2]) {
      if constexpr (GBWD) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          int64_t m = m0 + wid * 16 + erow + 8 * k;
          m = m < m_end ? m : m_end - 1;
          dst[k] = *(const uint4*)((const bf16_t*)e.aux_in + m * e.ld_aux_in + (int64_t)c * 64 + ecg * 8);
        }
      }
    };
    auto chunk = [&](int c, uint4 (&cur)[2], uint4 (&nxt)[2]) {
      __syncthreads();  // every wave is done reading chunk c-1's W image
#pragma unroll
      for (int t = 0; t < KT; ++t) OB::store(wimg + t * OB::BYTES, wreg[t], tid);
      __syncthreads();  // chunk c's W image complete
      if (c + 1 < nch) {
        load_w(c + 1);  // in flight under this chunk's MFMAs and epilogue
        load_aux(c + 1, nxt);
      }
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = OB::frag(wimg + (ks >> 1) * OB::BYTES, j * 16, ks & 1, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], bfr[j], acc[j], 0, 0, 0);
      }
      // wave-private staging: the previous chunk's epilogue reads of `st` come earlier in this
      // wave's program order, and LDS executes one wave's operations in order
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[((lane >> 4) * 4 + r) * LDS_T + j * 16 + (lane & 15)] = acc[j][r] * e.alpha;
      const int64_t n = (int64_t)c * 64 + ecg * 8;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int rr = erow + 8 * k;
        const int64_t m = m0 + wid * 16 + rr;
        const float* src = st + rr * LDS_T + ecg * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        if (m < m_end) {
          if constexpr (GBWD) {
            const uint32_t w[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float lo = __uint_as_float(w[q] << 16), hi = __uint_as_float(w[q] & 0xffff0000u);
              v[2 * q] *= MULA ? lo : gelu_fast_grad(lo);
              v[2 * q + 1] *= MULA ? hi : gelu_fast_grad(hi);
            }
            st8(e.c, m * e.ldc + n, e.out_bf16, v);
          } else {
            epi_eight<EF>(e, m, n, v, false);
          }
        }
      }
    };
    __syncthreads();  // the previous tile's readers of wimg are done
    load_w(0);
    load_aux(0, auxA);
    for (int c = 0; c < nch; c += 2) {
      chunk(c, auxA, auxB);
      if (c + 1 < nch) chunk(c + 1, auxB, auxA);
    }
  }
}

// ----------------------------------------------------------------------------------------------
// bf16 big-tile kernel for the MFMA-heavy products (K >= 512, N >= 512: ViT-Base's D = 768 /
// F = 3072 projections and their dX, 2-4 TFLOP/s-scale work per launch): 256 x 128 output tile per
// workgroup of 8 waves (4 x 2, 64 x 64 per wave: 16 accumulator tiles, 32 MFMAs per 64-deep k-step
// against 16 fragment reads), 2-stage LDS-DMA ring of 48-KB stages (asm DMA, vmcnt(0) + raw barrier;
// step t+1 in flight under step t's MFMAs; guide §5 "glds vs register staging": at ~1 block per CU
// this ties a register pipeline), one workgroup per CU; the per-tile kernels above (128 x 64, 4
// waves) re-read 4x more operand bytes per MFMA and ran these shapes at 0.1-0.2 of the MFMA roof.
// Epilogue: the f32 tile staged through the ring in two 128-row halves, 8-column groups per thread.
// ----------------------------------------------------------------------------------------------
template <bool BKC, uint32_t EF>
__global__ __launch_bounds__(512, 1) void gemm_bf16_big_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                               const bf16_t* __restrict__ B, int64_t ldb, int64_t K,
                                                               GridMap g, EpiParams e) {
  using OA = OperandBf16<256, true>;
  using OB = OperandBf16<128, BKC>;
  constexpr int STAGE = OA::BYTES + OB::BYTES;  // 48 KB
  constexpr int LDT = 128 + 4;
  constexpr int SMEM = CMax<3 * STAGE, 128 * LDT * 4>::v;  // 3-stage ring: 144 KB
  // DMA pieces (1 KB wave-instructions) one wave issues per stage: the counted wait of a step
  constexpr int PPW = OA::PIECES / 8 + OB::PIECES / 8;
  static_assert(PPW == 6, "vmcnt below assumes 6 pieces per wave and stage");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  int nt, mt, split;
  map_block(g, nt, mt, split);
  (void)split;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * 256, n0 = (int64_t)nt * 128;
  const int nk = (int)(K / 64);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int t, char* st) {
    const int64_t k0 = (int64_t)t * 64;
    OA::template dma_nw<8>(st, A, lda, m0, e.M, k0, wid, lane);
    OB::template dma_nw<8>(st + OA::BYTES, B, ldb, n0, e.N, k0, wid, lane);
  };
  auto compute = [&](const char* sa) {
    const char* sb = sa + OA::BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = OA::frag(sa, wr * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = OB::frag(sb, wc * 64 + j * 16, kk, lane);
#ifdef VS_GEMM_PRIO  // diagnostic builds: the MFMA cluster at raised wave priority
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
#ifdef VS_GEMM_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
    }
  };
  // 3-stage ring, two steps in flight (guide §5 "Pipelining across barriers": a stage stays in flight
  // across the barrier): step t waits for ITS pieces only (vmcnt(6) leaves step t+1's 6 in flight),
  // then the raw barrier makes every wave's pieces of t visible and every wave's reads of t-1 done,
  // so step t+2 may refill t-1's stage.
  auto step = [&](int t, auto sc) {
    constexpr int S = decltype(sc)::value;  // == t % 3
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) issue(t + 2, smem + ((S + 2) % 3) * STAGE);
    compute(smem + S * STAGE);
  };
  issue(0, smem);
  if (nk > 1) issue(1, smem + STAGE);
  for (int t = 0; t < nk; t += 3) {
    step(t, IC<0>{});
    if (t + 1 < nk) step(t + 1, IC<1>{});
    if (t + 2 < nk) step(t + 2, IC<2>{});
  }
  float* stg = (float*)smem;
  constexpr int CPR = 128 / 8;  // 8-column groups per row: 32 rows per pass of 512 threads
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    __syncthreads();  // every wave's last operand reads / the previous half's epilogue reads are done
    if ((wr >> 1) == part) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[((wr & 1) * 64 + i * 16 + (lane >> 4) * 4 + r) * LDT + wc * 64 + j * 16 + (lane & 15)] =
                acc[i][j][r] * e.alpha;
    }
    __syncthreads();
    // the 4 passes' operands are fetched before the first store (epi_eight_fetch: one store round
    // trip per half-tile instead of one per pass)
    EpiOps8 ops[EF == kEpiRuntime ? 1 : 4];
    if constexpr (EF != kEpiRuntime) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int64_t m = m0 + part * 128 + p * 32 + tid / CPR, n = n0 + (tid % CPR) * 8;
        epi_eight_fetch<EF>(e, m < e.M ? m : e.M - 1, n, ops[p], false);
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rr = p * 32 + tid / CPR, cg = tid % CPR;
      const int64_t m = m0 + part * 128 + rr, n = n0 + cg * 8;
      if (m < e.M) {
        const float* src = stg + rr * LDT + cg * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        if constexpr (EF != kEpiRuntime) epi_eight_finish<EF>(e, m, n, v, ops[p], false);
        else epi_eight<EF>(e, m, n, v, false);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// 256 x 256 persistent bf16 GEMM for the long-M block products of ViT-Base (C3: M = 200,704 token
// rows, N in {768, 2304, 3072}, K in {768, 2304, 3072}) where it beats the 256 x 128 big tile (VS_KNOB_G256).
//   * one persistent workgroup per CU (8 waves, 2 x 4, 128 x 64 outputs per wave: 4 x 4 16x16x32
//     MFMAs per 8 fragment reads), tiles dealt XCD-contiguously (a tile's A row-panel and the
//     weights stay in that XCD's L2);
//   * 64-deep k stages (2 x 32 KB: A and B images with 128-B rows), two LDS slots: the stage after
//     the current one is issued at its start and waited for at its last phase; the ring runs ACROSS
//     tiles, so the next tile's first stage loads under this tile's last stage and epilogue.  Full
//     128-B row segments per DMA piece (8 rows x 128 B): round 5's first version used 32-deep stages
//     whose pieces were 16 rows x 64 B, half-line requests that doubled the address path's work
//     (cdna_hip_programming.md: fragment-shaped 64-B loads +18-45 %);
//   * four phases per stage (k half x row half), the next phase's fragments read before the current
//     phase's MFMAs; one vmcnt(0) + raw barrier per stage;
//   * the product is computed transposed (C^T = B^T A^T on the MFMA), so a lane's accumulator quad is
//     4 consecutive output columns of one row: the epilogue works straight from registers with 8-B
//     (bf16) / 16-B (f32) vector loads and stores, no LDS staging, ring untouched.
// Operand images (per stage): A K-contiguous [256 rows][64 k] (128-B rows, 16-B chunk ^= (r >> 1) & 7:
// conflict-free ds_read_b128 over each 16-lane group); B K-contiguous likewise, or N-contiguous
// [64 k][256 n] (512-B rows, chunk ^= swz_mc(k): conflict-free ds_read_tr16_b64 pairs).
// ----------------------------------------------------------------------------------------------
// chunk key of the 256 x 256 kernel's K-contiguous B image: bits 1, 3, 4 of the row
__device__ __forceinline__ int g256_swzb(int r) { return ((r >> 1) & 1) | ((r >> 2) & 6); }
// a wave-uniform pointer pinned to SGPRs (the saddr operand of the asm DMA)
__device__ __forceinline__ const char* sgpr_ptr(const char* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const char*)(((uint64_t)hi << 32) | lo);
}

struct G256Map {
  int tiles_n, tiles, per_xcd, nk;  // nk = K / 64 stages per tile
  int dbg;      // VS_DEBUG_KNOBS builds: VS_KNOB_G256_DBG
  int stagger;  // odd-slot workgroups start this many s_sleep(127) (~4 us each) late (VS_KNOB_G256_STAGGER)
  int ed_ok;    // the early-DMA counted wait may be used: set by the host only when the instance has no
                // private (scratch) segment, i.e. its epilogue issues exactly `est` vector-memory ops
                // (a spill would add scratch loads / stores the count does not include)
  int a3;       // A (the streamed token-row operand) in THREE 32-KB slots, B in two: A's DMA is issued two
                // stages ahead and the stage wait is counted (vmcnt(4 + stores)), never 0 (VS_KNOB_G256_A3)
};

template <bool BKC, bool P8, uint32_t EF>
__global__ __launch_bounds__(512, 1) void gemm_bf16_g256_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                const bf16_t* __restrict__ B, int64_t ldb,
                                                                G256Map g, EpiParams e) {
  static_assert(!BKC || P8, "K-contiguous B fragments are always column-permuted (8-column vectors)");
  constexpr int AB = 256 * 64 * 2, STAGE = 2 * AB;  // 2 slots x 64 KB (a3: A 3 x 32 KB + B 2 x 32 KB)
  __shared__ __attribute__((aligned(16))) char smem[5 * AB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 2, wc = wid & 3;
  // this workgroup's tiles: XCD x = blockIdx % 8 owns logical tiles [x * per_xcd, (x+1) * per_xcd)
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, slots = gridDim.x >> 3;
  const int t_lo = xcd * g.per_xcd;
  const int t_hi = t_lo + g.per_xcd < g.tiles ? t_lo + g.per_xcd : g.tiles;
  const int my_tiles = t_lo + slot < t_hi ? (t_hi - t_lo - slot + slots - 1) / slots : 0;
  const int total = my_tiles * g.nk;  // stages of this workgroup
  if (total == 0) return;
#ifdef VS_DEBUG_KNOBS
  // diagnostic builds only (VS_KNOB_G256_DBG): bit 0 skips the operand DMA (MFMAs on stale LDS), bit
  // 1 the epilogue's stores -- the k-loop, the memory stream and the epilogue timed apart
  const int dbg = g.dbg;
#else
  constexpr int dbg = 0;
#endif
  auto tile_of = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
    const int L = t_lo + slot + k * slots;
    m0 = (L / g.tiles_n) * 256;
    n0 = (L % g.tiles_n) * 256;
  };
  // Staggered start: every CU runs the same tile schedule, so without it all 256 store their epilogue
  // at the same moment and then all stream operands at once; half of them starting late interleaves
  // the two phases across the chip.
  if (slot & 1)
    for (int i = 0; i < g.stagger; ++i) __builtin_amdgcn_s_sleep(127);

  // ---- DMA: stage s -> slot s & 1; wave w fills rows 32w .. 32w+31 of the A image (4 pieces of
  // 8 rows x 128 B) and the same of B (or k rows 8w .. 8w+7 of an N-contiguous B: 4 pieces of
  // 2 k-rows x 512 B).  Per-lane byte offsets are stage-invariant (the tile / k base is an SGPR).
  uint32_t a_off[4], b_off[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = wid * 32 + p * 8 + (lane >> 3);
    a_off[p] = (uint32_t)(r * lda * 2 + ((((lane & 7) ^ ((r >> 1) & 7))) << 4));
    if constexpr (BKC) {  // B image chunk key g256_swzb(r) (fragment rows are permuted, see below)
      b_off[p] = (uint32_t)(r * ldb * 2 + ((((lane & 7) ^ g256_swzb(r))) << 4));
    } else {
      const int k = wid * 8 + 2 * p + (lane >> 5);
      b_off[p] = (uint32_t)(k * ldb * 2 + ((((lane & 31) ^ swz_mc<128>(k))) << 4));
    }
  }
  // Slot byte offsets: A of stage s at a_at(slot), B at b_at(slot) + AB (the B read offsets include + AB);
  // slots cycle 0, 1 (A and B together) or, a3, A 0, 1, 2 and B 0, 1
  const bool a3 = g.a3 != 0;
  auto a_at = [&](int sl) __attribute__((always_inline)) { return a3 ? sl * AB : sl * STAGE; };
  auto b_at = [&](int sl) __attribute__((always_inline)) { return a3 ? 2 * AB + sl * AB : sl * STAGE; };
  auto a_nxt = [&](int sl) __attribute__((always_inline)) { return a3 ? (sl == 2 ? 0 : sl + 1) : (sl ^ 1); };
  // The A and B DMA streams each issue stages 0, 1, 2, ... in order: scalar state advanced per stage
  // (global base + 64 k, the tile's rows and bases recomputed once per tile), LDS destinations as
  // wave-uniform 32-bit addresses (the round-5 form recomputed the tile by two divisions and converted
  // each piece's generic LDS pointer -- ~300 scalar / vector instructions per stage and wave)
  const uint32_t lds_w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(VS_LDS char*)smem) +
                         (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 4096u;
  const int64_t b_step = BKC ? 128 : (int64_t)128 * ldb;  // bytes per 64-deep stage of B
  int sa_k = 0, sa_t = 0, sa_sl = 0, sb_k = 0, sb_t = 0, sb_sl = 0;
  int64_t sa_rows = 0;
  const char* sa_ptr = nullptr;
  const char* sb_ptr = nullptr;
  auto a_tile = [&]() __attribute__((always_inline)) {
    int m0, n0;
    tile_of(sa_k, m0, n0);
    (void)n0;
    sa_rows = e.M - m0;  // rows past M re-read row M-1 (never stored)
    sa_ptr = (const char*)(A + (int64_t)m0 * lda);
  };
  auto b_tile = [&]() __attribute__((always_inline)) {
    int m0, n0;
    tile_of(sb_k, m0, n0);
    (void)m0;
    sb_ptr = BKC ? (const char*)(B + (int64_t)n0 * ldb) : (const char*)(B + n0);
  };
  a_tile();
  b_tile();
  auto issue_a = [&]() __attribute__((always_inline)) {
    if (!(dbg & 1)) {
      const uint32_t l = lds_w + (uint32_t)a_at(sa_sl);
      if (sa_rows >= 256) {
        glds16x4_m0(sa_ptr, a_off[0], a_off[1], a_off[2], a_off[3], l, l + 1024, l + 2048, l + 3072);
      } else {
        uint32_t o[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int r = wid * 32 + p * 8 + (lane >> 3), rc = r < sa_rows ? r : (int)sa_rows - 1;
          o[p] = (uint32_t)(rc * lda * 2 + ((((lane & 7) ^ ((r >> 1) & 7))) << 4));
        }
        glds16x4_m0(sa_ptr, o[0], o[1], o[2], o[3], l, l + 1024, l + 2048, l + 3072);
      }
    }
    if (++sa_t == g.nk) {
      sa_t = 0;
      ++sa_k;
      a_tile();
    } else {
      sa_ptr += 128;
    }
    sa_sl = a_nxt(sa_sl);
  };
  auto issue_b = [&]() __attribute__((always_inline)) {
    if (!(dbg & 1)) {
      const uint32_t l = lds_w + (uint32_t)(b_at(sb_sl) + AB);
      glds16x4_m0(sb_ptr, b_off[0], b_off[1], b_off[2], b_off[3], l, l + 1024, l + 2048, l + 3072);
    }
    if (++sb_t == g.nk) {
      sb_t = 0;
      ++sb_k;
      b_tile();
    } else {
      sb_ptr += b_step;
    }
    sb_sl ^= 1;
  };
  auto issue = [&]() __attribute__((always_inline)) {
    issue_a();
    issue_b();
  };

  // ---- fragments (per lane, stage-invariant byte offsets; kk = 32-deep half of the stage)
  // K-contiguous B (the forward products, bf16 out): fragment j = 2p + e, row r holds output column
  // wc*64 + 32p + 8(r >> 2) + 4e + (r & 3), so the accumulator quads of fragments 2p and 2p+1 in one
  // lane are 8 CONSECUTIVE columns (8fc .. 8fc+7 of the 32-column half p) and the epilogue moves 16-B
  // bf16 vectors.  The image's chunk key g256_swzb(n) reads bits 1, 3, 4 of n -- unchanged by 4e and
  // 32p, so every fragment is the lane address + an immediate -- and keeps the ds_read_b128 groups
  // conflict-free (checked by enumeration).  N-contiguous B (read transposed, ds_read_tr16_b64) takes
  // the same permutation when the output is bf16 (P8: its quads then conflict 2-way) and keeps plain
  // 4-column quads for f32 outputs (16-B vectors already).
  const int fr = lane & 15, fc = lane >> 4;
  int a_rd[2], b_rd[4][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) a_rd[kk] = (wr * 128 + fr) * 128 + (((kk * 4 + fc) ^ ((fr >> 1) & 7)) << 4);
  if constexpr (BKC) {
    // image row n = R0 + 32p + 4e, R0 = wc*64 + 8(fr >> 2) + (fr & 3): key(n) = key(R0)
    const int R0 = wc * 64 + 8 * (fr >> 2) + (fr & 3);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) b_rd[kk][0] = AB + R0 * 128 + (((kk * 4 + fc) ^ g256_swzb(R0)) << 4);
  } else {  // k rows kr0 / kr1 of a 32-deep half (swz_mc has period 16 in k: the second half is + 16 KB)
    const int q = fr >> 2, kr0 = 8 * fc + q, kr1 = kr0 + 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = P8 ? wc * 64 + 32 * (j >> 1) + 8 * (lane & 3) + 4 * (j & 1) : wc * 64 + j * 16 + (lane & 3) * 4;
      b_rd[j][0] = AB + kr0 * 512 + (((col >> 3) ^ swz_mc<128>(kr0)) << 4) + (col & 7) * 2;
      b_rd[j][1] = AB + kr1 * 512 + (((col >> 3) ^ swz_mc<128>(kr1)) << 4) + (col & 7) * 2;
    }
  }
  auto read_a = [&](const char* st, int kk, int rh, bf16x8 (&af)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 4; ++f) af[f] = *(const bf16x8*)(st + a_rd[kk] + (rh * 64 + f * 16) * 128);
  };
  auto read_b = [&](const char* st, int kk, bf16x8 (&bf)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (BKC) {
        bf[j] = *(const bf16x8*)(st + b_rd[kk][0] + (32 * (j >> 1) + 4 * (j & 1)) * 128);
      } else {
        short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(st + b_rd[j][0] + kk * 16384));
        short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(st + b_rd[j][1] + kk * 16384));
        typedef __attribute__((ext_vector_type(8))) short short8v;
        short8v v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
        bf[j] = __builtin_bit_cast(bf16x8, v);
      }
    }
  };

  f32x4 acc[8][4];  // each tile's first k-step overwrites them (mfma16z); zeroed once so no path reads undef
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue geometry (see below) and the bias, which the early-DMA variants load one stage ahead
  constexpr int EW = P8 ? 8 : 4, ENV = 16 / EW, EVS = P8 ? 32 : 16;
  constexpr bool EBIAS = (EF & VS_EPI_BIAS) != 0;
  // ED (early DMA): the variants whose epilogue loads nothing per row (bias at most) issue each stage's
  // successor DMA right after the barrier that frees its slot -- before a tile's epilogue stores --
  // and wait for it with vmcnt(<stores issued since>), so the stores drain under the next tile's first
  // stage instead of stalling it (vmcnt retires loads, DMA and stores in order)
  constexpr bool ED = (EF & (VS_EPI_RESIDUAL | VS_EPI_MUL_AUX | VS_EPI_GELU_BWD)) == 0;
  // The early-DMA variants' bias by SCALAR loads (constant address space, wave-uniform base): counted by
  // lgkmcnt, so hipcc's wait for them never drains the in-flight DMA (a vector load's vmcnt wait does:
  // vmcnt retires in order); each lane then picks its EW columns of the wave's 4 x EW by fc
  float ebias[ENV][EW];
  auto load_bias = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_of(k, m0, n0);
    (void)m0;
    if constexpr (ED) {
      typedef const __attribute__((address_space(4))) float* cfp;
      const cfp bp = (cfp)e.bias + __builtin_amdgcn_readfirstlane(n0 + wc * 64);
#pragma unroll
      for (int vv = 0; vv < ENV; ++vv) {
        float sb[4 * EW];
#pragma unroll
        for (int q = 0; q < 4 * EW; ++q) sb[q] = bp[EVS * vv + q];
#pragma unroll
        for (int r = 0; r < EW; ++r)
          ebias[vv][r] = fc == 0 ? sb[r] : fc == 1 ? sb[EW + r] : fc == 2 ? sb[2 * EW + r] : sb[3 * EW + r];
      }
    } else {
      // the residual / GELU' variants drain vmcnt every stage anyway; scalar loads there cost SGPRs that
      // their epilogue's operand addressing needs (fc2: SGPR spills to VGPR lanes at 256 VGPRs, 974 -> 1,177 us)
#pragma unroll
      for (int vv = 0; vv < ENV; ++vv) {
        if constexpr (EW == 8) ld8(e.bias, n0 + wc * 64 + EW * fc + EVS * vv, 0, ebias[vv]);
        else ld4(e.bias, n0 + wc * 64 + EW * fc + EVS * vv, 0, ebias[vv]);
      }
    }
  };
  // epilogue store instructions per lane (vmcnt units), all issued after the early DMA
  const int est_c = 8 * ENV * ((EW == 8 && !e.out_bf16) ? 2 : 1);
  const int est = est_c + ((EF & VS_EPI_GELU) ? 8 * ENV : 0);

  // Epilogue straight from the accumulators (C^T layout: lane (fr, fc) holds row m0+...+fr and W = 8
  // consecutive columns per 32-column half v (K-contiguous B: acc[i][2v] | acc[i][2v+1], columns 8fc ..)
  // or W = 4 per 16-column block v (acc[i][v], columns 4fc ..)).  CDNA4's vmcnt counts stores as well
  // as loads and retires them in order, so a "load operand -> use -> store" sequence per vector would
  // wait for every earlier store; every operand a group of rows needs is loaded before its first
  // store: the bias once per tile, the residual / GELU' factor per 32 rows of the wave.
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int m0, n0;
    tile_of(k, m0, n0);
    constexpr uint32_t F = EF;
    constexpr bool BIAS = (F & VS_EPI_BIAS) != 0, RES = (F & VS_EPI_RESIDUAL) != 0;
    constexpr bool AUXIN = (F & (VS_EPI_MUL_AUX | VS_EPI_GELU_BWD)) != 0, GELU = (F & VS_EPI_GELU) != 0;
    constexpr int W = EW, NV = ENV;  // columns per vector, vectors per row fragment
    constexpr int VS = EVS;          // column step between a lane's vectors
    const int ncol = n0 + wc * 64 + W * fc;
    auto stv = [&](void* p, int64_t i, int bf, const float (&v)[W]) __attribute__((always_inline)) {
      if constexpr (W == 8) st8(p, i, bf, v);
      else st4(p, i, bf, v);
    };
    if constexpr (BIAS && !ED) load_bias(k);  // ED: loaded at the start of the tile's last stage
    // Operand rows (residual f32, GELU' factor bf16: g256 runs bf16 operands only) as raw 16-B vectors,
    // row fragment i+1's loads issued before fragment i's stores (round 6).  vmcnt retires in order, so
    // a load issued after a fragment's stores waited for all of them: round 5 loaded per 32 rows, and
    // each later group of the epilogue stalled on the previous group's store completion.
    struct Raw {
      float4 f[NV][W / 4];
      uint4 h8[NV];
      uint2 h4[NV];
    };
    auto ld_raw = [&](int i, Raw& rw) __attribute__((always_inline)) {
      const int64_t m = m0 + wr * 128 + i * 16 + fr;
      const int64_t mc = m < e.M ? m : e.M - 1;  // rows past M: any valid row (not stored)
#pragma unroll
      for (int vv = 0; vv < NV; ++vv) {
        if constexpr (RES) {
#pragma unroll
          for (int q = 0; q < W / 4; ++q) rw.f[vv][q] = *(const float4*)(e.residual + mc * e.ldr + ncol + VS * vv + 4 * q);
        } else if constexpr (W == 8) {
          rw.h8[vv] = *(const uint4*)((const bf16_t*)e.aux_in + mc * e.ld_aux_in + ncol + VS * vv);
        } else {
          rw.h4[vv] = *(const uint2*)((const bf16_t*)e.aux_in + mc * e.ld_aux_in + ncol + VS * vv);
        }
      }
    };
    auto unpack = [&](const Raw& rw, int vv, float (&o)[W]) __attribute__((always_inline)) {
      if constexpr (RES) {
#pragma unroll
        for (int q = 0; q < W / 4; ++q) {
          o[4 * q] = rw.f[vv][q].x;
          o[4 * q + 1] = rw.f[vv][q].y;
          o[4 * q + 2] = rw.f[vv][q].z;
          o[4 * q + 3] = rw.f[vv][q].w;
        }
      } else {
        uint32_t w4[W / 2];
        if constexpr (W == 8) {
          w4[0] = rw.h8[vv].x; w4[1] = rw.h8[vv].y; w4[2] = rw.h8[vv].z; w4[3] = rw.h8[vv].w;
        } else {
          w4[0] = rw.h4[vv].x; w4[1] = rw.h4[vv].y;
        }
#pragma unroll
        for (int q = 0; q < W / 2; ++q) {
          o[2 * q] = __uint_as_float(w4[q] << 16);
          o[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
        }
      }
    };
    Raw rbuf[2];
    if constexpr (RES || AUXIN) ld_raw(0, rbuf[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (RES || AUXIN) {
        if (i + 1 < 8) ld_raw(i + 1, rbuf[(i + 1) & 1]);
      }
      {
        const int64_t m = m0 + wr * 128 + i * 16 + fr;
        const bool live = m < e.M;
#pragma unroll
        for (int vv = 0; vv < NV; ++vv) {
          float opv[W];
          if constexpr (RES || AUXIN) unpack(rbuf[i & 1], vv, opv);
          float v[W], t[W];
#pragma unroll
          for (int r = 0; r < W; ++r) {
            v[r] = acc[i][(W / 4) * vv + (r >> 2)][r & 3] * e.alpha;
            if constexpr (BIAS) v[r] += ebias[vv][r];
          }
          if constexpr ((F & VS_EPI_GELU_BWD) != 0) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] *= gelu_fast_grad(opv[r]);
          }
          if constexpr ((F & VS_EPI_MUL_AUX) != 0) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] *= opv[r];
          }
          const int64_t n = ncol + VS * vv;
          if constexpr (GELU) {
            if constexpr ((F & VS_EPI_GELU_GRAD) != 0) {  // packed pairs (the epilogue's dominant VALU)
#pragma unroll
              for (int r = 0; r < W; r += 2) {
                const f32x2v x = {bf2f(f2bf(v[r])), bf2f(f2bf(v[r + 1]))};
                f32x2v gr;
                const f32x2v y = gelu_fast_both2(x, gr);
                v[r] = y.x;
                v[r + 1] = y.y;
                t[r] = gr.x;
                t[r + 1] = gr.y;
              }
            } else {
#pragma unroll
              for (int r = 0; r < W; ++r) {
                const float x = bf2f(f2bf(v[r]));
                t[r] = v[r];
                v[r] = gelu_fast(x);
              }
            }
            if (live && !(dbg & 2)) stv(e.aux_out, m * e.ld_aux_out + n, e.op_bf16, t);
          }
          if constexpr (RES) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] += opv[r];
          }
          if (live && !(dbg & 2)) stv(e.c, m * e.ldc + n, e.out_bf16, v);
          // ED: no re-zeroing (the next tile's first k-step MFMAs take a zero C operand); the residual /
          // GELU' variants keep the zeroing pass: with the zero-C copy of the MFMA block fc2 (256 VGPRs)
          // measured 974 -> 1,236 us
          if constexpr (!ED) {
#pragma unroll
            for (int q = 0; q < W / 4; ++q) acc[i][(W / 4) * vv + q] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
    }
  };

  auto mfma16 = [&](const bf16x8 (&bc)[4], const bf16x8 (&af)[4], int rh) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[rh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], af[i], acc[rh * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // a tile's first k-step: C = 0 (an inline constant), so the accumulators need no zeroing pass
  // (128 v_mov per wave and tile)
  auto mfma16z = [&](const bf16x8 (&bc)[4], const bf16x8 (&af)[4], int rh) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[rh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], af[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: stage 0 landed, its first fragments in registers
  bf16x8 a0[4], a1[4], b0[4], b1[4];
  issue();  // stage 0
  if (a3 && total > 1) {
    issue_a();  // A(1)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A(0), B(0) landed; A(1) in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_b(smem + b_at(0), 0, b0);
  read_a(smem + a_at(0), 0, 0, a0);

  // Stage s (slot s & 1), four phases; fragments of the next phase are read before this phase's MFMAs:
  //   P0: DMA stage s+1 into the other slot (every wave's reads of stage s-1 retired before the
  //       barrier of s-1's P3) | A(kk0, rh1) | MFMA B0 x A(kk0, rh0)
  //   P1: B(kk1), A(kk1, rh0) | MFMA B0 x A(kk0, rh1)
  //   P2: A(kk1, rh1) | MFMA B1 x A(kk1, rh0)
  //   P3: vmcnt(0) + lgkmcnt(0) + barrier (stage s+1 landed everywhere; stage s's reads retired) |
  //       B(kk0), A(kk0, rh0) of stage s+1 | MFMA B1 x A(kk1, rh1) | epilogue at a tile's last stage
  // a3: A(s+2) is issued with B(s+1) at P0 (ED: B(s+2) and A(s+3) after the barrier of stage s, into the
  // slots stage s just freed); the P3 wait keeps the youngest A stage (4 pieces per wave) and the stores in
  // flight.  Spreading A's pieces over the phases instead (one per phase, the guide's 8-phase interleave)
  // measured 1-11 % SLOWER on every dX product (profiles/r06_g256_a3s_ab.json)
  if (ED && total > 1) {
    if (a3) {
      issue_b();                  // B(1)
      if (total > 2) issue_a();   // A(2)
    } else {
      issue();                    // stage 1
    }
  }
  int nst = 0;  // ED: store instructions issued after the DMA in flight (the previous tile's epilogue)
  int ra = 0, rb = 0, tk = 0, tt = 0;  // compute side: slots of stage s, its tile and k-step
  for (int s = 0; s < total; ++s) {
    const char* cur = smem + a_at(ra);
    const char* curb = smem + b_at(rb);
    const bool last = tt == g.nk - 1;
    const bool a_next = a3 && s + 2 < total;  // A(s+2) in flight at this stage's wait
    if (!ED) {
      if (a3) {
        if (s + 1 < total) issue_b();  // B(s+1)
        if (a_next) issue_a();         // A(s+2)
      } else if (s + 1 < total) {
        issue();                       // stage s+1
      }
    }
    if (ED && EBIAS && last) load_bias(tk);
    read_a(cur, 0, 1, a1);
    __builtin_amdgcn_sched_barrier(0);
    if (ED && tt == 0) mfma16z(b0, a0, 0);
    else mfma16(b0, a0, 0);
    read_b(curb, 1, b1);
    read_a(cur, 1, 0, a0);
    __builtin_amdgcn_sched_barrier(0);
    if (ED && tt == 0) mfma16z(b0, a1, 1);
    else mfma16(b0, a1, 1);
    read_a(cur, 1, 1, a1);
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b1, a0, 0);
    // stage s+1 landed: vmcnt(0), or all but the youngest `allow` ops -- (ED) the nst stores issued after
    // its DMA, (a3) the 4 pieces of A(s+2) -- as the largest encodable count <= allow (waiting for more
    // than needed is always safe)
    const int allow = (ED ? nst : 0) + (a_next ? 4 : 0);
    if (allow < 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (allow < 16) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (allow < 20) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (allow < 32) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (allow < 36) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (allow < 48) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
    else if (allow < 52) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (allow < 63) asm volatile("s_waitcnt vmcnt(52)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (ED) {
      if (EBIAS && last) {  // the bias (scalar loads at this stage's start) in registers before the next DMA
#pragma unroll
        for (int vv = 0; vv < ENV; ++vv)
#pragma unroll
          for (int r = 0; r < EW; ++r) asm volatile("" : "+v"(ebias[vv][r]));
      }
      // into the slots of stage s: every wave's reads of stage s retired
      if (a3) {
        if (s + 2 < total) issue_b();  // B(s+2)
        if (s + 3 < total) issue_a();  // A(s+3)
      } else if (s + 2 < total) {
        issue();                       // stage s+2
      }
    }
    ra = a_nxt(ra);
    rb ^= 1;
    if (s + 1 < total) {
      read_b(smem + b_at(rb), 0, b0);
      read_a(smem + a_at(ra), 0, 0, a0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b1, a1, 1);
    nst = 0;
    if (last) {
      epilogue(tk);
      if constexpr (ED) {
        int m0, n0;
        tile_of(tk, m0, n0);
        (void)n0;
        // exact count only for a full tile (a ragged one skips the stores of all-dead rows) and real stores
        nst = (g.ed_ok && m0 + 256 <= e.M && !(dbg & 2)) ? (est < 63 ? est : 63) : 0;
      }
      tt = 0;
      ++tk;
    } else {
      ++tt;
    }
  }
}

// ----------------------------------------------------------------------------------------------
// 256 x 256 persistent weight-gradient GEMM: dW[M][N] += dY^T X over the token axis for the long-K
// products of ViT-Base (C3: K = 200,704 tokens; M, N in {768, 2304, 3072}), VERDICT r4 item 3 ("a
// true long-K GEMM with few splits and large tiles").  Same engine as gemm_bf16_g256_kernel (8 waves,
// 128 x 64 per wave, C^T on the MFMA, 64-deep stages of 2 x 32 KB, two slots, one barrier per
// stage), with both operands token-major: A = dY [K][M] and B = X [K][N] are staged as [64 k][256]
// images (512-B rows, chunk ^= swz_mc(k)) and BOTH are read by ds_read_tr16_b64.  The token axis is
// cut into `splits` equal slabs; an item = (split, tile) is processed by one workgroup and its f32
// 256 x 256 partial goes to the workspace, which gemm_dw256_reduce sums IN SPLIT ORDER into C (C +=
// sum: bitwise reproducible, no atomics).  Items are dealt XCD-contiguously, split-major: the
// workgroups of one XCD share one token slab's A and B rows in its L2.  The bias gradient (row sums
// of dY) is summed from the staged A image by VALU, spread over the tile's N-column items (item
// (mt, nt) takes the k rows r % tiles_n == nt), into per-item partial rows reduced the same way.
// A tile's A fragment offsets differ per 16-row fragment only in chunk bits 1-3, which the k-row
// swizzle also uses: the read address is a lane constant XOR an immediate (one v_xor per read).
// ----------------------------------------------------------------------------------------------
struct Dw256Map {
  int tiles_n, tiles, items, per_xcd, kps, nk;
};

template <bool SUMS>
__global__ __launch_bounds__(512, 1) void gemm_dw256_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                            const bf16_t* __restrict__ B, int64_t ldb, Dw256Map g,
                                                            float* __restrict__ part, float* __restrict__ sums) {
  constexpr int AB = 64 * 256 * 2, STAGE = 2 * AB;  // 2 slots x 64 KB (+ 16 KB of bias partials)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 2, wc = wid & 3;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, slots = gridDim.x >> 3;
  const int i_lo = xcd * g.per_xcd;
  const int i_hi = i_lo + g.per_xcd < g.items ? i_lo + g.per_xcd : g.items;
  const int my_items = i_lo + slot < i_hi ? (i_hi - i_lo - slot + slots - 1) / slots : 0;
  if (my_items == 0) return;
  auto item_of = [&](int k) __attribute__((always_inline)) { return i_lo + slot + k * slots; };
  auto steps_of = [&](int item) __attribute__((always_inline)) {
    const int k0 = (item / g.tiles) * g.kps;
    return g.nk - k0 < g.kps ? g.nk - k0 : g.kps;
  };

  // ---- DMA: wave w fills k rows 8w .. 8w+7 of both images (4 pieces of 2 k-rows x 512 B each)
  uint32_t a_off[4], b_off[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int k = wid * 8 + 2 * p + (lane >> 5), c = ((lane & 31) ^ swz_mc<128>(k)) << 4;
    a_off[p] = (uint32_t)(k * lda * 2 + c);
    b_off[p] = (uint32_t)(k * ldb * 2 + c);
  }
  // The DMA stream's global bases are recomputed (two divisions) only when it moves to a new item and
  // advanced by 64 token rows per stage otherwise; LDS destinations are wave-uniform 32-bit addresses
  // (glds16x4_m0: no per-piece generic -> LDS conversion)
  const uint32_t lds_w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(VS_LDS char*)smem) +
                         (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 4096u;
  const char* dA = nullptr;
  const char* dB = nullptr;
  auto item_bases = [&](int item, int t) __attribute__((always_inline)) {
    const int sp = item / g.tiles, tile = item - sp * g.tiles, mt = tile / g.tiles_n, nt = tile - mt * g.tiles_n;
    const int64_t k0 = (int64_t)(sp * g.kps + t) * 64;
    dA = (const char*)(A + k0 * lda + (int64_t)mt * 256);
    dB = (const char*)(B + k0 * ldb + (int64_t)nt * 256);
  };
  auto issue = [&](int item, int t, int slot_s) __attribute__((always_inline)) {
    if (t == 0) item_bases(item, 0);
    else {
      dA += (int64_t)128 * lda;  // 64 token rows
      dB += (int64_t)128 * ldb;
    }
    const uint32_t l = lds_w + (uint32_t)(slot_s * STAGE);
    glds16x4_m0(dA, a_off[0], a_off[1], a_off[2], a_off[3], l, l + 1024, l + 2048, l + 3072);
    glds16x4_m0(dB, b_off[0], b_off[1], b_off[2], b_off[3], l + AB, l + AB + 1024, l + AB + 2048, l + AB + 3072);
  };

  // ---- fragments: lane (fr, fc) reads k rows kr0 = 8 fc + (fr >> 2) and kr0 + 4, columns p4 .. p4+3
  // of each 16-column block (ds_read_tr16_b64 pairs: the MFMA operand layout row = lane & 15,
  // k = 8 (lane >> 4) + 0..7).  A: block base wr*128 + rh*64 + f*16 -> address = xa ^ ((rh*8 + f*2) << 4).
  const int fr = lane & 15, fc = lane >> 4;
  const int q = fr >> 2, p4 = (lane & 3) * 4, kr0 = 8 * fc + q, kr1 = kr0 + 4;
  const int lc = wr * 16 + (p4 >> 3);
  const int xa0 = kr0 * 512 + ((lc ^ swz_mc<128>(kr0)) << 4) + (p4 & 7) * 2;
  const int xa1 = kr1 * 512 + ((lc ^ swz_mc<128>(kr1)) << 4) + (p4 & 7) * 2;
  int b_rd[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wc * 64 + j * 16 + p4;
    b_rd[j][0] = AB + kr0 * 512 + (((col >> 3) ^ swz_mc<128>(kr0)) << 4) + (col & 7) * 2;
    b_rd[j][1] = AB + kr1 * 512 + (((col >> 3) ^ swz_mc<128>(kr1)) << 4) + (col & 7) * 2;
  }
  typedef __attribute__((ext_vector_type(8))) short short8v;
  auto tr_frag = [&](const char* p0, const char* p1) __attribute__((always_inline)) {
    short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)p0);
    short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)p1);
    short8v v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  auto read_a = [&](const char* st, int kk, int rh, bf16x8 (&af)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int x = (rh * 8 + f * 2) << 4;
      af[f] = tr_frag(st + kk * 16384 + (xa0 ^ x), st + kk * 16384 + (xa1 ^ x));
    }
  };
  auto read_b = [&](const char* st, int kk, bf16x8 (&bf)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = tr_frag(st + b_rd[j][0] + kk * 16384, st + b_rd[j][1] + kk * 16384);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias-gradient partials: thread -> 4-column group sg = tid & 63 of the A image, k rows
  // (tid >> 6) + 8 i whose index is = nt (mod tiles_n), 4 running sums in registers (8-column groups
  // in registers spilled 13 VGPRs; in a thread-private LDS slot they cost a read-modify-write per
  // stage: dW qkv 918 us with, 826 without the sums)
  const int sg = tid & 63, sr = tid >> 6;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  int bmask = 0;  // bit ii: k row sr + 8 ii belongs to this item's share (recomputed per item)
  auto set_bmask = [&](int it) __attribute__((always_inline)) {
    const int nt = (it % g.tiles) % g.tiles_n;
    bmask = 0;
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) bmask |= ((sr + 8 * ii) % g.tiles_n == nt) << ii;
  };
  auto bias_rows = [&](const char* st) __attribute__((always_inline)) {
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const int r = sr + 8 * ii;
      if ((bmask >> ii) & 1) {
        const uint2 u = *(const uint2*)(st + r * 512 + (((sg >> 1) ^ swz_mc<128>(r)) << 4) + (sg & 1) * 8);
        bsum[0] += __uint_as_float(u.x << 16);
        bsum[1] += __uint_as_float(u.x & 0xffff0000u);
        bsum[2] += __uint_as_float(u.y << 16);
        bsum[3] += __uint_as_float(u.y & 0xffff0000u);
      }
    }
  };
  auto epilogue = [&](int item) __attribute__((always_inline)) {
    float* pt = part + (int64_t)item * 65536;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float v[4] = {acc[i][jj][0], acc[i][jj][1], acc[i][jj][2], acc[i][jj][3]};
        st4(pt, (wr * 128 + i * 16 + fr) * 256 + wc * 64 + jj * 16 + 4 * fc, 0, v);
        acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    if constexpr (SUMS) {
      *(float4*)(sums + ((int64_t)item * 8 + sr) * 256 + sg * 4) = make_float4(bsum[0], bsum[1], bsum[2], bsum[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c) bsum[c] = 0.f;
    }
  };
  auto mfma16 = [&](const bf16x8 (&bc)[4], const bf16x8 (&af)[4], int rh) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[rh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], af[i], acc[rh * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  bf16x8 a0[4], a1[4], b0[4], b1[4];
  int item = item_of(0), nsteps = steps_of(item), k = 0, t = 0, s = 0;
  if constexpr (SUMS) set_bmask(item);
  issue(item, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_b(smem, 0, b0);
  read_a(smem, 0, 0, a0);
  // the four phases of gemm_bf16_g256_kernel's stage loop; (k, t) walks this workgroup's items and
  // their k-steps, the ring continues across items
  while (true) {
    const char* cur = smem + (s & 1) * STAGE;
    int nk_item = k, nt_step = t + 1;
    if (nt_step == nsteps) {
      nk_item = k + 1;
      nt_step = 0;
    }
    const bool more = nk_item < my_items;
    const int nitem = nk_item == k ? item : (more ? item_of(nk_item) : item);
    if (more) issue(nitem, nt_step, (s + 1) & 1);
    read_a(cur, 0, 1, a1);
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b0, a0, 0);
    read_b(cur, 1, b1);
    read_a(cur, 1, 0, a0);
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b0, a1, 1);
    read_a(cur, 1, 1, a1);
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b1, a0, 0);
    if constexpr (SUMS) bias_rows(cur);  // behind the queued MFMAs (a0's registers are dead here)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (more) {
      const char* nxt = smem + ((s + 1) & 1) * STAGE;
      read_b(nxt, 0, b0);
      read_a(nxt, 0, 0, a0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma16(b1, a1, 1);
    if (nk_item != k) epilogue(item);
    if (!more) break;
    if (nk_item != k) {
      item = nitem;
      nsteps = steps_of(item);
      if constexpr (SUMS) set_bmask(item);
    }
    k = nk_item;
    t = nt_step;
    ++s;
  }
}

// C[m][n] += sum over splits (in order) of the items' partial tiles; bias[m] += the bias partials
// (splits, then the tile row's N-column items, then the 8 partial rows, in order).  One thread per
// output float4, then one per bias element.
__global__ __launch_bounds__(256) void gemm_dw256_reduce(const float* __restrict__ part, const float* __restrict__ sums,
                                                         Dw256Map g, int splits, int64_t M, int64_t N,
                                                         float* __restrict__ c, int64_t ldc, float* __restrict__ bias) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, nc4 = M * N / 4;
  if (i < nc4) {
    const int64_t m = i / (N / 4), n = (i % (N / 4)) * 4;
    const int tile = (int)(m / 256) * g.tiles_n + (int)(n / 256);
    const int64_t off = (m % 256) * 256 + (n % 256);
    float4 acc = *(const float4*)(part + (int64_t)tile * 65536 + off);
    for (int sp = 1; sp < splits; ++sp) {
      const float4 v = *(const float4*)(part + ((int64_t)sp * g.tiles + tile) * 65536 + off);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4* cp = (float4*)(c + m * ldc + n);
    float4 o = *cp;
    o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
    *cp = o;
  } else if (bias && i < nc4 + M) {
    const int64_t m = i - nc4;
    const int mt = (int)(m / 256), ml = (int)(m % 256);
    float a = 0.f;
    for (int sp = 0; sp < splits; ++sp)
      for (int nt = 0; nt < g.tiles_n; ++nt) {
        const float* p = sums + ((int64_t)(sp * g.tiles + mt * g.tiles_n + nt) * 8) * 256 + ml;
#pragma unroll
        for (int r = 0; r < 8; ++r) a += p[r * 256];
      }
    bias[m] += a;
  }
}

// the split count: every workgroup one item per round (256 slots), the busiest one's k-steps
// (plus ~4 steps' worth per item for its partial-tile store) minimised, partials <= 128 MB
struct Dw256Plan {
  bool valid;
  int splits;
  Dw256Map g;
};
static Dw256Plan plan_dw256(int64_t M, int64_t N, int64_t K) {
  Dw256Plan p = {};
  // 768 x 768 (the projection's dW) measured no faster than the split-K dW tiles: 326 vs 308 us
  if (M % 256 || N % 256 || K % 64 || K < 64 * 64 || (M * N <= 768 * 768 && knob(VS_KNOB_DW256_ALL) != 1)) return p;
  const int64_t tiles = (M / 256) * (N / 256), nk = K / 64;
  double best = 1e30;
  for (int64_t S0 = 1; S0 <= 256 && S0 * 8 <= nk; ++S0) {
    const int64_t kps = (nk + S0 - 1) / S0, S = (nk + kps - 1) / kps;  // no empty last split
    const int64_t items = tiles * S;
    if (items * 65536 * 4 > (128ll << 20)) break;
    const int64_t rounds = (items + 255) / 256;
    const double t = (double)rounds * (double)(kps + 4);
    if (t < best - 1e-9) {
      best = t;
      p.valid = true;
      p.splits = (int)S;
      p.g.kps = (int)kps;
    }
  }
  if (!p.valid) return p;
  p.g.tiles_n = (int)(N / 256);
  p.g.tiles = (int)tiles;
  p.g.items = (int)(tiles * p.splits);
  p.g.per_xcd = (p.g.items + 7) / 8;
  p.g.nk = (int)nk;
  return p;
}
static size_t dw256_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const Dw256Plan p = plan_dw256(M, N, K);
  return p.valid ? (size_t)p.g.items * (65536 + 8 * 256) * 4 : 0;
}

// ----------------------------------------------------------------------------------------------
// f32 kernel (exact: v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain)
// ----------------------------------------------------------------------------------------------
template <bool KC>
struct OperandF32 {
  static constexpr int R = 64, BK = 32, LD = 80;  // LD % 32 == 16 -> conflict-free ds_read_b32
  static constexpr int BYTES = BK * LD * 4;
  __device__ __forceinline__ static void load(float4 (&reg)[2], const float* __restrict__ p, int64_t ld, int64_t r0,
                                              int64_t rows, int64_t k0, int64_t k_end, int tid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = tid + 256 * s;
      int64_t gr, gk;
      if constexpr (KC) {
        gr = r0 + (i >> 3);
        gk = k0 + (i & 7) * 4;
      } else {
        gk = k0 + (i >> 4);
        gr = r0 + (i & 15) * 4;
      }
      const bool ok = gr < rows && gk < k_end;
      const float* src = KC ? p + gr * ld + gk : p + gk * ld + gr;
      reg[s] = ok ? *(const float4*)src : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ __forceinline__ static void store(float* lds, const float4 (&reg)[2], int tid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = tid + 256 * s;
      if constexpr (KC) {
        const int r = i >> 3, k = (i & 7) * 4;
        lds[(k + 0) * LD + r] = reg[s].x;
        lds[(k + 1) * LD + r] = reg[s].y;
        lds[(k + 2) * LD + r] = reg[s].z;
        lds[(k + 3) * LD + r] = reg[s].w;
      } else {
        const int k = i >> 4, r = (i & 15) * 4;
        *(float4*)(lds + k * LD + r) = reg[s];
      }
    }
  }
};

template <bool AKC, bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ B, int64_t ldb, int64_t K,
                                                          GridMap g, EpiParams e) {
  using OA = OperandF32<AKC>;
  using OB = OperandF32<BKC>;
  constexpr int LD = OA::LD;
  constexpr int STAGE = (OA::BYTES + OB::BYTES) / 4;  // floats
  constexpr int SMEM = CMax<2 * STAGE, 64 * 68>::v;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];

  int nt, mt, split;
  map_block(g, nt, mt, split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * 64, n0 = (int64_t)nt * 64;
  const int64_t k_begin = (int64_t)split * g.k_per_split;
  const int64_t k_end = k_begin + g.k_per_split < K ? k_begin + g.k_per_split : K;
  const int nk = (int)((k_end - k_begin + 31) / 32);

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool rowsum_on = e.a_rowsum != nullptr && nt == 0 && wc == 0;
  float rs[2] = {0.f, 0.f};

  float4 ra[2], rb[2];
  if (nk > 0) {
    OA::load(ra, A, lda, m0, e.M, k_begin, k_end, tid);
    OB::load(rb, B, ldb, n0, e.N, k_begin, k_end, tid);
    OA::store(smem, ra, tid);
    OB::store(smem + OA::BYTES / 4, rb, tid);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const float* sa = smem + (t & 1) * STAGE;
    const float* sb = sa + OA::BYTES / 4;
    const bool more = t + 1 < nk;
    if (more) {
      const int64_t kn = k_begin + (int64_t)(t + 1) * 32;
      OA::load(ra, A, lda, m0, e.M, kn, k_end, tid);
      OB::load(rb, B, ldb, n0, e.N, kn, k_end, tid);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = 4 * s + (lane >> 4);
      float af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = sa[k * LD + wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = sb[k * LD + wc * 32 + j * 16 + (lane & 15)];
      if (rowsum_on) {
        rs[0] += af[0];
        rs[1] += af[1];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      float* dst = smem + ((t + 1) & 1) * STAGE;
      OA::store(dst, ra, tid);
      OB::store(dst + OA::BYTES / 4, rb, tid);
    }
    __syncthreads();
  }
  if (rowsum_on) flush_rowsum<2>(e.a_rowsum, rs, m0 + wr * 32, e.M, lane);
  store_tile<64, 64, 2, 2, kEpiRuntime>(e, smem, acc, m0, n0, split);
}

// ----------------------------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------------------------
template <int BM, int BN, uint32_t EF>
static void launch_bf16_ef(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e, hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->a_kcontig && d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, true, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else if (d->a_kcontig)
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, true, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, false, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, false, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
}

template <int BM, int BN, int KT, uint32_t EF>
static void launch_bf16_fullk_ef(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e,
                                 hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->a_kcontig && d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_fullk_kernel<BM, BN, KT, true, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, g, e);
  else if (d->a_kcontig)
    hipLaunchKernelGGL((gemm_bf16_fullk_kernel<BM, BN, KT, true, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, g, e);
  else if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_fullk_kernel<BM, BN, KT, false, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, g, e);
  else
    hipLaunchKernelGGL((gemm_bf16_fullk_kernel<BM, BN, KT, false, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, g, e);
}

template <int BM, int BN, uint32_t EF>
static void launch_bf16_ring_ef(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e,
                                hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->a_kcontig && d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, true, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else if (d->a_kcontig)
    hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, true, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, false, true, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else
    hipLaunchKernelGGL((gemm_bf16_ring_kernel<BM, BN, false, false, EF>), dim3(nblk), dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
}

template <int KT, uint32_t EF>
static void launch_bf16_panel_ef(const vs_gemm_desc* d, unsigned grid, int64_t items, const EpiParams& e,
                                 hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_panel_kernel<KT, true, EF>), dim3(grid), dim3(256), 0, s, a, d->lda, b, d->ldb, items, e);
  else
    hipLaunchKernelGGL((gemm_bf16_panel_kernel<KT, false, EF>), dim3(grid), dim3(256), 0, s, a, d->lda, b, d->ldb, items, e);
}

// 8 waves x 128-row tiles once a workgroup's slab holds at least two of them (M >= 131,072 rows at
// the 512-workgroup grid: 128 clips of C2) and the W slice re-streamed per tile is the larger operand
// stream (K >= 384); 4 waves x 64 rows otherwise (VS_KNOB_SLAB_WV forces 4 / 8).  Measured at 128
// clips (per launch, 4 -> 8 waves): dh2 + LN2' 247 -> 218 us, dh1 + LN1' 222 -> 195, fc2 200 -> 198;
// the K = 192 products lose (proj + LN2 102 -> 107, do 40 -> 45).
static inline bool slab_wide(int64_t M, int64_t K, unsigned grid) {
  const int f = knob(VS_KNOB_SLAB_WV);
  if (f == 4 || f == 8) return f == 8;
  return M / (int64_t)grid >= 256 && K >= 384;
}
template <int NT, uint32_t EF, bool LNB = false, bool LNF = false>
static void launch_bf16_slab_ef(const vs_gemm_desc* d, unsigned grid, const EpiParams& e, hipStream_t s,
                                const LnBwdParams& ln = LnBwdParams{}) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (slab_wide(d->M, d->K, grid)) {
    if (d->b_kcontig)
      hipLaunchKernelGGL((gemm_bf16_slab_kernel<NT, true, EF, LNB, LNF, 8>), dim3(grid), dim3(512), 0, s, a, d->lda, b,
                         d->ldb, d->K, e, ln);
    else
      hipLaunchKernelGGL((gemm_bf16_slab_kernel<NT, false, EF, LNB, LNF, 8>), dim3(grid), dim3(512), 0, s, a, d->lda, b,
                         d->ldb, d->K, e, ln);
    return;
  }
  if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_slab_kernel<NT, true, EF, LNB, LNF>), dim3(grid), dim3(256), 0, s, a, d->lda, b,
                       d->ldb, d->K, e, ln);
  else
    hipLaunchKernelGGL((gemm_bf16_slab_kernel<NT, false, EF, LNB, LNF>), dim3(grid), dim3(256), 0, s, a, d->lda, b,
                       d->ldb, d->K, e, ln);
}
template <int NT>
static void launch_bf16_slab(const vs_gemm_desc* d, unsigned grid, const EpiParams& e, hipStream_t s) {
  switch (e.flags) {
    case 0: launch_bf16_slab_ef<NT, 0u>(d, grid, e, s); break;
    case VS_EPI_BIAS: launch_bf16_slab_ef<NT, (uint32_t)VS_EPI_BIAS>(d, grid, e, s); break;
    case VS_EPI_BIAS | VS_EPI_POS:  // the patch embedding + sinusoid table (K = 1536)
      launch_bf16_slab_ef<NT, (uint32_t)(VS_EPI_BIAS | VS_EPI_POS)>(d, grid, e, s);
      break;
    default: launch_bf16_slab_ef<NT, (uint32_t)(VS_EPI_BIAS | VS_EPI_RESIDUAL)>(d, grid, e, s); break;
  }
}

template <int KT, uint32_t EF>
static void launch_bf16_wslab_ef(const vs_gemm_desc* d, unsigned grid, const EpiParams& e, hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_wslab_kernel<KT, true, EF>), dim3(grid), dim3(256), 0, s, a, d->lda, b, d->ldb, e);
  else
    hipLaunchKernelGGL((gemm_bf16_wslab_kernel<KT, false, EF>), dim3(grid), dim3(256), 0, s, a, d->lda, b, d->ldb, e);
}
template <int KT>
static void launch_bf16_wslab(const vs_gemm_desc* d, unsigned grid, const EpiParams& e, hipStream_t s) {
  switch (e.flags) {
    case 0: launch_bf16_wslab_ef<KT, 0u>(d, grid, e, s); break;
    case VS_EPI_BIAS: launch_bf16_wslab_ef<KT, (uint32_t)VS_EPI_BIAS>(d, grid, e, s); break;
    case VS_EPI_BIAS | VS_EPI_GELU: launch_bf16_wslab_ef<KT, (uint32_t)(VS_EPI_BIAS | VS_EPI_GELU)>(d, grid, e, s); break;
    case VS_EPI_MUL_AUX: launch_bf16_wslab_ef<KT, (uint32_t)VS_EPI_MUL_AUX>(d, grid, e, s); break;
    default: launch_bf16_wslab_ef<KT, (uint32_t)VS_EPI_GELU_BWD>(d, grid, e, s); break;
  }
}

// the W-resident kernel addresses every operand through 32-bit buffer descriptors
static inline bool wres_extent_ok(int64_t M, std::initializer_list<int64_t> lds) {
  for (int64_t ld : lds)
    if (M * ld * 2 >= ((int64_t)1 << 31)) return false;
  return true;
}

template <uint32_t EF>
static void launch_bf16_wres_ef(const vs_gemm_desc* d, const EpiParams& e, hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  // VSPIKE_WRES_WV=8: 8 waves per workgroup (16 per CU sharing 2 W parts; the GELU' / aux-product
  // instantiations need > 128 VGPRs, so one workgroup per CU there).  Measured at 128 clips: qkv
  // 94.3 -> 95.2 us, fc1 + GELU 216 -> 225 us (more waves do not raise the store-bound rate): 4 waves.
  const bool wide = knob(VS_KNOB_WRES_WV) == 8;
  void (*kern)(const bf16_t*, int64_t, const bf16_t*, int64_t, EpiParams, int);
  if (d->b_kcontig) kern = wide ? gemm_bf16_wres_kernel<true, EF, 8> : gemm_bf16_wres_kernel<true, EF, 4>;
  else kern = wide ? gemm_bf16_wres_kernel<false, EF, 8> : gemm_bf16_wres_kernel<false, EF, 4>;
#ifdef VS_DEBUG_KNOBS
  // diagnostic builds only: VS_KNOB_WRES_DBG makes the kernel re-read / re-write L2-resident blocks
  // (timing isolation; the results are WRONG)
  const int dbg = knob(VS_KNOB_WRES_DBG);
#else
  const int dbg = 0;
#endif
  hipLaunchKernelGGL(kern, dim3(512), dim3(wide ? 512 : 256), 0, s, a, d->lda, b, d->ldb, e, dbg);
}

template <uint32_t EF>
static void launch_bf16_big_ef(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e,
                               hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  if (d->b_kcontig)
    hipLaunchKernelGGL((gemm_bf16_big_kernel<true, EF>), dim3(nblk), dim3(512), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  else
    hipLaunchKernelGGL((gemm_bf16_big_kernel<false, EF>), dim3(nblk), dim3(512), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
}

template <uint32_t EF>
static void launch_bf16_g256_ef(const vs_gemm_desc* d, const G256Map& g, unsigned grid, const EpiParams& e,
                                hipStream_t s) {
  const bf16_t* a = (const bf16_t*)d->a;
  const bf16_t* b = (const bf16_t*)d->b;
  // P8 (8-column epilogue vectors): always with K-contiguous B; with N-contiguous B only for bf16
  // outputs (its transposed B reads conflict 2-way, which the f32 outputs' 16-B quads do not repay:
  // dX fc2 1,603 -> 1,463 us, dX proj 310 -> 281; dX fc1 989 -> 1,011)
  G256Map gm = g;
  auto go = [&](auto kern) {
    // the early-DMA wait counts the epilogue's stores exactly (`est`); an instance that spills to scratch
    // issues more vector-memory ops than that, so it falls back to vmcnt(0) (checked once per instance)
    static const int ok = [&] {
      hipFuncAttributes fa{};
      return hipFuncGetAttributes(&fa, (const void*)kern) == hipSuccess && fa.localSizeBytes == 0 ? 1 : 0;
    }();
    gm.ed_ok = ok;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, a, d->lda, b, d->ldb, gm, e);
  };
  if (d->b_kcontig)
    go(gemm_bf16_g256_kernel<true, true, EF>);
  else if (e.out_bf16)
    go(gemm_bf16_g256_kernel<false, true, EF>);
  else
    go(gemm_bf16_g256_kernel<false, false, EF>);
}

// G256 early-DMA guard, for tests: 1 when every compiled 256 x 256 forward / dX instance has no private
// segment (the counted vmcnt of the early DMA is then exact), else 0
template <bool BKC, bool P8>
static int g256_no_scratch_all() {
  int ok = 1;
#define CHK_(EF)                                                                                    \
  {                                                                                                 \
    hipFuncAttributes fa{};                                                                          \
    if (hipFuncGetAttributes(&fa, (const void*)gemm_bf16_g256_kernel<BKC, P8, EF>) != hipSuccess || \
        fa.localSizeBytes != 0)                                                                     \
      ok = 0;                                                                                       \
  }
  CHK_(0u) CHK_((uint32_t)VS_EPI_BIAS) CHK_((uint32_t)(VS_EPI_BIAS | VS_EPI_RESIDUAL))
  CHK_((uint32_t)(VS_EPI_BIAS | VS_EPI_GELU)) CHK_((uint32_t)VS_EPI_GELU_BWD)
  CHK_((uint32_t)(VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD)) CHK_((uint32_t)VS_EPI_MUL_AUX)
#undef CHK_
  return ok;
}

// compile-time epilogue variants: the flag sets of the ViT block (vit_exec.hip) and patch embed
#define VS_EPI_SWITCH(F, CALL)                                                             \
  switch (F) {                                                                             \
    case 0: CALL(0u); break;                                                               \
    case VS_EPI_BIAS: CALL((uint32_t)VS_EPI_BIAS); break;                                  \
    case VS_EPI_BIAS | VS_EPI_RESIDUAL: CALL((uint32_t)(VS_EPI_BIAS | VS_EPI_RESIDUAL)); break; \
    case VS_EPI_BIAS | VS_EPI_GELU: CALL((uint32_t)(VS_EPI_BIAS | VS_EPI_GELU)); break;    \
    case VS_EPI_GELU_BWD: CALL((uint32_t)VS_EPI_GELU_BWD); break;                          \
    case VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD:                                     \
      CALL((uint32_t)(VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD)); break;               \
    case VS_EPI_MUL_AUX: CALL((uint32_t)VS_EPI_MUL_AUX); break;                            \
    default: CALL(kEpiRuntime); break;                                                     \
  }

extern "C" int vs_g256_scratch_free(void) {
  return g256_no_scratch_all<true, true>() & g256_no_scratch_all<false, true>() & g256_no_scratch_all<false, false>();
}

static void launch_bf16_g256(const vs_gemm_desc* d, const G256Map& g, unsigned grid, const EpiParams& e,
                             hipStream_t s) {
#define L_(EF) launch_bf16_g256_ef<EF>(d, g, grid, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

static void launch_bf16_big(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e, hipStream_t s) {
#define L_(EF) launch_bf16_big_ef<EF>(d, nblk, g, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

template <int BM, int BN>
static void launch_bf16(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e, hipStream_t s) {
#define L_(EF) launch_bf16_ef<BM, BN, EF>(d, nblk, g, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

template <int BM, int BN>
static void launch_bf16_ring(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e, hipStream_t s) {
#define L_(EF) launch_bf16_ring_ef<BM, BN, EF>(d, nblk, g, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

template <int KT>
static void launch_bf16_panel(const vs_gemm_desc* d, unsigned grid, int64_t items, const EpiParams& e, hipStream_t s) {
#define L_(EF) launch_bf16_panel_ef<KT, EF>(d, grid, items, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

template <int BM, int BN, int KT>
static void launch_bf16_fullk(const vs_gemm_desc* d, unsigned nblk, const GridMap& g, const EpiParams& e,
                              hipStream_t s) {
#define L_(EF) launch_bf16_fullk_ef<BM, BN, KT, EF>(d, nblk, g, e, s)
  VS_EPI_SWITCH(e.flags, L_)
#undef L_
}

// Split-K for the token reductions (dW): aim at ~2 blocks per CU, at least 8 k-tiles per split
// (the f32 atomics of every split's tile cost ~1.3 TB/s chip-wide: fewer, longer splits).
static int pick_splits(int64_t tiles, int64_t nk, int want, bool atomic_ok) {
  if (!atomic_ok) return 1;
  if (want > 0) return (int)(want < nk ? want : nk);
  if (tiles >= 384 || nk < 16) return 1;
  int64_t s = (512 + tiles - 1) / tiles;
  const int64_t max_s = nk / 8;
  if (s > max_s) s = max_s;
  return s < 1 ? 1 : (int)s;
}

// C[m, n] += bias[n] + sum_s part[s][m][n].  Vector path: a workgroup owns 64 float4 of C and
// its 4 waves split the splits (wave w sums s = w, w+4, ...: every load of a wave's share is
// issued before the first add), then the 4 partial float4 are added in wave order through LDS
// (deterministic: the order depends only on `splits`).  The dW partials are 7-13 MB spread over
// ~150 workgroups at one float4 per thread: that version was latency-bound at ~20 us per launch.
__global__ __launch_bounds__(256) void gemm_splitk_reduce(const float* __restrict__ part, int splits, int64_t M,
                                                          int64_t N, float* __restrict__ c, int64_t ldc,
                                                          const float* __restrict__ bias, int vec) {
  const int64_t MN = M * N;
  if (vec) {
    __shared__ float4 red[4][64];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int64_t e4 = ((int64_t)blockIdx.x * 64 + l) * 4;
    const bool live = e4 < MN;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
      for (int sp0 = w; sp0 < splits; sp0 += 4 * 16) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int sp = sp0 + 4 * u;
          v[u] = sp < splits ? *(const float4*)(part + sp * MN + e4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
        }
      }
    }
    red[w][l] = acc;
    __syncthreads();
    if (w == 0 && live) {
      float4 a = red[0][l];
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float4 b = red[k][l];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      const int64_t m = e4 / N, n = e4 % N;
      if (bias) {
        const float4 bb = *(const float4*)(bias + n);
        a.x += bb.x; a.y += bb.y; a.z += bb.z; a.w += bb.w;
      }
      float4* dst = (float4*)(c + m * ldc + n);
      float4 o = *dst;
      o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
      *dst = o;
    }
  } else {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= MN) return;
    const int64_t m = i / N, n = i % N;
    float acc = 0.f;
    for (int sp0 = 0; sp0 < splits; sp0 += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = sp0 + u < splits ? part[(sp0 + u) * MN + i] : 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
    if (bias) acc += bias[n];
    c[m * ldc + n] += acc;
  }
}

// Few outputs, many splits (the head's z = x W_enc^T: 16 x 64 outputs, 512 splits of K): the
// per-output kernel above runs as ONE workgroup whose threads each walk 512 splits (24 us).  Here a
// workgroup owns one float4 of C, its 256 threads stride over the splits, and a fixed-shape LDS tree
// adds the 256 partial sums (deterministic: the order depends only on `splits`).
__global__ __launch_bounds__(256) void gemm_splitk_reduce_wide(const float* __restrict__ part, int splits, int64_t M,
                                                               int64_t N, float* __restrict__ c, int64_t ldc,
                                                               const float* __restrict__ bias, int relu = 0) {
  __shared__ float4 red[256];
  const int64_t MN = M * N;
  const int64_t e4 = (int64_t)blockIdx.x * 4;
  const int t = threadIdx.x;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sp = t; sp < splits; sp += 256) {
    const float4 v = *(const float4*)(part + (int64_t)sp * MN + e4);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  red[t] = acc;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      const float4 o = red[t + w];
      float4 a = red[t];
      a.x += o.x; a.y += o.y; a.z += o.z; a.w += o.w;
      red[t] = a;
    }
    __syncthreads();
  }
  if (t == 0) {
    float4 s = red[0];
    const int64_t m = e4 / N, n = e4 % N;
    if (bias) {
      const float4 bb = *(const float4*)(bias + n);
      s.x += bb.x; s.y += bb.y; s.z += bb.z; s.w += bb.w;
    }
    float4* dst = (float4*)(c + m * ldc + n);
    float4 o = *dst;
    o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
    if (relu) {  // VS_EPI_ATOMIC | VS_EPI_RELU on the skinny path: C = relu(C + sum)
      o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
    }
    *dst = o;
  }
}

// tile / split geometry shared by vs_gemm and vs_gemm_splitk_workspace_bytes
struct GemmPlan {
  int BM, BN, BK;
  GridMap g;
};
static GemmPlan plan_gemm(int dtype, int64_t M, int64_t N, int64_t K, int want_split, bool atomic_ok,
                          int64_t ws_bytes) {
  GemmPlan p;
  if (dtype == VS_BF16) {
    p.BM = M <= 64 ? 64 : 128;
    p.BN = (N <= 64 || (N % 128 != 0 && N % 64 == 0 && N < 1024)) ? 64 : 128;
    p.BK = 64;
  } else {
    p.BM = p.BN = 64;
    p.BK = 32;
  }
  p.g.tiles_n = (int)cdiv(N, p.BN);
  p.g.tiles_m = (int)cdiv(M, p.BM);
  const int64_t nk = cdiv(K, p.BK);
  int splits = pick_splits((int64_t)p.g.tiles_n * p.g.tiles_m, nk, want_split, atomic_ok);
  if (ws_bytes > 0 && splits > 1) {  // partials must fit the workspace
    const int64_t fit = ws_bytes / (M * N * 4);
    if (splits > fit) splits = (int)(fit < 1 ? 1 : fit);
  }
  p.g.k_per_split = cdiv(nk, splits) * p.BK;
  p.g.splits = (int)(K > 0 ? cdiv(K, p.g.k_per_split) : 1);
  return p;
}

static bool vec_ok(const vs_gemm_desc* d) {
  const uint32_t f = d->epilogue;
  const int ovec = d->out_dtype == VS_BF16 ? 8 : 4;
  const int avec = d->dtype == VS_BF16 ? 8 : 4;
  bool ok = d->ldc % ovec == 0 && aligned16(d->c);
  if (f & VS_EPI_BIAS) ok = ok && aligned16(d->bias);
  if (f & VS_EPI_POS) ok = ok && aligned16(d->pos) && d->N % 4 == 0;
  if (f & VS_EPI_RESIDUAL) ok = ok && aligned16(d->residual) && d->ld_residual % 4 == 0;
  if (f & (VS_EPI_GELU_BWD | VS_EPI_RELU_BWD)) ok = ok && aligned16(d->aux_in) && d->ld_aux_in % avec == 0;
  if (f & VS_EPI_GELU) ok = ok && aligned16(d->aux_out) && d->ld_aux_out % avec == 0;
  return ok;
}

// Bytes a perfect kernel moves for this call (the roofline numerator): A and B read once, C written
// once (read too when accumulated into), every epilogue operand read / written once.
static double gemm_algorithmic_bytes(const vs_gemm_desc* d) {
  const double ea = esize(d->dtype), ec = esize(d->out_dtype), mn = (double)d->M * (double)d->N;
  const uint32_t f = d->epilogue;
  double b = ((double)d->M + (double)d->N) * (double)d->K * ea + mn * ec;
  if (f & (VS_EPI_ATOMIC | VS_EPI_ACCUM)) b += mn * 4.0;
  if (f & VS_EPI_BIAS) b += (double)d->N * 4.0;
  if (f & VS_EPI_RESIDUAL) b += mn * 4.0;
  if (f & VS_EPI_POS) b += (double)(d->pos_rows < d->M ? d->pos_rows : d->M) * (double)d->N * 4.0;
  if (f & (VS_EPI_GELU_BWD | VS_EPI_RELU_BWD | VS_EPI_MUL_AUX)) b += mn * ea;
  if (f & VS_EPI_GELU) b += mn * ea;
  if (d->a_rowsum) b += (double)d->M * 8.0;
  return b;
}

}  // namespace vs

// the same K split re-planned for 64-wide column tiles (ring kernel); splits as in the 128-wide
// plan, re-capped by the workspace (its size was computed for the plan's split count)
static vs::GridMap plan_gemm_bn64(const vs_gemm_desc* d, const vs::GridMap& g) {
  vs::GridMap r = g;
  r.tiles_n = (int)vs::cdiv(d->N, 64);
  return r;
}

extern "C" int vs_gemm(const vs_gemm_desc* d, void* stream) {
  using namespace vs;
  VS_REQUIRE(d != nullptr, "vs_gemm: null descriptor");
  VS_REQUIRE(d->dtype == VS_F32 || d->dtype == VS_BF16, "vs_gemm: dtype must be VS_F32 or VS_BF16");
  VS_REQUIRE(d->out_dtype == VS_F32 || d->out_dtype == VS_BF16, "vs_gemm: bad out_dtype");
  VS_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, "vs_gemm: negative extent");
  if (d->M == 0 || d->N == 0) return VS_OK;
  VS_REQUIRE(d->a && d->b && d->c, "vs_gemm: null operand");
  const uint32_t f = d->epilogue;
  const int vec = d->dtype == VS_BF16 ? 8 : 4;
  // contiguous extents and leading dims must allow 16-byte vector loads
  VS_REQUIRE(aligned16(d->a) && aligned16(d->b), "vs_gemm: operands must be 16-byte aligned");
  VS_REQUIRE(d->lda % vec == 0 && d->ldb % vec == 0, "vs_gemm: lda/ldb must be multiples of 16 bytes");
  VS_REQUIRE(d->a_kcontig ? (d->K % vec == 0 && d->lda >= d->K) : (d->M % vec == 0 && d->lda >= d->M),
             "vs_gemm: A contiguous extent must be a multiple of 16 bytes and <= lda");
  VS_REQUIRE(d->b_kcontig ? (d->K % vec == 0 && d->ldb >= d->K) : (d->N % vec == 0 && d->ldb >= d->N),
             "vs_gemm: B contiguous extent must be a multiple of 16 bytes and <= ldb");
  VS_REQUIRE(d->ldc >= d->N, "vs_gemm: ldc < N");
  VS_REQUIRE(!(f & VS_EPI_BIAS) || d->bias, "vs_gemm: BIAS needs bias");
  VS_REQUIRE(!(f & VS_EPI_RESIDUAL) || d->residual, "vs_gemm: RESIDUAL needs residual");
  VS_REQUIRE(!(f & VS_EPI_POS) || (d->pos && d->pos_rows > 0), "vs_gemm: POS needs pos/pos_rows");
  VS_REQUIRE(!(f & (VS_EPI_GELU_BWD | VS_EPI_RELU_BWD)) || d->aux_in, "vs_gemm: *_BWD needs aux_in");
  VS_REQUIRE(!(f & VS_EPI_GELU) || d->aux_out, "vs_gemm: GELU needs aux_out");
  VS_REQUIRE(!(f & (VS_EPI_ATOMIC | VS_EPI_ACCUM)) || d->out_dtype == VS_F32, "vs_gemm: ATOMIC/ACCUM need f32 C");
  VS_REQUIRE(!((f & VS_EPI_ATOMIC) && (f & ~(VS_EPI_ATOMIC | VS_EPI_BIAS | VS_EPI_RELU))),
             "vs_gemm: ATOMIC combines with BIAS (and RELU on the skinny split-K path) only");
  VS_REQUIRE(d->split_k <= 1 || (f & VS_EPI_ATOMIC), "vs_gemm: split_k > 1 needs VS_EPI_ATOMIC");

  EpiParams e;
  e.M = d->M; e.N = d->N; e.c = d->c; e.ldc = d->ldc;
  e.out_bf16 = d->out_dtype == VS_BF16; e.op_bf16 = d->dtype == VS_BF16;
  e.flags = f; e.alpha = d->alpha; e.bias = d->bias;
  e.residual = d->residual; e.ldr = d->ld_residual;
  e.pos = d->pos; e.pos_rows = d->pos_rows;
  e.aux_in = d->aux_in; e.ld_aux_in = d->ld_aux_in;
  e.aux_out = d->aux_out; e.ld_aux_out = d->ld_aux_out;
  e.vec_ok = vec_ok(d);
  e.a_rowsum = d->a_rowsum;
  e.part = nullptr;

  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : (f & VS_EPI_ATOMIC) ? VS_TIMER_GEMM_DW : VS_TIMER_GEMM, s,
                    gemm_algorithmic_bytes(d));
  const bool atomic_ok = (f & VS_EPI_ATOMIC) != 0;
  const bool use_ws = atomic_ok && d->workspace && d->workspace_bytes > 0 && aligned16(d->workspace);
  // token-reduction weight gradients (dW = dY^T X, both operands token-major): the long-K products
  // with 256-multiple widths on the 256 x 256 persistent kernel, the rest on the split-K dW kernel
  // (gemm_dw.hip); both reduce their partials in a fixed order
  if (!knob(VS_KNOB_NO_DW256) && d->dtype == VS_BF16 && d->out_dtype == VS_F32 && f == VS_EPI_ATOMIC &&
      !d->a_kcontig && !d->b_kcontig && d->split_k <= 0 && use_ws && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
      d->ldc % 4 == 0 && aligned16(d->c) && 64 * d->lda * 2 < (1ll << 31) && 64 * d->ldb * 2 < (1ll << 31)) {
    const Dw256Plan p = plan_dw256(d->M, d->N, d->K);
    if (p.valid && (size_t)d->workspace_bytes >= dw256_workspace_bytes(d->M, d->N, d->K)) {
      count_path(VS_PATH_GEMM_DW256);
      float* part = (float*)d->workspace;
      float* sums = part + (int64_t)p.g.items * 65536;
      const unsigned grid = p.g.items < 256 ? (unsigned)((p.g.items + 7) / 8 * 8) : 256u;
      if (d->a_rowsum)
        hipLaunchKernelGGL((gemm_dw256_kernel<true>), dim3(grid), dim3(512), 0, s, (const bf16_t*)d->a, d->lda,
                           (const bf16_t*)d->b, d->ldb, p.g, part, sums);
      else
        hipLaunchKernelGGL((gemm_dw256_kernel<false>), dim3(grid), dim3(512), 0, s, (const bf16_t*)d->a, d->lda,
                           (const bf16_t*)d->b, d->ldb, p.g, part, sums);
      const int64_t n = d->M * d->N / 4 + (d->a_rowsum ? d->M : 0);
      hipLaunchKernelGGL(gemm_dw256_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, sums, p.g,
                         p.splits, d->M, d->N, (float*)d->c, d->ldc, d->a_rowsum);
      VS_LAUNCH_CHECK();
      return VS_OK;
    }
  }
  if (!knob(VS_KNOB_DW_OLD) && d->dtype == VS_BF16 && d->out_dtype == VS_F32 && f == VS_EPI_ATOMIC && !d->a_kcontig &&
      !d->b_kcontig && d->split_k <= 0 && use_ws && d->K >= 1 && d->M % 8 == 0 && d->N % 8 == 0 &&
      d->lda % 8 == 0 && d->ldb % 8 == 0 && (size_t)d->workspace_bytes >= dw_workspace_bytes(d->M, d->N, d->K))
    return count_path(VS_PATH_GEMM_DW), launch_dw(d, s);
  // skinny split-K with K-contiguous operands (the head forward): fragments straight from HBM
  const bool dense_c = d->ldc == d->N && aligned16(d->c) && (!(f & VS_EPI_BIAS) || aligned16(d->bias));
  const bool skinny = !knob(VS_KNOB_NO_SKINNY) && use_ws && dense_c && skinny_ok(d) &&
                      (size_t)d->workspace_bytes >= skinny_workspace_bytes(d->dtype, d->M, d->N, d->K);
  VS_REQUIRE(skinny || !((f & VS_EPI_ATOMIC) && (f & VS_EPI_RELU)),
             "vs_gemm: ATOMIC|RELU needs the skinny split-K path (M <= 64, N <= 256, K-contiguous, workspace)");
  if (skinny) {
    int S = 0;
    count_path(VS_PATH_GEMM_SKINNY);
    VS_CALL(launch_skinny(d, s, &S));
    const int64_t n4 = d->M * d->N / 4;
    hipLaunchKernelGGL(gemm_splitk_reduce_wide, dim3((unsigned)n4), dim3(256), 0, s, (const float*)d->workspace, S, d->M,
                       d->N, (float*)d->c, d->ldc, (f & VS_EPI_BIAS) ? d->bias : nullptr, (f & VS_EPI_RELU) ? 1 : 0);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  // row-slab path: N <= 192 outputs of a large-M, K-contiguous-A product, no split / reduction
  if (!knob(VS_KNOB_NO_SLAB) && d->dtype == VS_BF16 && d->a_kcontig && (d->N == 64 || d->N == 128 || d->N == 192) &&
      d->K % 64 == 0 && d->K >= 64 && d->M >= 8192 && d->split_k <= 1 && !d->a_rowsum && e.vec_ok &&
      (f == 0 || f == VS_EPI_BIAS || f == (VS_EPI_BIAS | VS_EPI_RESIDUAL) || f == (VS_EPI_BIAS | VS_EPI_POS))) {
    const int64_t G = d->M / 16 < 512 ? d->M / 16 : 512;
    count_path(VS_PATH_GEMM_SLAB);
    if (d->N == 64) launch_bf16_slab<1>(d, (unsigned)G, e, s);
    else if (d->N == 128) launch_bf16_slab<2>(d, (unsigned)G, e, s);
    else launch_bf16_slab<3>(d, (unsigned)G, e, s);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  // 256 x 256 persistent path: long-M ViT-Base block products (N % 256 == 0, K % 64 == 0, rows
  // and leading dims addressable with 32-bit per-lane DMA offsets)
  const bool g256_ef = f == 0 || f == VS_EPI_BIAS || f == (VS_EPI_BIAS | VS_EPI_RESIDUAL) ||
                       f == (VS_EPI_BIAS | VS_EPI_GELU) || f == VS_EPI_GELU_BWD ||
                       f == (VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD) || f == VS_EPI_MUL_AUX;
  const int g256k = knob(VS_KNOB_G256);
  // measured per C3 product: the 256 x 256 kernel wins where N or K >= 2304 and
  // on the bf16-output dX products (fc2's GELU' product, proj); the 768 x 768 forward proj stays on the
  // 256 x 128 tile
  const bool g256_pick = g256k == 1 || (g256k == 0 && ((d->N >= 2304 || d->K >= 2304) || (!d->b_kcontig && e.out_bf16)));
  if (g256_pick && g256_ef && d->dtype == VS_BF16 && e.op_bf16 &&
      d->a_kcontig && d->M >= 16384 && d->N % 256 == 0 &&
      d->K >= 256 && d->K % 64 == 0 && d->split_k <= 1 && !d->a_rowsum && e.vec_ok && d->ldc % 4 == 0 &&
      !(f & (VS_EPI_ATOMIC)) && 256 * d->lda * 2 < (1ll << 31) && (d->b_kcontig ? d->N * d->ldb : d->K * d->ldb) * 2 <
      (1ll << 31)) {
    G256Map g;
    g.tiles_n = (int)(d->N / 256);
    g.tiles = (int)(cdiv(d->M, 256) * g.tiles_n);
    g.nk = (int)(d->K / 64);
    const int gcap = knob(VS_KNOB_G256_GRID) > 0 ? knob(VS_KNOB_G256_GRID) : 256;
    int grid = g.tiles < gcap ? (g.tiles + 7) / 8 * 8 : gcap;
    grid = grid < 8 ? 8 : grid / 8 * 8;
    g.per_xcd = (int)cdiv(g.tiles, 8);
#ifdef VS_DEBUG_KNOBS
    g.dbg = knob(VS_KNOB_G256_DBG);
#else
    g.dbg = 0;
#endif
    g.stagger = knob(VS_KNOB_G256_STAGGER);
    g.ed_ok = 1;  // launch_bf16_g256_ef clears it for an instance with a private segment
    g.a3 = knob(VS_KNOB_G256_A3) != 2;  // default on (round 6: every forward / dX product faster)
    count_path(VS_PATH_GEMM_G256);
    launch_bf16_g256(d, g, (unsigned)grid, e, s);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  // big-tile path: MFMA-heavy products (K >= 512, N >= 512, N % 128 == 0: the ViT-Base block)
  if (!knob(VS_KNOB_NO_BIG) && d->dtype == VS_BF16 && d->a_kcontig && d->M >= 4096 && d->N >= 512 && d->N % 128 == 0 &&
      d->K >= 512 && d->K % 64 == 0 && d->split_k <= 1 && !d->a_rowsum && e.vec_ok &&
      !(f & (VS_EPI_ATOMIC | VS_EPI_ACCUM))) {
    GridMap g;
    g.tiles_m = (int)cdiv(d->M, 256);
    g.tiles_n = (int)(d->N / 128);
    g.splits = 1;
    g.k_per_split = d->K;
    count_path(VS_PATH_GEMM_BIG);
    launch_bf16_big(d, (unsigned)((int64_t)g.tiles_m * g.tiles_n), g, e, s);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  // W-resident path: K = 192, N a multiple of 192 (>= 384): qkv, fc1 + GELU, the GELU' product
  {
    const bool no_wres = knob(VS_KNOB_NO_WRES) != 0;
    // the GELU' product (GELU_BWD, or MUL_AUX on the stored gelu') stays on the wide row-slab kernel
    // unless VSPIKE_WRES_GBWD=1: 35.7 vs 41.2 us (GELU_BWD), 27.8 vs 32.6 us (MUL_AUX) there — its
    // operand stream (a 16-B aux read per 8 outputs) overlaps better with the row-slab schedule
    const bool gbwd = knob(VS_KNOB_WRES_GBWD) != 0;
    const bool ef_ok = (f == VS_EPI_BIAS || f == (VS_EPI_BIAS | VS_EPI_GELU) || f == 0 ||
                        f == (VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD) ||
                        (gbwd && (f == VS_EPI_GELU_BWD || f == VS_EPI_MUL_AUX))) &&
                       e.op_bf16 && e.out_bf16;
    if (!no_wres && ef_ok && d->dtype == VS_BF16 && d->a_kcontig && d->K == 192 && d->N % kWresNH == 0 &&
        d->N >= 2 * kWresNH && d->N <= 64 * kWresNH && d->M >= 8192 && d->split_k <= 1 && !d->a_rowsum && e.vec_ok && d->lda % 8 == 0 &&
        d->ldb % 8 == 0 && aligned16(d->a) && aligned16(d->b) &&
        wres_extent_ok(d->M, {d->lda, d->ldc, e.aux_out ? e.ld_aux_out : 0, e.aux_in ? e.ld_aux_in : 0})) {
      count_path(VS_PATH_GEMM_WRES);
      if (f == VS_EPI_BIAS) launch_bf16_wres_ef<(uint32_t)VS_EPI_BIAS>(d, e, s);
      else if (f == (VS_EPI_BIAS | VS_EPI_GELU)) launch_bf16_wres_ef<(uint32_t)(VS_EPI_BIAS | VS_EPI_GELU)>(d, e, s);
      else if (f == 0) launch_bf16_wres_ef<0u>(d, e, s);
      else if (f == (VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD))
        launch_bf16_wres_ef<(uint32_t)(VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD)>(d, e, s);
      else if (f == VS_EPI_MUL_AUX) launch_bf16_wres_ef<(uint32_t)VS_EPI_MUL_AUX>(d, e, s);
      else launch_bf16_wres_ef<(uint32_t)VS_EPI_GELU_BWD>(d, e, s);
      VS_LAUNCH_CHECK();
      return VS_OK;
    }
  }
  // wide row-slab path: K <= 192, N > 192 (qkv, fc1 + GELU, the GELU' dX product)
  // Measured (scripts/microbench.py, bench shapes): faster than the panel kernel for the GELU'
  // product (39.7 -> 36.8 us), slower than the whole-K tile kernel for the store-bound forward
  // products (qkv 19.0 -> 22.2, fc1 + GELU 37.9 -> 41.2 us), which therefore stay on it unless
  // VSPIKE_WSLAB=1 forces this path for every eligible epilogue.
  const int all_wslab = knob(VS_KNOB_WSLAB);
  if (!knob(VS_KNOB_NO_WSLAB) && d->dtype == VS_BF16 && d->a_kcontig && d->N % 64 == 0 && d->N > 192 &&
      (d->K == 64 || d->K == 128 || d->K == 192) && d->M >= 8192 && d->split_k <= 1 && !d->a_rowsum && e.vec_ok &&
      (f == VS_EPI_GELU_BWD || (f == VS_EPI_MUL_AUX && e.op_bf16) ||
       (all_wslab && (f == 0 || f == VS_EPI_BIAS || f == (VS_EPI_BIAS | VS_EPI_GELU))))) {
    const int gw = knob(VS_KNOB_WSLAB_G) > 0 ? knob(VS_KNOB_WSLAB_G) : 512;
    count_path(VS_PATH_GEMM_WSLAB);
    const int64_t G = d->M / 16 < gw ? d->M / 16 : gw;
    if (d->K == 64) launch_bf16_wslab<1>(d, (unsigned)G, e, s);
    else if (d->K == 128) launch_bf16_wslab<2>(d, (unsigned)G, e, s);
    else launch_bf16_wslab<3>(d, (unsigned)G, e, s);
    VS_LAUNCH_CHECK();
    return VS_OK;
  }
  const GemmPlan plan = plan_gemm(d->dtype, d->M, d->N, d->K, d->split_k, atomic_ok, use_ws ? d->workspace_bytes : 0);
  const GridMap& g = plan.g;
  if (use_ws && g.splits > 1) e.part = (float*)d->workspace;
  if (d->dtype == VS_BF16) {
    const int BM = plan.BM, BN = plan.BN;
    const int64_t nblk = (int64_t)g.tiles_n * g.tiles_m * g.splits;
    VS_REQUIRE(nblk < (1ll << 31), "vs_gemm: grid too large");
    // whole-K-in-LDS path: K = 64..192 in 64-steps, no split, no fused row sums, 128 x 64 tiles
    // (72 KB of LDS at K = 192: 2 blocks per CU)
    // row-panel path (K <= 192, whole 64-column chunks, no split / row sums / atomics).  Measured
    // (scripts/microbench.py, ViT-Tiny shapes): faster than the per-tile kernels only for the
    // GELU' product (da: 43.2 -> 38.7 us); the per-tile whole-K kernel wins on the others (its
    // 2352 short tiles balance better than 512 persistent workgroups that each load a 48-KB A panel
    // before their first MFMA).  VSPIKE_PANEL=1 forces it for every eligible shape.
    const bool panel = ((f & VS_EPI_GELU_BWD) || knob(VS_KNOB_PANEL)) && d->a_kcontig && g.splits == 1 && d->K % 64 == 0 && d->K >= 64 && d->K <= 192 &&
                       d->N % 64 == 0 && !d->a_rowsum && !(f & (VS_EPI_ATOMIC | VS_EPI_ACCUM)) && e.vec_ok &&
                       knob(VS_KNOB_NO_PANEL) == 0;
    if (panel) {
      const int64_t items = cdiv(d->M, 128) * (d->N / 64);
      const int gcap = knob(VS_KNOB_PANEL_GRID) > 0 ? knob(VS_KNOB_PANEL_GRID) : 512;
      count_path(VS_PATH_GEMM_PANEL);
      const unsigned grid = (unsigned)(items < gcap ? items : gcap);
      const int KT = (int)(d->K / 64);
      if (KT == 1) launch_bf16_panel<1>(d, grid, items, e, s);
      else if (KT == 2) launch_bf16_panel<2>(d, grid, items, e, s);
      else launch_bf16_panel<3>(d, grid, items, e, s);
      VS_LAUNCH_CHECK();
      return VS_OK;
    }
    const bool fullk = g.splits == 1 && d->K % 64 == 0 && d->K >= 64 && d->K <= 192 && BM == 128 && !d->a_rowsum &&
                       !(f & VS_EPI_ATOMIC) && knob(VS_KNOB_NO_FULLK) == 0;
    if (fullk) {
      GridMap gf = g;
      gf.tiles_n = (int)cdiv(d->N, 64);
      const int64_t nbf = (int64_t)gf.tiles_n * gf.tiles_m;
      const int KT = (int)(d->K / 64);
      count_path(VS_PATH_GEMM_FULLK);
      if (KT == 1) launch_bf16_fullk<128, 64, 1>(d, (unsigned)nbf, gf, e, s);
      else if (KT == 2) launch_bf16_fullk<128, 64, 2>(d, (unsigned)nbf, gf, e, s);
      else launch_bf16_fullk<128, 64, 3>(d, (unsigned)nbf, gf, e, s);
    } else if (d->K % 64 == 0 && knob(VS_KNOB_NO_RING) == 0) {
      count_path(VS_PATH_GEMM_RING);
      // long K: 3-stage DMA ring, BN = 64 tiles (72 KB of LDS at BM = 128: 2 blocks per CU)
      GridMap gr = plan_gemm_bn64(d, g);
      const int64_t nbr = (int64_t)gr.tiles_n * gr.tiles_m * gr.splits;
      if (BM == 128) launch_bf16_ring<128, 64>(d, (unsigned)nbr, gr, e, s);
      else launch_bf16_ring<64, 64>(d, (unsigned)nbr, gr, e, s);
    } else if (BM == 128 && BN == 128) {
      count_path(VS_PATH_GEMM_TILE);
      launch_bf16<128, 128>(d, (unsigned)nblk, g, e, s);
    } else if (BM == 128) {
      count_path(VS_PATH_GEMM_TILE);
      launch_bf16<128, 64>(d, (unsigned)nblk, g, e, s);
    } else if (BN == 128) {
      count_path(VS_PATH_GEMM_TILE);
      launch_bf16<64, 128>(d, (unsigned)nblk, g, e, s);
    } else {
      count_path(VS_PATH_GEMM_TILE);
      launch_bf16<64, 64>(d, (unsigned)nblk, g, e, s);
    }
  } else {
    const int64_t nblk = (int64_t)g.tiles_n * g.tiles_m * g.splits;
    VS_REQUIRE(nblk < (1ll << 31), "vs_gemm: grid too large");
    const float* a = (const float*)d->a;
    const float* b = (const float*)d->b;
    dim3 grid((unsigned)nblk);
    count_path(VS_PATH_GEMM_F32);
    if (d->a_kcontig && d->b_kcontig)
      hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
    else if (d->a_kcontig)
      hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
    else if (d->b_kcontig)
      hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
    else
      hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(256), 0, s, a, d->lda, b, d->ldb, d->K, g, e);
  }
  if (e.part) {
    const int vec = d->N % 4 == 0 && d->ldc % 4 == 0 && aligned16(d->c) && (!(f & VS_EPI_BIAS) || aligned16(d->bias));
    const int64_t n_items = vec ? d->M * d->N / 4 : d->M * d->N;
    if (vec && g.splits >= 64 && n_items <= 4096)
      hipLaunchKernelGGL(gemm_splitk_reduce_wide, dim3((unsigned)n_items), dim3(256), 0, s, e.part, g.splits, d->M,
                         d->N, (float*)d->c, d->ldc, (f & VS_EPI_BIAS) ? d->bias : nullptr);
    else
      hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)cdiv(n_items, vec ? 64 : 256)), dim3(256), 0, s, e.part, g.splits,
                       d->M, d->N, (float*)d->c, d->ldc, (f & VS_EPI_BIAS) ? d->bias : nullptr, vec);
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_patch_embed_fwd(int64_t B, int64_t F, int64_t C, int64_t H, int64_t W, int64_t tubelet,
                                  int64_t patch, const float* pixels, const void* weight, const float* bias,
                                  const float* pos, int64_t D, float* out, void* cols, void* stream) {
  using namespace vs;
  VS_REQUIRE(pixels && weight && bias && pos && out, "vs_patch_embed_fwd: null pointer");
  VS_REQUIRE(tubelet == 2 && patch == 16, "vs_patch_embed_fwd: the fused path is built for tubelet 2, patch 16");
  VS_REQUIRE(B > 0 && F % 2 == 0 && H % 16 == 0 && W % 16 == 0 && C >= 1 && C <= 8,
             "vs_patch_embed_fwd: frames / size must divide by the tubelet / patch");
  VS_REQUIRE(D == 64 || D == 128 || D == 192, "vs_patch_embed_fwd: D must be 64, 128 or 192 (one row slab)");
  VS_REQUIRE(aligned16(pixels) && aligned16(weight) && aligned16(bias) && aligned16(pos) && aligned16(out) &&
                 (!cols || aligned16(cols)),
             "vs_patch_embed_fwd: pointers must be 16-byte aligned");
  const int64_t n_tok = (F / 2) * (H / 16) * (W / 16), M = B * n_tok, K = C * 512;
  VS_REQUIRE(B * F * C * H * W < (1ll << 40), "vs_patch_embed_fwd: batch too large");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_MISC, s,
                    (double)M * (double)K * (4.0 + (cols ? 2.0 : 0.0)) + (double)D * (double)K * 2.0 +
                        (double)M * (double)D * 4.0 + (double)n_tok * (double)D * 4.0);
  EpiParams e = {};
  e.M = M; e.N = D; e.c = out; e.ldc = D; e.out_bf16 = 0; e.op_bf16 = 1; e.flags = VS_EPI_BIAS | VS_EPI_POS;
  e.alpha = 1.0f; e.bias = bias; e.pos = pos; e.pos_rows = n_tok; e.vec_ok = 1;
  PatchGeo g;
  g.F = (int)F; g.C = (int)C; g.H = (int)H; g.W = (int)W;
  g.n_tok = (int)n_tok; g.HpWp = (int)((H / 16) * (W / 16)); g.Wp = (int)(W / 16);
  const int64_t G = M / 16 < 512 ? (M / 16 > 0 ? M / 16 : 1) : 512;
  count_path(VS_PATH_PATCH_FUSED);
  const bf16_t* w = (const bf16_t*)weight;
#define PF_(NT_, CO_)                                                                                        \
  hipLaunchKernelGGL((patch_embed_fwd_kernel<NT_, CO_>), dim3((unsigned)G), dim3(256), 0, s, pixels, g, w, K, e, \
                     (bf16_t*)cols)
  if (D == 64) { if (cols) PF_(1, true); else PF_(1, false); }
  else if (D == 128) { if (cols) PF_(2, true); else PF_(2, false); }
  else { if (cols) PF_(3, true); else PF_(3, false); }
#undef PF_
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" size_t vs_patch_embed_dw_workspace_bytes(int64_t tokens, int64_t D, int64_t K) {
  return vs::dw_workspace_bytes(D, K, tokens);
}

// The patch embedding's weight gradient without cols (mv:176-181): dW[D][K] += dx^T gather(pixels),
// db[D] += column sums of dx — gemm_dw_kernel with the tubelet gather in its B-operand load
// (gemm_dw.hip), bitwise equal to vs_patch_im2col + the dW product of vs_gemm.
extern "C" int vs_patch_embed_dw(int64_t B, int64_t F, int64_t C, int64_t H, int64_t W, int64_t tubelet, int64_t patch,
                                 const float* pixels, const void* dx, int64_t lddx, int64_t D, float* dweight,
                                 int64_t ldw, float* dbias, void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace vs;
  VS_REQUIRE(pixels && dx && dweight && workspace, "vs_patch_embed_dw: null pointer");
  VS_REQUIRE(tubelet == 2 && patch == 16, "vs_patch_embed_dw: built for tubelet 2, patch 16");
  VS_REQUIRE(B > 0 && F % 2 == 0 && H % 16 == 0 && W % 16 == 0 && C >= 1 && C <= 8,
             "vs_patch_embed_dw: frames / size must divide by the tubelet / patch");
  VS_REQUIRE(D % 64 == 0 && D >= 64 && D <= 1024 && lddx % 8 == 0 && lddx >= D && ldw >= C * 512,
             "vs_patch_embed_dw: D must be a multiple of 64, dx rows 16-byte aligned");
  VS_REQUIRE(aligned16(pixels) && aligned16(dx) && aligned16(workspace), "vs_patch_embed_dw: pointers must be 16-byte aligned");
  const int64_t n_tok = (F / 2) * (H / 16) * (W / 16), M = B * n_tok, K = C * 512;
  VS_REQUIRE(M < (1ll << 24), "vs_patch_embed_dw: more than 2^24 tokens per launch");
  VS_REQUIRE(B * F * C * H * W < (1ll << 40), "vs_patch_embed_dw: batch too large");
  VS_REQUIRE((size_t)workspace_bytes >= dw_workspace_bytes(D, K, M), "vs_patch_embed_dw: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  // algorithmic bytes: the pixels once (f32), dx (bf16), dW / db read + written
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM_DW, s,
                    (double)M * (double)K * 4.0 + (double)M * (double)D * 2.0 + (double)D * (double)K * 8.0 +
                        (dbias ? (double)D * 8.0 : 0.0));
  PatchDwGeo g;
  g.F = (int)F; g.C = (int)C; g.H = (int)H; g.W = (int)W;
  g.n_tok = (int)n_tok; g.HpWp = (int)((H / 16) * (W / 16)); g.Wp = (int)(W / 16);
  g.inv_ntok = 1.0f / (float)g.n_tok; g.inv_hpwp = 1.0f / (float)g.HpWp; g.inv_wp = 1.0f / (float)g.Wp;
  count_path(VS_PATH_PATCH_DW);
  return launch_patch_dw((const bf16_t*)dx, lddx, D, pixels, g, M, K, dweight, ldw, dbias, (float*)workspace, s);
}

extern "C" int vs_gemm_ln_fwd(const vs_gemm_desc* d, const float* gamma, const float* beta, float eps, void* h,
                              int64_t ldh, float* mean, float* rstd, void* stream) {
  using namespace vs;
  VS_REQUIRE(d && gamma && beta && h && mean && rstd, "vs_gemm_ln_fwd: null pointer");
  VS_REQUIRE((d->epilogue & ~(uint32_t)VS_EPI_BIAS) == VS_EPI_RESIDUAL && d->out_dtype == VS_F32 && d->split_k <= 1 &&
                 !d->a_rowsum,
             "vs_gemm_ln_fwd: the product is y = x W^T (+ bias) + residual, f32 out");
  if (d->M == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t M = d->M, N = d->N;
  VS_REQUIRE(d->a && d->b && d->c && d->residual, "vs_gemm_ln_fwd: null operand");
  VS_REQUIRE(d->ldc >= N && d->ld_residual >= N && ldh >= N, "vs_gemm_ln_fwd: ldc / ld_residual / ldh < N");
  VS_REQUIRE(!(d->epilogue & VS_EPI_BIAS) || d->bias, "vs_gemm_ln_fwd: BIAS needs bias");
  const bool fused = !knob(VS_KNOB_NO_LNF_FUSE) && d->dtype == VS_BF16 && d->a_kcontig && N == 192 && d->K % 64 == 0 && d->K >= 64 &&
                     M >= 8192 && aligned16(d->a) && aligned16(d->b) && d->lda % 8 == 0 && d->ldb % 8 == 0 &&
                     d->lda >= d->K && (d->b_kcontig ? d->ldb >= d->K : d->ldb >= N) && aligned16(d->c) &&
                     d->ldc % 4 == 0 && aligned16(d->residual) && d->ld_residual % 4 == 0 &&
                     (!(d->epilogue & VS_EPI_BIAS) || aligned16(d->bias)) && aligned16(gamma) && aligned16(beta) &&
                     (((uintptr_t)h) & 7) == 0 && ldh % 4 == 0;
  if (!fused) {  // the same two GPU launches, unfused
    VS_CALL(vs_gemm(d, stream));
    return vs_layernorm_fwd(VS_BF16, M, N, (const float*)d->c, d->ldc, gamma, beta, eps, h, ldh, mean, rstd, stream);
  }
  const double ea = esize(d->dtype);
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM, s,
                    (double)(M + N) * (double)d->K * ea + (double)M * (double)N * (4.0 + 4.0 + 2.0) +
                        (double)M * 8.0 + (double)N * 12.0);
  EpiParams e = {};
  e.M = M; e.N = N; e.alpha = d->alpha; e.vec_ok = 1;
  e.c = d->c; e.ldc = d->ldc; e.out_bf16 = 0; e.flags = d->epilogue;
  e.bias = d->bias; e.residual = d->residual; e.ldr = d->ld_residual;
  LnBwdParams ln = {};
  ln.gamma = gamma; ln.beta = beta; ln.eps = eps; ln.h = (bf16_t*)h; ln.ldh = ldh; ln.mean_out = mean; ln.rstd_out = rstd;
  const int64_t G = M / 16 < 512 ? M / 16 : 512;
  count_path(VS_PATH_GEMM_LN_FWD);
  if (d->epilogue & VS_EPI_BIAS) launch_bf16_slab_ef<3, (uint32_t)(VS_EPI_BIAS | VS_EPI_RESIDUAL), false, true>(d, (unsigned)G, e, s, ln);
  else launch_bf16_slab_ef<3, (uint32_t)VS_EPI_RESIDUAL, false, true>(d, (unsigned)G, e, s, ln);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_gemm_ln_bwd(const vs_gemm_desc* d, const float* x, int64_t ldx, const float* mean,
                              const float* rstd, const float* gamma, const float* dres, int64_t lddres, float* dx,
                              int64_t lddx, void* dx_lp, float* dgamma, float* dbeta, void* workspace, void* stream) {
  using namespace vs;
  VS_REQUIRE(d && x && mean && rstd && gamma && dx && dgamma && dbeta, "vs_gemm_ln_bwd: null pointer");
  VS_REQUIRE(d->epilogue == 0 && d->split_k <= 1 && !d->a_rowsum, "vs_gemm_ln_bwd: the product takes no epilogue");
  if (d->M == 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t M = d->M, N = d->N;
  VS_REQUIRE(d->a && d->b, "vs_gemm_ln_bwd: null operand");
  VS_REQUIRE(ldx >= N && lddx >= N && (!dres || lddres >= N), "vs_gemm_ln_bwd: ldx / lddx / lddres < N");
  const bool fused = !knob(VS_KNOB_NO_LN_FUSE) && d->dtype == VS_BF16 && d->a_kcontig && (N == 64 || N == 128 || N == 192) &&
                     d->K % 64 == 0 && d->K >= 64 && M >= 8192 && workspace &&
                     aligned16(d->a) && aligned16(d->b) && d->lda % 8 == 0 && d->ldb % 8 == 0 && d->lda >= d->K &&
                     (d->b_kcontig ? d->ldb >= d->K : d->ldb >= N) && aligned16(x) && ldx % 4 == 0 && aligned16(dx) &&
                     lddx % 4 == 0 && aligned16(gamma) && (!dres || (aligned16(dres) && lddres % 4 == 0)) &&
                     (!dx_lp || (((uintptr_t)dx_lp) & 7) == 0);
  if (!fused) {
    VS_REQUIRE(d->c && d->out_dtype == VS_F32, "vs_gemm_ln_bwd: the unfused path needs an f32 scratch d->c");
    VS_CALL(vs_gemm(d, stream));
    return vs_layernorm_bwd(M, N, (const float*)d->c, d->ldc, x, ldx, mean, rstd, gamma, dres, lddres, dx, lddx, dx_lp,
                            dgamma, dbeta, workspace, stream);
  }
  const double ea = esize(d->dtype);
  // minimal bytes: A and W, then per output element x (f32 read), dres (f32 read), dx (f32 write) and
  // its bf16 copy; dh itself never leaves the chip (round 3 charged 4 B more per element: VERDICT r3)
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM, s,
                    (double)(M + N) * (double)d->K * ea + (double)M * (double)N * (8.0 + (dres ? 4.0 : 0.0) +
                    (dx_lp ? 2.0 : 0.0)) + (double)M * 8.0 + (double)N * 20.0);
  EpiParams e = {};
  e.M = M; e.N = N; e.alpha = d->alpha; e.vec_ok = 1;
  LnBwdParams ln;
  ln.x = x; ln.ldx = ldx; ln.mean = mean; ln.rstd = rstd; ln.gamma = gamma; ln.dres = dres; ln.ldr = lddres;
  ln.dx = dx; ln.lddx = lddx; ln.dx_lp = (bf16_t*)dx_lp; ln.part = (float*)workspace;
  const int64_t G = M / 16 < 512 ? M / 16 : 512;  // <= the 1024 partial rows of the LN workspace
  count_path(VS_PATH_GEMM_LN_BWD);
  if (N == 64) launch_bf16_slab_ef<1, 0u, true>(d, (unsigned)G, e, s, ln);
  else if (N == 128) launch_bf16_slab_ef<2, 0u, true>(d, (unsigned)G, e, s, ln);
  else launch_bf16_slab_ef<3, 0u, true>(d, (unsigned)G, e, s, ln);
  launch_ln_partsum((const float*)workspace, (int)G, (int)N, dgamma, dbeta, s);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" size_t vs_gemm_splitk_workspace_bytes(int32_t dtype, int64_t M, int64_t N, int64_t K) {
  using namespace vs;
  if (M <= 0 || N <= 0 || K <= 0 || (dtype != VS_F32 && dtype != VS_BF16)) return 0;
  const GemmPlan p = plan_gemm(dtype, M, N, K, 0, true, 0);
  size_t b = p.g.splits > 1 ? (size_t)p.g.splits * (size_t)(M * N) * 4 : 0;
  if (dtype == VS_BF16) {  // the dW kernels' partial tiles + bias sums (if this shape is a dW product)
    const size_t dw = dw_workspace_bytes(M, N, K);
    if (dw > b) b = dw;
    const size_t dw256 = knob(VS_KNOB_NO_DW256) ? 0 : dw256_workspace_bytes(M, N, K);
    if (dw256 > b) b = dw256;
  }
  const size_t sk = skinny_workspace_bytes(dtype, M, N, K);   // skinny split-K (head / Linear layer 0)
  if (sk > b) b = sk;
  return b;
}

#ifdef VS_STAMP
extern "C" int vs_dbg_gstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vs::g_gstamp), (size_t)n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
