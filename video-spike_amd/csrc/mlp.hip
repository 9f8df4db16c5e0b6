// mlp.hip — the ViT block's MLP (VideoMAEIntermediate + VideoMAEOutput, modeling_videomae.py:370-399)
// as fused bf16 kernels for the narrow widths (D = 192: ViT-Tiny, the bench's C2), gfx950.
//
// Forward, one launch:  x' = y + gelu(h2 W1^T + b1) W2^T + b2.
//   The 4x-wide intermediate never reaches HBM: per launch the kernel reads h2 (bf16) and the f32
//   residual y and writes x' (f32) — 1,920 B per token at D = 192 instead of the 5,000 B the two
//   GEMMs moved with the stored gelu / gelu' pair.
// Backward, one launch (vs_mlp_bwd_da):  pre = h2 W1^T + b1 is RECOMPUTED from h2 (same MFMA
//   chain as the forward: bitwise the same pre and gelu), da = (dx' W2) * gelu'(pre) and a = gelu(pre)
//   are written (bf16) for the dh2 / dW1 / dW2 products that follow.
//
// Structure (both kernels): 8 waves (2 per SIMD), one workgroup per CU, persistent over rounds of
// 256 tokens (32 per wave).  Each wave computes TRANSPOSED products with its 32 tokens on the MFMA
// N axis (lanes): pre^T = W1_c h2^T (32x32x16, W1 rows from LDS as the A operand, h2 rows straight
// from HBM as B fragments, kept in registers for the round), then the accumulator IS the next
// product's B operand (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
// The weights stream through LDS in chunks of 64 intermediate features (W1_c: 64 x D, W2_c: D x 64,
// 48 KB per stage, two stages) by LDS-DMA, shared by the 8 waves, one barrier per chunk.
// Row permutation: the W1 (and forward W2) rows of every 32-row MFMA tile are stored with bits 2 and
// 3 of the row index swapped (DMA source selection), so that a lane's 16 accumulator registers are
// two runs of 8 CONSECUTIVE features (registers 0-7: 8h .. 8h+7, 8-15: 16+8h ..): the accumulator
// feeds the next MFMA in natural k order, and the epilogues write 16-byte / 32-byte runs.
// LDS images: W1_c rows of 2D bytes, W2_c rows of 128 B; 16-B chunk c of row r is stored at chunk
// position (c & ~7) | ((c & 7) ^ ((r >> 1) & 7)): every ds_read_b128 of a 32x32x16 operand is
// conflict-free (16 lanes of a group = 16 rows of distinct (r & 1, chunk position)).
#include "common.h"

namespace vs {

constexpr int kMlpWaves = 8;
constexpr int kMlpFC = 64;          // intermediate features per chunk
constexpr int kMlpMaxF = 3072;

__device__ __forceinline__ int mlp_swap23(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }
__device__ __forceinline__ int mlp_cpos(int c, int r) { return (c & ~7) | ((c & 7) ^ ((r >> 1) & 7)); }
// chunk XOR key of the backward's W2 image (read only by ds_read_b64_tr_b16): a 32-lane group reads
// rows d0 .. d0 + 3 (d0 % 4 == 0), 4 chunks of one half-row each, and rows d and d + 2 share banks
// (256 B apart); bit 2 of the key = bit 1 of the row puts them in opposite half-rows (the (d >> 1) & 7
// key mapped them onto the same chunks: 2-way conflicts, 30 % of the LDS cycles in the PMC)
__device__ __forceinline__ int mlp_key_tr(int d) { return (((d >> 1) & 1) << 2) | ((d >> 2) & 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlp_rsrc(const void* base, int64_t rows_left, int64_t ld, int es) {
  const int64_t n = rows_left > 0 ? rows_left : 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(n * ld * es), 0x00020000);
}

// sum over lanes l and l ^ 32 (the two halves of a token's row) without LDS
__device__ __forceinline__ float pair_sum(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// GELU for the fused bf16 MLP: x * sigmoid(x (k1 + k3 x^2 + k5 x^4)), a minimax fit of x * Phi(x)
// (scipy Nelder-Mead on [-9, 9]): |gelu - x Phi(x)| <= 2.5e-5 everywhere (the tanh form: 4.7e-4;
// A&S 7.1.26 in common.h: 1.5e-7 but twice the VALU), i.e. ~1 % of the bf16 rounding the result gets
// anyway.  x^2 is clamped at 81 (the quartic turns negative past |x| = 11.1; sigmoid is saturated
// there).  7 VALU + exp2 + rcp per value.  The backward uses the SAME function's exact derivative
// s + x s (1 - s) u'(x) (|error vs Phi(x) + x phi(x)| <= 1.1e-4).
constexpr float kGk1 = 1.59501577f, kGk3 = 7.40112920e-2f, kGk5 = -7.03033577e-4f;
constexpr float kGl2e = 1.4426950408889634f;
__device__ __forceinline__ float gelu_sp_s(float x, float& t) {  // sigmoid(u(x)); t = min(x^2, 81)
  t = fminf(x * x, 81.f);
  float p = fmaf(t, -kGk5 * kGl2e, -kGk3 * kGl2e);
  p = fmaf(t, p, -kGk1 * kGl2e);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * p));
}
__device__ __forceinline__ float gelu_sp(float x) {
  float t;
  return x * gelu_sp_s(x, t);
}
__device__ __forceinline__ float gelu_sp_both(float x, float& grad) {
  float t;
  const float sg = gelu_sp_s(x, t);
  float q = fmaf(t, 5.f * kGk5, 3.f * kGk3);
  q = fmaf(t, q, kGk1);                      // u'(x)
  grad = fmaf(x * fmaf(-sg, sg, sg), q, sg);  // s + x s (1 - s) u'
  return x * sg;
}

// The same GELU over a 16-value tile, spread over the 12 MFMA segments of a product by STAGE: in
// segment k every value advances one step of the chain, so a segment carries 16 independent
// operations instead of the 1-2 dependent chains of 9 that left the wave waiting on VALU latency
// (stages 5-6 / 8-9 split the exp / rcp so no segment holds 16 transcendentals).
// Packed f32: the multiply / add / fma stages as v_pk_{mul,add,fma}_f32 on value
// pairs (8 instructions per stage instead of 16; the min and the transcendentals stay scalar; every
// lane's arithmetic is the scalar form's, bit for bit).  Measured (scripts/mlp_bench.py, two A/B
// pairs, profiles/r05_mlp_pk_ab.txt): the forward with the LayerNorm epilogue 241 -> 229 us, the plain
// forward 230-233 -> 215-229; the backward's gelu_both_stage packed the same way was SLOWER (243 ->
// 250-260 us), so it stays scalar (the packed form is kept for diagnostic builds, -DVS_MLP_PK_BWD).
struct GeluStages {
  f32x2 t[8], p[8];
};
__device__ __forceinline__ f32x2 pk_splat(float c) { return (f32x2){c, c}; }
__device__ __forceinline__ void gelu_stage(int k, const f32x16& x, GeluStages& s, float (&g)[16]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x2 xv = {x[2 * j], x[2 * j + 1]};
    if (k == 0) s.t[j] = xv * xv;
    if (k == 1) s.t[j] = (f32x2){fminf(s.t[j][0], 81.f), fminf(s.t[j][1], 81.f)};
    if (k == 2) s.p[j] = __builtin_elementwise_fma(s.t[j], pk_splat(-kGk5 * kGl2e), pk_splat(-kGk3 * kGl2e));
    if (k == 3) s.p[j] = __builtin_elementwise_fma(s.t[j], s.p[j], pk_splat(-kGk1 * kGl2e));
    if (k == 4) s.p[j] = xv * s.p[j];
    if ((k == 5 && j < 4) || (k == 6 && j >= 4))
      s.p[j] = (f32x2){__builtin_amdgcn_exp2f(s.p[j][0]), __builtin_amdgcn_exp2f(s.p[j][1])};
    if (k == 7) s.p[j] = s.p[j] + pk_splat(1.f);
    if ((k == 8 && j < 4) || (k == 9 && j >= 4))
      s.p[j] = (f32x2){__builtin_amdgcn_rcpf(s.p[j][0]), __builtin_amdgcn_rcpf(s.p[j][1])};
    if (k == 10) {
      const f32x2 r = xv * s.p[j];
      g[2 * j] = r[0];
      g[2 * j + 1] = r[1];
    }
  }
}
#ifdef VS_MLP_PK_BWD
__device__ __forceinline__ void gelu_both_stage(int k, const f32x16& x, GeluStages& s, float (&a)[16],
                                                float (&grad)[16]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x2 xv = {x[2 * j], x[2 * j + 1]};
    f32x2 gr = {grad[2 * j], grad[2 * j + 1]};
    if (k == 0) s.t[j] = xv * xv;
    if (k == 1) s.t[j] = (f32x2){fminf(s.t[j][0], 81.f), fminf(s.t[j][1], 81.f)};
    if (k == 2) {
      s.p[j] = __builtin_elementwise_fma(s.t[j], pk_splat(-kGk5 * kGl2e), pk_splat(-kGk3 * kGl2e));
      gr = __builtin_elementwise_fma(s.t[j], pk_splat(5.f * kGk5), pk_splat(3.f * kGk3));
    }
    if (k == 3) {
      s.p[j] = __builtin_elementwise_fma(s.t[j], s.p[j], pk_splat(-kGk1 * kGl2e));
      gr = __builtin_elementwise_fma(s.t[j], gr, pk_splat(kGk1));
    }
    if (k == 4) s.p[j] = xv * s.p[j];
    if ((k == 5 && j < 4) || (k == 6 && j >= 4))
      s.p[j] = (f32x2){__builtin_amdgcn_exp2f(s.p[j][0]), __builtin_amdgcn_exp2f(s.p[j][1])};
    if (k == 7) s.p[j] = s.p[j] + pk_splat(1.f);
    if ((k == 8 && j < 4) || (k == 9 && j >= 4))
      s.p[j] = (f32x2){__builtin_amdgcn_rcpf(s.p[j][0]), __builtin_amdgcn_rcpf(s.p[j][1])};
    if (k == 10) {
      const f32x2 r = xv * s.p[j];
      a[2 * j] = r[0];
      a[2 * j + 1] = r[1];
      s.t[j] = __builtin_elementwise_fma(-s.p[j], s.p[j], s.p[j]);
    }
    if (k == 11) gr = __builtin_elementwise_fma(xv * s.t[j], gr, s.p[j]);
    if (k == 2 || k == 3 || k == 11) {
      grad[2 * j] = gr[0];
      grad[2 * j + 1] = gr[1];
    }
  }
}
#else
struct GeluStagesS {
  float t[16], p[16];
};

// ... and gelu with its derivative (the backward), same staging: a = x s, grad = s + x s (1 - s) u'(x)
__device__ __forceinline__ void gelu_both_stage(int k, const f32x16& x, GeluStagesS& s, float (&a)[16],
                                                float (&grad)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (k == 0) s.t[i] = x[i] * x[i];
    if (k == 1) s.t[i] = fminf(s.t[i], 81.f);
    if (k == 2) {
      s.p[i] = fmaf(s.t[i], -kGk5 * kGl2e, -kGk3 * kGl2e);
      grad[i] = fmaf(s.t[i], 5.f * kGk5, 3.f * kGk3);
    }
    if (k == 3) {
      s.p[i] = fmaf(s.t[i], s.p[i], -kGk1 * kGl2e);
      grad[i] = fmaf(s.t[i], grad[i], kGk1);  // u'(x), kept in grad until stage 11
    }
    if (k == 4) s.p[i] = x[i] * s.p[i];
    if ((k == 5 && i < 8) || (k == 6 && i >= 8)) s.p[i] = __builtin_amdgcn_exp2f(s.p[i]);
    if (k == 7) s.p[i] = 1.f + s.p[i];
    if ((k == 8 && i < 8) || (k == 9 && i >= 8)) s.p[i] = __builtin_amdgcn_rcpf(s.p[i]);
    if (k == 10) {
      a[i] = x[i] * s.p[i];
      s.t[i] = fmaf(-s.p[i], s.p[i], s.p[i]);  // s (1 - s)
    }
    if (k == 11) grad[i] = fmaf(x[i] * s.t[i], grad[i], s.p[i]);
  }
}
#endif
#ifdef VS_MLP_PK_BWD
using GeluStagesB = GeluStages;
#else
using GeluStagesB = GeluStagesS;
#endif

__device__ __forceinline__ u32x4v mlp_pack8(const float* v) {
  u32x4v u;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    u[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){v[2 * q], v[2 * q + 1]}, bf16x2v));
  return u;
}

template <int D>
struct MlpGeom {
  static constexpr int KS1 = D / 16;            // k-steps of the W1 product (32x32x16)
  static constexpr int NT = D / 32;             // 32-row output tiles of the W2 product
  static constexpr int W1B = kMlpFC * D * 2;    // bytes of one W1 chunk image
  static constexpr int W2B = D * kMlpFC * 2;
  static constexpr int STG = W1B + W2B;
  static constexpr int DMA1 = W1B / 1024 / kMlpWaves;  // 1-KB LDS-DMA pieces per wave per chunk
  static constexpr int DMA2 = W2B / 1024 / kMlpWaves;
  static_assert(DMA1 * 1024 * kMlpWaves == W1B && DMA2 * 1024 * kMlpWaves == W2B, "DMA split");
};

// Per-lane DMA source offsets (bytes, chunk-invariant) of the W1 / W2 chunk images; the chunk adds a
// wave-uniform base.  fwd_w2_perm: the forward's W2 image has its rows (d) swap23-permuted too.
template <int D>
__device__ __forceinline__ void mlp_dma_offsets(int wave, int lane, int64_t F, bool fwd_w2_perm,
                                                uint32_t (&o1)[MlpGeom<D>::DMA1], uint32_t (&o2)[MlpGeom<D>::DMA2]) {
  using G = MlpGeom<D>;
#pragma unroll
  for (int k = 0; k < G::DMA1; ++k) {
    const int P = 64 * (wave * G::DMA1 + k) + lane;  // 16-B chunk index of the image
    const int r = P / (D / 8), cp = P % (D / 8);
    const int grow = 32 * (r >> 5) + mlp_swap23(r & 31);
    const int cl = mlp_cpos(cp, r);  // the map is an involution on the low 3 bits
    o1[k] = (uint32_t)((grow * D + 8 * cl) * 2);
  }
#pragma unroll
  for (int k = 0; k < G::DMA2; ++k) {
    const int P = 64 * (wave * G::DMA2 + k) + lane;
    const int p = P / 8, cp = P % 8;
    const int d = fwd_w2_perm ? 32 * (p >> 5) + mlp_swap23(p & 31) : p;
    const int cl = cp ^ (fwd_w2_perm ? (p >> 1) & 7 : mlp_key_tr(p));
    o2[k] = (uint32_t)(((int64_t)d * F + 8 * cl) * 2);
  }
}

template <int D>
__device__ __forceinline__ void mlp_dma_chunk(const bf16_t* w1, const bf16_t* w2, int c, char* stage, int wave,
                                              const uint32_t (&o1)[MlpGeom<D>::DMA1],
                                              const uint32_t (&o2)[MlpGeom<D>::DMA2]) {
  using G = MlpGeom<D>;
  const bf16_t* s1 = w1 + (int64_t)c * kMlpFC * D;
  const bf16_t* s2 = w2 + (int64_t)c * kMlpFC;
#pragma unroll
  for (int k = 0; k < G::DMA1; ++k) glds16_asm_so(s1, o1[k], stage + 1024 * (wave * G::DMA1 + k));
#pragma unroll
  for (int k = 0; k < G::DMA2; ++k) glds16_asm_so(s2, o2[k], stage + G::W1B + 1024 * (wave * G::DMA2 + k));
}

// pre^T tile t (features 32 t .. of the chunk x 32 tokens) = W1_c h2^T: 12 MFMAs (D = 192)
// Per-lane byte offsets of a 32x32x16 A-fragment read of k-step s from an image whose 16-B chunk c
// of row r sits at (c & ~7) | ((c & 7) ^ ((r >> 1) & 7)): for c = 2 s + h the position is
// 8 (s >> 2) + 2 ((s & 3) ^ (key >> 1)) + (h ^ (key & 1)), so 4 per-lane offsets (s & 3) plus the
// immediate 128 (s >> 2) cover every k-step (and +32 rows per tile is an immediate too).
__device__ __forceinline__ void mlp_frag_offsets(int lane, int row_bytes, uint32_t (&off)[4]) {
  const int rr = lane & 31, h = lane >> 5, key = (rr >> 1) & 7;
#pragma unroll
  for (int j = 0; j < 4; ++j) off[j] = (uint32_t)(rr * row_bytes + 16 * (2 * (j ^ (key >> 1)) + (h ^ (key & 1))));
}

// the bias of pre^T tile t of chunk c in accumulator order (features c*64 + 32 t + 16 j2 + 8 h + j),
// the W1 product's initial accumulator: the MFMA chain then yields h2 W1^T + b1 directly
__device__ __forceinline__ f32x16 mlp_bias_acc(const float* b1s, int c, int t, int h) {
  f32x16 a;
#pragma unroll
  for (int j2 = 0; j2 < 2; ++j2) {
    const float* bb = b1s + c * kMlpFC + 32 * t + 16 * j2 + 8 * h;
    const f32x4 bl = *(const f32x4*)bb, bh = *(const f32x4*)(bb + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[8 * j2 + j] = bl[j];
      a[8 * j2 + 4 + j] = bh[j];
    }
  }
  return a;
}

template <int D>
__device__ __forceinline__ f32x16 mlp_s1(const char* st, const uint32_t (&off)[4], const u32x4v (&xf)[MlpGeom<D>::KS1],
                                         int t, f32x16 pre) {
  using G = MlpGeom<D>;
#pragma unroll
  for (int s = 0; s < G::KS1; ++s) {
    const bf16x8 wa = *(const bf16x8*)(st + off[s & 3] + 32 * t * (2 * D) + 128 * (s >> 2));
    pre = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, __builtin_bit_cast(bf16x8, xf[s]), pre, 0, 0, 0);
  }
  return pre;
}

// Software pipelining by pinned segments: hipcc's scheduler (and T19's sched_group_barrier, which it
// ignored here) clusters a product's 12 MFMAs and puts the independent GELU work of the other tile
// after them, so one wave alternates long MFMA-only and VALU-only stretches and the two waves of a
// SIMD, aligned by the per-chunk barrier, do the same at the same time.  Each MFMA is therefore
// emitted in its own segment (closed by sched_barrier(0)) together with a share of the VALU work
// and the LDS read of the fragment two MFMAs ahead.
// Values of a 16-value tile processed in segment i of 12: [i * 4 / 3, (i + 1) * 4 / 3)
__device__ __forceinline__ constexpr int mlp_seg_lo(int i) { return i * 4 / 3; }

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
// The next block's LayerNorm1 on the rows this epilogue owns (LNF): h = LN(x'; g, b, eps) in bf16
// with its row mean / rstd (two-pass variance, as ln_fwd_vec_kernel), so that block skips its own
// LayerNorm launch (x' is not read back).
struct MlpLnOut {
  const float* g;
  const float* b;
  float eps;
  bf16_t* h;
  int64_t ldh;
  float* mean;
  float* rstd;
};

// s_waitcnt vmcnt(N): every vector-memory op but the newest N has completed (they complete in order)
template <int N>
__device__ __forceinline__ void mlp_vmcnt_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}
#ifdef VS_MLP_STAMP
// Diagnostic build only (-DVS_MLP_STAMP, scripts/stamp_mlp.py): per wave of the last forward launch
// {total, chunk-start wait (vmcnt + barrier), epilogue, chunks} in shader-clock cycles.
__device__ unsigned long long g_mlp_stamp[4 * 4096];
#define MLP_CLK() __builtin_amdgcn_s_memtime()
#else
#define MLP_CLK() 0ull
#endif
template <int D, bool LNF>
__global__ __launch_bounds__(64 * kMlpWaves, 1) void mlp_fwd_kernel(const bf16_t* __restrict__ h2, int64_t ldh,
                                                                    const bf16_t* __restrict__ w1,
                                                                    const float* __restrict__ b1,
                                                                    const bf16_t* __restrict__ w2,
                                                                    const float* __restrict__ b2,
                                                                    const float* __restrict__ y, int64_t ldy,
                                                                    float* __restrict__ xo, int64_t ldx, int64_t M,
                                                                    int F, MlpLnOut ln) {
  using G = MlpGeom<D>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::STG];
  __shared__ __attribute__((aligned(16))) float b1s[kMlpMaxF];
  __shared__ __attribute__((aligned(16))) float b2s[D];
  __shared__ __attribute__((aligned(16))) float lngs[LNF ? D : 4];
  __shared__ __attribute__((aligned(16))) float lnbs[LNF ? D : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rr = lane & 31, h = lane >> 5;
  const int nch = F / kMlpFC;
  if ((int64_t)blockIdx.x * 32 >= M) return;  // workgroup-uniform: no block at all
  uint32_t o1[G::DMA1], o2[G::DMA2];
  mlp_dma_offsets<D>(wave, lane, F, true, o1, o2);
  mlp_dma_chunk<D>(w1, w2, 0, smem, wave, o1, o2);  // chunk 0 of the first round -> stage 0
  for (int i = tid; i < F; i += 64 * kMlpWaves) b1s[i] = b1[i];
  if (tid < D) b2s[tid] = b2[tid];
  if constexpr (LNF) {
    if (tid < D) {
      lngs[tid] = ln.g[tid];
      lnbs[tid] = ln.b[tid];
    }
  }

  // Rounds: in round r wave w owns the 32-token block b = r * 8 G + w G + blockIdx.x (blocks dealt
  // over the workgroups first: the last, partial round gives single live waves to as many workgroups
  // as it has blocks instead of filling a few, so it costs about half a round instead of a whole one).
  const int64_t nb = (M + 31) / 32, Gs = gridDim.x;
  auto blk = [&](int64_t r) { return r * Gs * kMlpWaves + (int64_t)wave * Gs + blockIdx.x; };
  // h2 fragments of a round: lane (token rr, half h) holds d = 16 s + 8 h .. + 7 of its token
  u32x4v xf[G::KS1];
  const uint32_t hxo = (uint32_t)((rr * ldh + 8 * h) * 2);
  auto load_x = [&](int64_t r) {
    const int64_t row0 = blk(r) * 32;
    const auto rx = mlp_rsrc(h2 + row0 * ldh, M - row0, ldh, 2);
#pragma unroll
    for (int s = 0; s < G::KS1; ++s)
      xf[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, hxo + 32 * s, 0, 0);
  };
  uint32_t off1[4], off2[4];
  mlp_frag_offsets(lane, 2 * D, off1);
  mlp_frag_offsets(lane, 128, off2);
  auto pack16 = [&](const float (&g)[16], u32x4v& f0, u32x4v& f1) {
    f0 = mlp_pack8(g);
    f1 = mlp_pack8(g + 8);
  };
  // pre^T tile 1 (12 MFMAs) with the GELU of tile 0 (`p0` + bias -> g) spread over its segments
  auto s1_act = [&](const char* st, const f32x16& p0, f32x16 p1, float (&g)[16]) {
    GeluStages gs;
    auto rd = [&](int k) { return *(const bf16x8*)(st + off1[k & 3] + 32 * (2 * D) + 128 * (k >> 2)); };
    bf16x8 wr[3] = {rd(0), rd(1), rd(1)};  // fragments two MFMAs ahead (LDS latency > one segment)
#pragma unroll
    for (int k = 0; k < G::KS1; ++k) {
      const bf16x8 cur = wr[k % 3];
      if (k + 2 < G::KS1) wr[(k + 2) % 3] = rd(k + 2);
      p1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, __builtin_bit_cast(bf16x8, xf[k]), p1, 0, 0, 0);
      gelu_stage(k, p0, gs, g);
      __builtin_amdgcn_sched_barrier(0);
    }
    return p1;
  };
  // x'^T += W2_c a^T over k-steps 2 t, 2 t + 1 (12 MFMAs); optionally the GELU of the other tile
  // (`pn` + bias -> g) spread over the segments
  auto s2_act = [&](const char* st2, int t, const u32x4v& f0, const u32x4v& f1, f32x16 (&acc)[G::NT],
                    const f32x16* pn, float (&g)[16]) {
    GeluStages gs;
    auto rd = [&](int k) {
      const int s1 = 2 * t + k / G::NT, T1 = k % G::NT;
      return *(const bf16x8*)(st2 + off2[s1 & 3] + 32 * T1 * 128);
    };
    bf16x8 wr[3] = {rd(0), rd(1), rd(1)};
#pragma unroll
    for (int k = 0; k < 2 * G::NT; ++k) {
      const int sk = 2 * t + k / G::NT, T = k % G::NT;
      const bf16x8 cur = wr[k % 3];
      if (k + 2 < 2 * G::NT) wr[(k + 2) % 3] = rd(k + 2);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, __builtin_bit_cast(bf16x8, sk & 1 ? f1 : f0), acc[T], 0, 0, 0);
      if (pn) gelu_stage(k, *pn, gs, g);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // The residual is the W2 product's initial accumulator: y of a round's tokens is loaded into acc
  // right after the previous round's epilogue stored it (the loads then have chunk 0's W1 products to
  // land), so the epilogue only adds b2 and stores.  Lane (token rr, half h) holds d = 32 T + 16 j2 +
  // 8 h .. + 7 in acc[T][8 j2 ..].
  f32x16 acc[G::NT];
  // per-lane byte bases of the y / x' / h rows (the (T, j2) group adds an immediate: 24 precomputed
  // offsets per lane were spilled around the round loop)
  const uint32_t yb = (uint32_t)((rr * ldy + 8 * h) * 4), xb = (uint32_t)((rr * ldx + 8 * h) * 4);
  const uint32_t hb = LNF ? (uint32_t)((rr * ln.ldh + 8 * h) * 2) : 0u;
  auto load_y = [&](int64_t r) {
    const int64_t row0 = blk(r) * 32;
    const auto ry = mlp_rsrc(y + row0 * ldy, M - row0, ldy, 4);
#pragma unroll
    for (int T = 0; T < G::NT; ++T)
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2) {
        const uint32_t oy = yb + 4 * (32 * T + 16 * j2);  // lane base + an immediate
        const f32x4 y0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, oy, 0, 0));
        const f32x4 y1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, oy + 16, 0, 0));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[T][8 * j2 + j] = y0[j];
          acc[T][8 * j2 + 4 + j] = y1[j];
        }
      }
  };
  load_x(0);
  if (blk(0) < nb) load_y(0);
  int q = 0;  // chunk stream position: stage q & 1
  // Vector-memory ops a live wave issues after the DMA of a round's chunk 0 (started at the previous
  // round's last chunk): the h2 prefetch, the epilogue's stores, the next round's y loads.  Chunk 0
  // waits for the DMA only (vmcnt(N) with N = the ops issued after it), not for those.
  constexpr int kNX = G::KS1, kNS = 4 * G::NT + (LNF ? 2 * G::NT + 2 : 0), kNY = 4 * G::NT;
  bool live_prev = false;
  unsigned long long t_wait = 0, t_epi = 0, n_chunks = 0;
  const unsigned long long t_begin = MLP_CLK();
  for (int64_t r = 0; r * Gs * kMlpWaves + blockIdx.x < nb; ++r) {
    const bool more = (r + 1) * Gs * kMlpWaves + blockIdx.x < nb;
    const bool live = blk(r) < nb;  // wave-uniform
    // one chunk: its DMA pieces (every wave's) landed, every wave is done with the other stage; the
    // last chunk of a round (PF) also prefetches the next round's h2 fragments
    auto chunk = [&](int c, auto pfc) {
      constexpr bool PF = decltype(pfc)::value;
      const unsigned long long cw = MLP_CLK();
      if (c == 0 && live_prev && live) mlp_vmcnt_le<kNX + kNS + kNY>();
      else if (c == 0 && live_prev) mlp_vmcnt_le<kNX + kNS>();
      else mlp_vmcnt_le<0>();
      __syncthreads();
      t_wait += MLP_CLK() - cw;
      ++n_chunks;
      // chunk 0 issues the next chunk's DMA after its first W2 tile: hipcc cannot see the asm DMA, and
      // its wait for the y loads (the accumulators' first use, in that tile) would drain it too
      const bool late_dma = !PF && c == 0;
      auto dma_next = [&] { mlp_dma_chunk<D>(w1, w2, PF ? 0 : c + 1, smem + ((q + 1) & 1) * G::STG, wave, o1, o2); };
      if (!late_dma && (!PF || more)) dma_next();
      if (live) {
        const char* st = smem + (q & 1) * G::STG;
        const char* st2 = st + G::W1B;
        // software pipeline over the chunk's two 32-feature tiles: S1(t0) | S1(t1) + GELU(t0) |
        // S2(t0) + GELU(t1) | S2(t1)
        float g[16];
        const f32x16 p0 = mlp_s1<D>(st, off1, xf, 0, mlp_bias_acc(b1s, c, 0, h));
        __builtin_amdgcn_sched_barrier(0);
        const f32x16 p1 = s1_act(st, p0, mlp_bias_acc(b1s, c, 1, h), g);
        u32x4v a0, a1, a2, a3;
        pack16(g, a0, a1);
        if constexpr (PF) {
          if (more) load_x(r + 1);  // the fragments are dead after the last chunk's W1 products
        }
        __builtin_amdgcn_sched_barrier(0);
        s2_act(st2, 0, a0, a1, acc, &p1, g);
        pack16(g, a2, a3);
        __builtin_amdgcn_sched_barrier(0);
        if (late_dma) dma_next();
        s2_act(st2, 1, a2, a3, acc, nullptr, g);
      } else if (late_dma) {
        dma_next();
      }
      ++q;
    };
    for (int c = 0; c + 1 < nch; ++c) chunk(c, IC<0>{});
    chunk(nch - 1, IC<1>{});
    if (!live) {  // (and every later round: blocks only grow)
      live_prev = false;
      continue;
    }
    const unsigned long long ce = MLP_CLK();
    // epilogue: x' = acc + b2 (acc started from y)
    const int64_t row0 = blk(r) * 32;
    const auto rxo = mlp_rsrc(xo + row0 * ldx, M - row0, ldx, 4);
#pragma unroll
    for (int T = 0; T < G::NT; ++T)
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2) {
        const int d0 = 32 * T + 16 * j2 + 8 * h;
        const uint32_t ox = xb + 4 * (32 * T + 16 * j2);
        const f32x4 c0 = *(const f32x4*)(b2s + d0), c1 = *(const f32x4*)(b2s + d0 + 4);
        f32x4 r0, r1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          r0[j] = acc[T][8 * j2 + j] + c0[j];
          r1[j] = acc[T][8 * j2 + 4 + j] + c1[j];
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, r0), rxo, ox, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, r1), rxo, ox + 16, 0, 0);
        if constexpr (LNF) {  // keep x' in the accumulators for the LayerNorm below
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[T][8 * j2 + j] = r0[j];
            acc[T][8 * j2 + 4 + j] = r1[j];
          }
        }
      }
    if constexpr (LNF) {
      // token rr's row: this lane's 96 values + lane rr ^ 32's 96
      float sm = 0.f;
#pragma unroll
      for (int T = 0; T < G::NT; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) sm += acc[T][i];
      const float mu = pair_sum(sm) * (1.0f / D);
      float sq = 0.f;
#pragma unroll
      for (int T = 0; T < G::NT; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          acc[T][i] -= mu;
          sq += acc[T][i] * acc[T][i];
        }
      const float rs = rsqrtf(pair_sum(sq) * (1.0f / D) + ln.eps);
      const auto rh = mlp_rsrc(ln.h + row0 * ln.ldh, M - row0, ln.ldh, 2);
#pragma unroll
      for (int T = 0; T < G::NT; ++T)
#pragma unroll
        for (int j2 = 0; j2 < 2; ++j2) {
          const int d0 = 32 * T + 16 * j2 + 8 * h;
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = acc[T][8 * j2 + j] * rs * lngs[d0 + j] + lnbs[d0 + j];
          __builtin_amdgcn_raw_buffer_store_b128(mlp_pack8(v), rh, hb + 2 * (32 * T + 16 * j2), 0, 0);
        }
      if (h == 0 && row0 + rr < M) {
        ln.mean[row0 + rr] = mu;
        ln.rstd[row0 + rr] = rs;
      }
    }
    if (more && blk(r + 1) < nb) load_y(r + 1);
    live_prev = live;
    t_epi += MLP_CLK() - ce;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA left in flight at exit
#ifdef VS_MLP_STAMP
  if (lane == 0 && !LNF) {
    unsigned long long* st = g_mlp_stamp + 4 * (blockIdx.x * kMlpWaves + wave);
    st[0] = MLP_CLK() - t_begin;
    st[1] = t_wait;
    st[2] = t_epi;
    st[3] = n_chunks;
  }
#else
  (void)t_wait;
  (void)t_epi;
  (void)n_chunks;
  (void)t_begin;
#endif
}

// ---------------------------------------------------------------------------------------------
// backward: da = (dx' W2) * gelu'(pre), a = gelu(pre), pre recomputed from h2
// ---------------------------------------------------------------------------------------------
// The W2 product here is da^T = W2_c^T dx'^T: its A operand (rows = features, k = d) is a COLUMN read
// of the W2 image, done with ds_read_b64_tr_b16 (each lane of a 16-lane group supplies the address
// of one 4-column quad of one row, so the swap23 feature order of the W1 product is chosen per lane).
template <int D>
__global__ __launch_bounds__(64 * kMlpWaves, 1) void mlp_bwd_da_kernel(const bf16_t* __restrict__ h2, int64_t ldh,
                                                                       const bf16_t* __restrict__ w1,
                                                                       const float* __restrict__ b1,
                                                                       const bf16_t* __restrict__ w2,
                                                                       const bf16_t* __restrict__ dy, int64_t lddy,
                                                                       bf16_t* __restrict__ da, int64_t ldda,
                                                                       bf16_t* __restrict__ aout, int64_t lda,
                                                                       int64_t M, int F) {
  using G = MlpGeom<D>;
  __shared__ __attribute__((aligned(16))) char smem[2 * G::STG];
  __shared__ __attribute__((aligned(16))) float b1s[kMlpMaxF];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rr = lane & 31, h = lane >> 5;
  const int nch = F / kMlpFC;
  if ((int64_t)blockIdx.x * 32 >= M) return;
  uint32_t o1[G::DMA1], o2[G::DMA2];
  mlp_dma_offsets<D>(wave, lane, F, false, o1, o2);  // W2 image rows in natural d order
  mlp_dma_chunk<D>(w1, w2, 0, smem, wave, o1, o2);
  for (int i = tid; i < F; i += 64 * kMlpWaves) b1s[i] = b1[i];

  // transposed-read addresses (bytes within the W2 image) of the A operand of da^T, per tile t
  // (features 32 t ..), k-step s and half e (k = 16 s + 8 hh + 4 e + qrow): lane i of 16-lane group
  // g supplies row qrow = i >> 2 and column quad pq = i & 3 -> feature quad 16 (g & 1) + 4 swap(pq)
  const int g16 = lane >> 4, i16 = lane & 15, hh = g16 >> 1;
  const int pq = i16 & 3, qrow = i16 >> 2;
  const int fq = 16 * (g16 & 1) + 4 * (((pq & 1) << 1) | (pq >> 1));  // swap23 on the feature index
  auto tr_addr = [&](int t, int s, int e) {
    const int d = 16 * s + 8 * hh + 4 * e + qrow;  // image row (natural order)
    const int f = 32 * t + fq;                     // first column of the quad
    const int cl = f >> 3;
    return d * 128 + 16 * (cl ^ mlp_key_tr(d)) + 2 * (f & 7);
  };

  uint32_t off1[4];
  mlp_frag_offsets(lane, 2 * D, off1);
  const int64_t nb = (M + 31) / 32, Gs = gridDim.x;
  auto blk = [&](int64_t r) { return r * Gs * kMlpWaves + (int64_t)wave * Gs + blockIdx.x; };
  u32x4v xf[G::KS1], yf[G::KS1];
  const uint32_t xo = (uint32_t)((rr * ldh + 8 * h) * 2), yo = (uint32_t)((rr * lddy + 8 * h) * 2);
  auto load_xy = [&](int64_t r) {
    const int64_t row0 = blk(r) * 32;
    const auto rx = mlp_rsrc(h2 + row0 * ldh, M - row0, ldh, 2);
    const auto ry = mlp_rsrc(dy + row0 * lddy, M - row0, lddy, 2);
#pragma unroll
    for (int s = 0; s < G::KS1; ++s) {
      xf[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, xo + 32 * s, 0, 0);
      yf[s] = __builtin_amdgcn_raw_buffer_load_b128(ry, yo + 32 * s, 0, 0);
    }
  };
  // the two 12-MFMA products of a chunk, each MFMA in a pinned segment with work(k) beside it
  // (see mlp_seg_lo): pre^T tile t = W1_c h2^T, da^T tile t = W2_c^T dx'^T (transposed A reads)
  auto s1_w = [&](const char* st, int t, f32x16 acc, auto&& work) {
    auto rd = [&](int k) { return *(const bf16x8*)(st + off1[k & 3] + 32 * t * (2 * D) + 128 * (k >> 2)); };
    bf16x8 wr[3] = {rd(0), rd(1), rd(1)};  // fragments two MFMAs ahead
#pragma unroll
    for (int k = 0; k < G::KS1; ++k) {
      const bf16x8 cur = wr[k % 3];
      if (k + 2 < G::KS1) wr[(k + 2) % 3] = rd(k + 2);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, __builtin_bit_cast(bf16x8, xf[k]), acc, 0, 0, 0);
      work(k);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  };
  typedef __attribute__((ext_vector_type(8))) short short8v;
  // tr_addr(t, k, e) = trb[t][e] + 2048 k: the chunk XOR key mlp_key_tr(d) reads bits 1-3 of d = 16 k + ..., not k
  uint32_t trb[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 2; ++e) trb[t][e] = (uint32_t)tr_addr(t, 0, e);
  auto trw = [&](const char* st2, int t, int k) {
    const short4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(st2 + trb[t][0] + 2048 * k));
    const short4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VS_LDS short4v*)(st2 + trb[t][1] + 2048 * k));
    const short8v wv = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    return __builtin_bit_cast(bf16x8, wv);
  };
  auto da_w = [&](const char* st2, int t, auto&& work) {
    f32x16 acc = f32x16{};
    bf16x8 wr[3] = {trw(st2, t, 0), trw(st2, t, 1), trw(st2, t, 1)};
#pragma unroll
    for (int k = 0; k < G::KS1; ++k) {
      const bf16x8 cur = wr[k % 3];
      if (k + 2 < G::KS1) wr[(k + 2) % 3] = trw(st2, t, k + 2);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, __builtin_bit_cast(bf16x8, yf[k]), acc, 0, 0, 0);
      work(k);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  };
  auto store16 = [&](const __amdgpu_buffer_rsrc_t& rs, int64_t ld, int c, int t, const float (&v)[16]) {
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2) {
      // every offset in voffset, soffset 0: a dwordx4 store whose soffset is an SGPR, followed at once
      // by a VALU write of its data VGPRs, stored the NEW value of dwords 1.. in lanes 12-15 of each
      // 16 on gfx950 (measured: da's dword 1 took the next segment's v_pk_fma result; hipcc inserts
      // no wait state there), so the chunk offset is added to the lane offset instead
      __builtin_amdgcn_raw_buffer_store_b128(mlp_pack8(v + 8 * j2), rs,
                                             (uint32_t)((rr * ld + 8 * h) * 2) + (uint32_t)(c * kMlpFC * 2) +
                                                 64 * t + 32 * j2,
                                             0, 0);
    }
  };
  load_xy(0);
  int q = 0;
  // Vector-memory ops a live wave issues after a chunk's DMA (started one chunk earlier): that
  // chunk's 8 stores of a / da (6 in chunk 0, whose DMA goes out after its first W2 tile: hipcc
  // cannot see the asm DMA, and its waits for the prefetched h2 / dx' fragments would drain it), and
  // in a round's last chunk also the next round's h2 / dx' prefetch.  The chunk start waits for the
  // DMA only (vmcnt(N), N = those ops): the stores stay in flight.
  constexpr int kNSt = 8, kNSt0 = 6, kNPf = 8 + 2 * G::KS1;
  bool live_prev = false;
  for (int64_t r = 0; r * Gs * kMlpWaves + blockIdx.x < nb; ++r) {
    const bool more = (r + 1) * Gs * kMlpWaves + blockIdx.x < nb;
    const bool live = blk(r) < nb;
    const int64_t row0 = blk(r) * 32;
    const auto rda = mlp_rsrc(da + row0 * ldda, M - row0, ldda, 2);
    const auto raa = mlp_rsrc(aout + row0 * lda, M - row0, lda, 2);
    auto chunk = [&](int c, auto pfc) {
      constexpr bool PF = decltype(pfc)::value;
      if (c > 1 && live) mlp_vmcnt_le<kNSt>();
      else if (c == 1 && live) mlp_vmcnt_le<kNSt0>();
      else if (c == 0 && live_prev) mlp_vmcnt_le<kNPf>();
      else mlp_vmcnt_le<0>();
      __syncthreads();
      const bool late_dma = !PF && c == 0;
      auto dma_next = [&] { mlp_dma_chunk<D>(w1, w2, PF ? 0 : c + 1, smem + ((q + 1) & 1) * G::STG, wave, o1, o2); };
      if (!late_dma && (!PF || more)) dma_next();
      if (live) {
        const char* st = smem + (q & 1) * G::STG;
        const char* st2 = st + G::W1B;
        // S1(t0) | S1(t1) + act(t0) | da(t0) + act(t1) | da(t1) + da-product(t0) | da-product(t1)
        float av[16], g0[16], g1[16];  // g0 / g1 become the da values in place
        const f32x16 p0 = s1_w(st, 0, mlp_bias_acc(b1s, c, 0, h), [&](int) {});
        GeluStagesB gs;
        const f32x16 p1 = s1_w(st, 1, mlp_bias_acc(b1s, c, 1, h), [&](int k) { gelu_both_stage(k, p0, gs, av, g0); });
        store16(raa, lda, c, 0, av);
        if constexpr (PF) {  // h2 fragments are dead after the last chunk's W1 products
          if (more) {
            const int64_t nrow0 = blk(r + 1) * 32;
            const auto rx = mlp_rsrc(h2 + nrow0 * ldh, M - nrow0, ldh, 2);
#pragma unroll
            for (int s = 0; s < G::KS1; ++s)
              xf[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, xo + 32 * s, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        const f32x16 d0 = da_w(st2, 0, [&](int k) { gelu_both_stage(k, p1, gs, av, g1); });
        store16(raa, lda, c, 1, av);
        __builtin_amdgcn_sched_barrier(0);
        if (late_dma) dma_next();
        const f32x16 d1 = da_w(st2, 1, [&](int k) {
#pragma unroll
          for (int i = mlp_seg_lo(k); i < mlp_seg_lo(k + 1); ++i) g0[i] *= d0[i];
        });
        store16(rda, ldda, c, 0, g0);
        if constexpr (PF) {  // dx' fragments are dead after the last chunk's W2 products
          if (more) {
            const int64_t nrow0 = blk(r + 1) * 32;
            const auto ry = mlp_rsrc(dy + nrow0 * lddy, M - nrow0, lddy, 2);
#pragma unroll
            for (int s = 0; s < G::KS1; ++s)
              yf[s] = __builtin_amdgcn_raw_buffer_load_b128(ry, yo + 32 * s, 0, 0);
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) g1[i] *= d1[i];
        store16(rda, ldda, c, 1, g1);
      } else if (late_dma) {
        dma_next();
      }
      ++q;
    };
    for (int c = 0; c + 1 < nch; ++c) chunk(c, IC<0>{});
    chunk(nch - 1, IC<1>{});
    live_prev = live;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int mlp_grid(int64_t M) {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  const int64_t blocks = (M + 31) / 32;  // every workgroup needs at least one 32-token block
  return (int)(blocks < cus ? blocks : cus);
}

}  // namespace vs

using namespace vs;

extern "C" int vs_mlp_fused_ok(int64_t M, int64_t D, int64_t F) {
  return D == 192 && F % kMlpFC == 0 && F >= kMlpFC && F <= kMlpMaxF && M > 0 && M * F * 2 < (int64_t(1) << 31) &&
                 M * D * 4 < (int64_t(1) << 31)
             ? 1
             : 0;
}

extern "C" int vs_mlp_fwd_ln(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1,
                             const float* b1, const void* w2, const float* b2, const float* y, int64_t ldy,
                             float* x_out, int64_t ldx, const float* ln_g, const float* ln_b, float eps, void* h_out,
                             int64_t ld_h_out, float* mean_out, float* rstd_out, void* stream);

extern "C" int vs_mlp_fwd(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1, const float* b1,
                          const void* w2, const float* b2, const float* y, int64_t ldy, float* x_out, int64_t ldx,
                          void* stream) {
  return vs_mlp_fwd_ln(M, D, F, h2, ldh, w1, b1, w2, b2, y, ldy, x_out, ldx, nullptr, nullptr, 0.f, nullptr, 0, nullptr,
                       nullptr, stream);
}

extern "C" int vs_mlp_fwd_ln(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1,
                             const float* b1, const void* w2, const float* b2, const float* y, int64_t ldy,
                             float* x_out, int64_t ldx, const float* ln_g, const float* ln_b, float eps, void* h_out,
                             int64_t ld_h_out, float* mean_out, float* rstd_out, void* stream) {
  VS_REQUIRE(vs_mlp_fused_ok(M, D, F), "vs_mlp_fwd: needs D = 192, F % 64 == 0, F <= 3072");
  VS_REQUIRE(h2 && w1 && b1 && w2 && b2 && y && x_out, "vs_mlp_fwd: null pointer");
  VS_REQUIRE(ldh >= D && ldh % 8 == 0 && ldy >= D && ldy % 4 == 0 && ldx >= D && ldx % 4 == 0 &&
                 aligned16(h2) && aligned16(w1) && aligned16(w2) && aligned16(y) && aligned16(x_out) &&
                 aligned16(b1) && aligned16(b2),
             "vs_mlp_fwd: rows must be 16-byte aligned");
  VS_REQUIRE(M * ldy * 4 < (int64_t(1) << 31) && M * ldx * 4 < (int64_t(1) << 31) && M * ldh * 2 < (int64_t(1) << 31),
             "vs_mlp_fwd: operand too large for 32-bit buffer offsets");
  hipStream_t s = (hipStream_t)stream;
  // bytes: h2 (bf16) + y, x' (f32) per element, both weights, the biases; with the LayerNorm: + h (bf16)
  // per element and mean / rstd per row
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM, s,
                    (double)M * (double)D * (2.0 + 4.0 + 4.0 + (ln_g ? 2.0 : 0.0)) + (ln_g ? (double)M * 8.0 : 0.0) +
                        (double)F * (double)D * 4.0 + (double)(F + D) * 4.0);
  const bool lnf = ln_g != nullptr;
  VS_REQUIRE(!lnf || (ln_b && h_out && mean_out && rstd_out && ld_h_out >= D && ld_h_out % 8 == 0 && aligned16(h_out) &&
                      M * ld_h_out * 2 < (int64_t(1) << 31)),
             "vs_mlp_fwd_ln: the LayerNorm output needs g, b, an aligned bf16 h and mean / rstd");
  MlpLnOut ln = {ln_g, ln_b, eps, (bf16_t*)h_out, ld_h_out, mean_out, rstd_out};
  count_path(VS_PATH_MLP_FWD);
  if (lnf) {
    hipLaunchKernelGGL((mlp_fwd_kernel<192, true>), dim3((unsigned)mlp_grid(M)), dim3(64 * kMlpWaves), 0, s,
                       (const bf16_t*)h2, ldh, (const bf16_t*)w1, b1, (const bf16_t*)w2, b2, y, ldy, x_out, ldx, M,
                       (int)F, ln);
  } else {
    hipLaunchKernelGGL((mlp_fwd_kernel<192, false>), dim3((unsigned)mlp_grid(M)), dim3(64 * kMlpWaves), 0, s,
                       (const bf16_t*)h2, ldh, (const bf16_t*)w1, b1, (const bf16_t*)w2, b2, y, ldy, x_out, ldx, M,
                       (int)F, ln);
  }
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_mlp_bwd_da(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1,
                             const float* b1, const void* w2, const void* dy, int64_t lddy, void* da, int64_t ldda,
                             void* a, int64_t lda, void* stream) {
  VS_REQUIRE(vs_mlp_fused_ok(M, D, F), "vs_mlp_bwd_da: needs D = 192, F % 64 == 0, F <= 3072");
  VS_REQUIRE(h2 && w1 && b1 && w2 && dy && da && a, "vs_mlp_bwd_da: null pointer");
  VS_REQUIRE(ldh >= D && ldh % 8 == 0 && lddy >= D && lddy % 8 == 0 && ldda >= F && ldda % 8 == 0 && lda >= F &&
                 lda % 8 == 0 && aligned16(h2) && aligned16(w1) && aligned16(w2) && aligned16(dy) && aligned16(da) &&
                 aligned16(a) && aligned16(b1),
             "vs_mlp_bwd_da: rows must be 16-byte aligned");
  VS_REQUIRE(M * ldda * 2 < (int64_t(1) << 31) && M * lda * 2 < (int64_t(1) << 31) && M * ldh * 2 < (int64_t(1) << 31) &&
                 M * lddy * 2 < (int64_t(1) << 31),
             "vs_mlp_bwd_da: operand too large for 32-bit buffer offsets");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM, s,
                    (double)M * (double)D * 4.0 + (double)M * (double)F * 4.0 + (double)F * (double)D * 4.0 +
                        (double)F * 4.0);
  count_path(VS_PATH_MLP_BWD);
  hipLaunchKernelGGL(mlp_bwd_da_kernel<192>, dim3((unsigned)mlp_grid(M)), dim3(64 * kMlpWaves), 0, s,
                     (const bf16_t*)h2, ldh, (const bf16_t*)w1, b1, (const bf16_t*)w2, (const bf16_t*)dy, lddy,
                     (bf16_t*)da, ldda, (bf16_t*)a, lda, M, (int)F);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

#ifdef VS_MLP_STAMP
extern "C" int vs_dbg_mlp_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vs::g_mlp_stamp), (size_t)n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
