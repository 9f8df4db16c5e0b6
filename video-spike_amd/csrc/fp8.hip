// fp8.hip — MX-FP8 (OCP e4m3 elements, E8M0 power-of-two scale per 32 consecutive k) forward
// products for BASELINE C5 (ViT-Base at 32 frames, "fp8 MFMA"): the ViT block's four Linear
// forwards (qkv, proj, fc1, fc2: modeling_videomae.py:233-236, 312-319, 373-383, 390-397) on the
// block-scaled matrix cores, v_mfma_scale_f32_32x32x64_f8f6f4 (twice the bf16 MFMA rate per clock,
// MI355X_MICROARCH.md "Matrix cores"); the scales are applied by the instruction itself.
//
// Quantisation (vs_quant_mxfp8): per (row, 32-element block along k) the scale is 2^e with
// e = ceil(log2(amax / 448)) (448 = the largest finite e4m3), so every scaled element lies in
// [-448, 448] and nothing saturates; elements are rounded to nearest-even e4m3.  No global amax
// pass, no delayed-scaling state: each block's scale depends on that block alone.
//
// GEMM (vs_gemm_mxfp8): C[M, N] = sum_k A[m, k] B[n, k] (both k-contiguous fp8, nn.Linear layout for
// B) with scales sa[M][K/32], sb[N][K/32]; the f32 tile then runs the same epilogue as vs_gemm
// (bias, GELU + stored gelu', residual, bf16 / f32 output).  256 x 128 tile, 8 waves (4 x 2, 64 x 64
// per wave: 2 x 2 tiles of 32 x 32), 128-deep k-steps (two 64-deep MFMA k-steps), 3-stage LDS-DMA
// ring of 49.5 KB stages (fp8 rows of 128 B with a 16-B chunk XOR of (row >> 1) & 7; one dword of
// scales per row); operand layout of the 32x32x64 f8 MFMA: lane (r = lane & 31, h = lane >> 5)
// holds row r, k = 16 h .. 16 h + 15 in VGPRs 0-3 and k = 32 + 16 h .. in VGPRs 4-7 (32 bytes), and
// its scale (byte 0 of the scale VGPR: the instruction reads byte 0 whatever OPSEL says) is that
// row's scale of k-block h (block 0 = k 0-31 = VGPRs 0-3 of both halves, block 1 = VGPRs 4-7).
#include "common.h"
#include "gemm_common.h"

namespace vs {

typedef __attribute__((ext_vector_type(8))) int i32x8;

// e4m3 (OCP) of 8 floats packed into 2 dwords (element 0 in the lowest byte)
__device__ __forceinline__ uint2 fp8x8(const float (&v)[8]) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
  return make_uint2((uint32_t)lo, (uint32_t)hi);
}

// E8M0 exponent e (biased, as stored) with 2^(e - 127) >= amax / 448, and the multiplier 2^-(e - 127)
__device__ __forceinline__ uint32_t mx_scale(float amax, float& inv) {
  if (!(amax > 0.f) || !(amax < 3.0e38f)) {  // zero block (or non-finite input): scale 1
    inv = 1.f;
    return 127u;
  }
  const uint32_t b = __float_as_uint(amax * (1.0f / 448.0f));
  int e = (int)((b >> 23) & 0xff) - 127;
  if ((b & 0x7fffff) != 0) e += 1;  // ceil(log2) of a normal float
  if (((b >> 23) & 0xff) == 0) e = -126;  // subnormal ratio: the smallest scale that still fits
  e = e < -126 ? -126 : (e > 127 ? 127 : e);
  inv = __uint_as_float((uint32_t)(127 - e) << 23);
  return (uint32_t)(e + 127);
}

// one thread per (row, 32-element block): 32 elements in, 32 bytes + 1 scale byte out
template <typename T>
__global__ __launch_bounds__(256) void quant_mxfp8_kernel(const T* __restrict__ x, int64_t ldx, int64_t M, int64_t K,
                                                          uint8_t* __restrict__ q, int64_t ldq,
                                                          uint8_t* __restrict__ sc, int64_t ldsc) {
  const int64_t nb = K / 32;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * nb) return;
  const int64_t m = i / nb, kb = i % nb;
  float v[32];
  if constexpr (std::is_same_v<T, float>) {
    const float4* p = (const float4*)(x + m * ldx + kb * 32);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float4 f = p[c];
      v[4 * c] = f.x; v[4 * c + 1] = f.y; v[4 * c + 2] = f.z; v[4 * c + 3] = f.w;
    }
  } else {
    const uint4* p = (const uint4*)(x + m * ldx + kb * 32);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 u = p[c];
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[8 * c + 2 * k] = __uint_as_float(w[k] << 16);
        v[8 * c + 2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      }
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < 32; ++k) amax = fmaxf(amax, fabsf(v[k]));
  float inv;
  const uint32_t e = mx_scale(amax, inv);
  uint4* dst = (uint4*)(q + m * ldq + kb * 32);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[k] = v[16 * c + k] * inv;
      b[k] = v[16 * c + 8 + k] * inv;
    }
    const uint2 lo = fp8x8(a), hi = fp8x8(b);
    dst[c] = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
  sc[m * ldsc + kb] = (uint8_t)e;
}

// ---------------------------------------------------------------------------------------------
// GEMM
// ---------------------------------------------------------------------------------------------
constexpr int kFp8BM = 256, kFp8BN = 128, kFp8KT = 128;
constexpr int kFp8ABytes = kFp8BM * kFp8KT, kFp8BBytes = kFp8BN * kFp8KT;
constexpr int kFp8Stage = kFp8ABytes + kFp8BBytes + 4 * (kFp8BM + kFp8BN);

template <uint32_t EF>
__global__ __launch_bounds__(512, 1) void gemm_mxfp8_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                            const uint8_t* __restrict__ sa, int64_t ldsa,
                                                            const uint8_t* __restrict__ B, int64_t ldb,
                                                            const uint8_t* __restrict__ sb, int64_t ldsb, int64_t K,
                                                            GridMap g, EpiParams e) {
  constexpr int LDT = kFp8BN + 4;
  constexpr int SMEM = 3 * kFp8Stage > (kFp8BM / 2) * LDT * 4 ? 3 * kFp8Stage : (kFp8BM / 2) * LDT * 4;  // 148.5 KB
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  int nt, mt, split;
  map_block(g, nt, mt, split);
  (void)split;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t m0 = (int64_t)mt * kFp8BM, n0 = (int64_t)nt * kFp8BN;
  const int nk = (int)(K / kFp8KT);

  // per-lane DMA source offsets (bytes, step-invariant; the k-step adds 128 B of data and 4 B of scales)
  // A: 32 wave-instructions of 1 KB = 8 rows x 8 chunks each, 4 per wave; B: 16, 2 per wave
  uint32_t oa[4], ob[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int P = 64 * (wid * 4 + k) + lane, r = P >> 3, cp = P & 7;
    const int64_t row = m0 + r < e.M ? m0 + r : e.M - 1;  // rows past M re-read the last row
    oa[k] = (uint32_t)(row * lda + 16 * (cp ^ ((r >> 1) & 7)));
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int P = 64 * (wid * 2 + k) + lane, r = P >> 3, cp = P & 7;
    const int64_t row = n0 + r < e.N ? n0 + r : e.N - 1;
    ob[k] = (uint32_t)(row * ldb + 16 * (cp ^ ((r >> 1) & 7)));
  }
  // scales: one dword (4 k-blocks) per row and k-step, 4 B per lane: A rows 64 w + lane (waves 0-3),
  // B rows 64 (w - 4) + lane (waves 4-5)
  uint32_t os = 0;
  if (wid < 4) {
    const int64_t row = m0 + 64 * wid + lane < e.M ? m0 + 64 * wid + lane : e.M - 1;
    os = (uint32_t)(row * ldsa);
  } else if (wid < 6) {
    const int64_t row = n0 + 64 * (wid - 4) + lane < e.N ? n0 + 64 * (wid - 4) + lane : e.N - 1;
    os = (uint32_t)(row * ldsb);
  }
  auto issue = [&](int t, char* st) {
    const uint8_t* a = A + (int64_t)t * kFp8KT;
    const uint8_t* b = B + (int64_t)t * kFp8KT;
#pragma unroll
    for (int k = 0; k < 4; ++k) glds16_asm_so(a, oa[k], st + 1024 * (wid * 4 + k));
#pragma unroll
    for (int k = 0; k < 2; ++k) glds16_asm_so(b, ob[k], st + kFp8ABytes + 1024 * (wid * 2 + k));
    if (wid < 4) glds4_asm_so(sa + 4 * t, os, st + kFp8ABytes + kFp8BBytes + 256 * wid);
    else if (wid < 6) glds4_asm_so(sb + 4 * t, os, st + kFp8ABytes + kFp8BBytes + 4 * kFp8BM + 256 * (wid - 4));
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int rr = lane & 31, h = lane >> 5;
  // 32 bytes of `row` for MFMA k-step kk: VGPRs 0-3 = k 64 kk + 16 h .. + 15 and VGPRs 4-7 =
  // k 64 kk + 32 + 16 h .. + 15.  The instruction's 32-element scale block 0 is VGPRs 0-3 of BOTH lane
  // halves (its scale from lane h = 0), block 1 VGPRs 4-7 (scale from lane h = 1): measured with a
  // single nonzero k and a distinct scale per block (test_gpu_fp8.py map (k)).  A data-only test cannot
  // see this (any k permutation shared by A and B gives the same product).
  auto frag = [&](const char* img, int row, int kk) {
    const int key = (row >> 1) & 7, c0 = 4 * kk + h;
    const u32x4v lo = *(const u32x4v*)(img + row * 128 + 16 * (c0 ^ key));
    const u32x4v hi = *(const u32x4v*)(img + row * 128 + 16 * ((c0 + 2) ^ key));
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto compute = [&](const char* st) {
    const char* sA = st;
    const char* sB = st + kFp8ABytes;
    const uint32_t* scA = (const uint32_t*)(st + kFp8ABytes + kFp8BBytes);
    const uint32_t* scB = scA + kFp8BM;
    uint32_t ua[2], ub[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) ua[i] = scA[wr * 64 + 32 * i + rr];
#pragma unroll
    for (int j = 0; j < 2; ++j) ub[j] = scB[wc * 64 + 32 * j + rr];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      i32x8 af[2], bfr[2];
      int sca[2], scb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = frag(sA, wr * 64 + 32 * i + rr, kk);
        sca[i] = (int)vopaque(ua[i] >> (8 * (2 * kk + h)));  // opaque: a constant scale would be taken as f32
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bfr[j] = frag(sB, wc * 64 + 32 * j + rr, kk);
        scb[j] = (int)vopaque(ub[j] >> (8 * (2 * kk + h)));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, sca[i], 0,
                                                                      scb[j]);
    }
  };
  // 3-stage ring with one step in flight across each barrier (as gemm_bf16_big_kernel): a wave's
  // pieces per step are 4 (A) + 2 (B) + 1 scale dword piece for waves 0-5
  auto step = [&](int t, auto sc) {
    constexpr int S = decltype(sc)::value;  // == t % 3
    if (t + 1 < nk) {
      if (wid < 6) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) issue(t + 2, smem + ((S + 2) % 3) * kFp8Stage);
    compute(smem + S * kFp8Stage);
  };
  issue(0, smem);
  if (nk > 1) issue(1, smem + kFp8Stage);
  for (int t = 0; t < nk; t += 3) {
    step(t, IC<0>{});
    if (t + 1 < nk) step(t + 1, IC<1>{});
    if (t + 2 < nk) step(t + 2, IC<2>{});
  }
  // epilogue: the f32 tile staged in two 128-row halves, 8-column groups per thread (vs_gemm's epilogue)
  float* stg = (float*)smem;
  constexpr int CPR = kFp8BN / 8;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    __syncthreads();
    if ((wr >> 1) == part) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            stg[((wr & 1) * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * LDT + wc * 64 + 32 * j + rr] =
                acc[i][j][r] * e.alpha;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = p * 32 + tid / CPR, cg = tid % CPR;
      const int64_t m = m0 + part * 128 + row, n = n0 + cg * 8;
      if (m < e.M) {
        const float* src = stg + row * LDT + cg * 8;
        float v[8];
        const float4 a = *(const float4*)src;
        const float4 b = *(const float4*)(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_eight<EF>(e, m, n, v, false);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace vs

using namespace vs;

extern "C" int vs_quant_mxfp8(int32_t in_dtype, int64_t M, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                              void* scales, int64_t ld_scales, void* stream) {
  VS_REQUIRE(in_dtype == VS_F32 || in_dtype == VS_BF16, "vs_quant_mxfp8: in_dtype must be VS_F32 or VS_BF16");
  VS_REQUIRE(M >= 0 && K % 32 == 0, "vs_quant_mxfp8: K must be a multiple of 32");
  if (M == 0 || K == 0) return VS_OK;
  VS_REQUIRE(x && q && scales, "vs_quant_mxfp8: null pointer");
  VS_REQUIRE(aligned16(x) && aligned16(q) && ldx >= K && ldq >= K && ld_scales >= K / 32 && ldq % 16 == 0 &&
                 (ldx * (int64_t)esize(in_dtype)) % 16 == 0,
             "vs_quant_mxfp8: rows must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_MISC, s,
                    (double)M * (double)K * ((double)esize(in_dtype) + 1.0) + (double)M * (double)(K / 32));
  const int64_t n = M * (K / 32);
  const unsigned grid = (unsigned)cdiv(n, 256);
  if (in_dtype == VS_BF16)
    hipLaunchKernelGGL(quant_mxfp8_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, ldx, M, K,
                       (uint8_t*)q, ldq, (uint8_t*)scales, ld_scales);
  else
    hipLaunchKernelGGL(quant_mxfp8_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, ldx, M, K, (uint8_t*)q,
                       ldq, (uint8_t*)scales, ld_scales);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

template <uint32_t EF>
static void launch_mxfp8(const vs_gemm_desc* d, const uint8_t* sa, int64_t ldsa, const uint8_t* sb, int64_t ldsb,
                         const GridMap& g, const EpiParams& e, hipStream_t s) {
  const unsigned nblk = (unsigned)(g.tiles_m * g.tiles_n);
  hipLaunchKernelGGL(gemm_mxfp8_kernel<EF>, dim3(nblk), dim3(512), 0, s, (const uint8_t*)d->a, d->lda, sa, ldsa,
                     (const uint8_t*)d->b, d->ldb, sb, ldsb, d->K, g, e);
}

extern "C" int vs_gemm_mxfp8(const vs_gemm_desc* d, const void* scale_a, int64_t ld_scale_a, const void* scale_b,
                             int64_t ld_scale_b, void* stream) {
  VS_REQUIRE(d && scale_a && scale_b, "vs_gemm_mxfp8: null descriptor / scales");
  VS_REQUIRE(d->dtype == VS_FP8 && d->a_kcontig && d->b_kcontig, "vs_gemm_mxfp8: A and B must be k-contiguous VS_FP8");
  VS_REQUIRE(d->out_dtype == VS_F32 || d->out_dtype == VS_BF16, "vs_gemm_mxfp8: bad out_dtype");
  if (d->M == 0 || d->N == 0) return VS_OK;
  VS_REQUIRE(d->a && d->b && d->c, "vs_gemm_mxfp8: null operand");
  VS_REQUIRE(d->K % kFp8KT == 0 && d->K > 0 && d->N % kFp8BN == 0, "vs_gemm_mxfp8: needs K % 128 == 0, N % 128 == 0");
  VS_REQUIRE(aligned16(d->a) && aligned16(d->b) && d->lda % 16 == 0 && d->ldb % 16 == 0 && d->lda >= d->K &&
                 d->ldb >= d->K && ld_scale_a % 4 == 0 && ld_scale_b % 4 == 0 && ld_scale_a >= d->K / 32 &&
                 ld_scale_b >= d->K / 32 && (((uintptr_t)scale_a) & 3) == 0 && (((uintptr_t)scale_b) & 3) == 0,
             "vs_gemm_mxfp8: rows must be 16-byte aligned, scale rows 4-byte aligned");
  VS_REQUIRE(d->M * d->lda < (int64_t(1) << 31) && d->N * d->ldb < (int64_t(1) << 31),
             "vs_gemm_mxfp8: operand too large for 32-bit DMA offsets");
  VS_REQUIRE(d->ldc >= d->N && d->ldc % 8 == 0 && aligned16(d->c), "vs_gemm_mxfp8: C rows must be 16-byte aligned");
  const uint32_t f = d->epilogue;
  VS_REQUIRE(!(f & VS_EPI_BIAS) || (d->bias && aligned16(d->bias)), "vs_gemm_mxfp8: BIAS needs an aligned bias");
  VS_REQUIRE(!(f & VS_EPI_RESIDUAL) || (d->residual && aligned16(d->residual) && d->ld_residual % 4 == 0),
             "vs_gemm_mxfp8: RESIDUAL needs an aligned residual");
  VS_REQUIRE(!(f & VS_EPI_GELU) || (d->aux_out && aligned16(d->aux_out) && d->ld_aux_out % 8 == 0),
             "vs_gemm_mxfp8: GELU needs an aligned aux_out");
  EpiParams e = {};
  e.M = d->M; e.N = d->N; e.c = d->c; e.ldc = d->ldc;
  e.out_bf16 = d->out_dtype == VS_BF16;
  e.op_bf16 = 1;  // GELU / GELU' rounding as the bf16 path (the block's activations are bf16)
  e.flags = f; e.alpha = d->alpha; e.bias = d->bias;
  e.residual = d->residual; e.ldr = d->ld_residual;
  e.aux_out = d->aux_out; e.ld_aux_out = d->ld_aux_out;
  e.vec_ok = 1;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(g_timer_tag >= 0 ? g_timer_tag : VS_TIMER_GEMM, s,
                    (double)(d->M + d->N) * (double)d->K * (1.0 + 1.0 / 32.0) +
                        (double)d->M * (double)d->N * (d->out_dtype == VS_BF16 ? 2.0 : 4.0));
  GridMap g = {(int)(d->N / kFp8BN), (int)cdiv(d->M, kFp8BM), 1, d->K};
  count_path(VS_PATH_GEMM_FP8);
  const uint8_t* sa = (const uint8_t*)scale_a;
  const uint8_t* sb = (const uint8_t*)scale_b;
  if (f == VS_EPI_BIAS) launch_mxfp8<(uint32_t)VS_EPI_BIAS>(d, sa, ld_scale_a, sb, ld_scale_b, g, e, s);
  else if (f == (VS_EPI_BIAS | VS_EPI_RESIDUAL))
    launch_mxfp8<(uint32_t)(VS_EPI_BIAS | VS_EPI_RESIDUAL)>(d, sa, ld_scale_a, sb, ld_scale_b, g, e, s);
  else if (f == (VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD))
    launch_mxfp8<(uint32_t)(VS_EPI_BIAS | VS_EPI_GELU | VS_EPI_GELU_GRAD)>(d, sa, ld_scale_a, sb, ld_scale_b, g, e, s);
  else if (f == 0) launch_mxfp8<0u>(d, sa, ld_scale_a, sb, ld_scale_b, g, e, s);
  else VS_REQUIRE(false, "vs_gemm_mxfp8: epilogue must be 0, BIAS, BIAS|RESIDUAL or BIAS|GELU|GELU_GRAD");
  VS_LAUNCH_CHECK();
  return VS_OK;
}
