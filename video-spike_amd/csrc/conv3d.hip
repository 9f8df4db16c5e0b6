// conv3d.hip — the R3D-18 encoder's kernels (BASELINE C4: ResNet-18 3D-conv, 32x112x112 clips, fp32).
//
// The reference has no CNN encoder: these replace what torch runs for a
// torchvision-style r3d_18 behind the plugin surface (nn.Conv3d forward and its autograd dX / dW,
// nn.BatchNorm3d in training mode, the residual add + ReLU, nn.AdaptiveAvgPool3d(1)).
//
// MI355X design (include/vspike.h "R3D-18 video encoder"):
//   * Activations channels-last f32 [N][D][H][W][C]: every (voxel, tap) reads C contiguous floats, so
//     the implicit GEMM's operand gather is 16-B vector loads of whole channel runs.
//   * Conv3d = implicit GEMM, no im2col tensor (an explicit im2col of layer1 at 16 clips would be
//     11 GB written and read back per conv: 2x the conv's f32-MFMA time in HBM traffic).  Rows = output
//     voxels, k = (tap, channel), the A operand gathered per k-tile into LDS (zero outside the padded
//     volume), the weights K-contiguous [Co][taps][Ci] as the B operand; v_mfma_f32_16x16x4_f32 (exact
//     f32: a k-ordered fmaf chain).  128 x 64 output tile, 4 waves of 64 x 32, BK = 32, register-staged
//     prefetch into a 2-stage LDS ring (the loads of k-tile t+1 in flight under the MFMAs of t).
//   * dX of a stride-1 conv is the same kernel on dy with the flipped offsets; of a stride-2 conv one
//     launch per parity class of the input positions with only the taps that reach it (1..8 of 27),
//     so no MFMA multiplies a structural zero; weights regrouped per class ([Ci][class taps][Co]).
//   * dW: tiles of (64 out channels x 64 k) summed over the output voxels (the gather as the B
//     operand), split over the voxel rows; partial tiles summed in split order (no atomics).
//   * BatchNorm3d statistics ride in the forward conv's epilogue (per 128-row tile column sums of y and
//     of the squared deviations from the tile mean), merged in f64 in a fixed order (Chan); apply (+ residual + ReLU) and the backward are
//     channel-vectorised elementwise passes with fixed-order reductions.
#include <cstdlib>

#include "common.h"

namespace vs {

// ------------------------------------------------------------------------------------------------
// geometry of one implicit-GEMM launch
// ------------------------------------------------------------------------------------------------
struct Igemm {
  const float* x;             // gathered operand, channels-last [N][Di][Hi][Wi][C]
  int N, Di, Hi, Wi, C, cshift;
  int Gd, Gh, Gw;             // GEMM row grid: rows = N * Gd * Gh * Gw
  int sd, sh, sw;             // input step per grid step
  // taps: per dim j in [0, cnt): input offset o0 + ostep * j (added to g * s)
  int cd, ch, cw;
  int od0, oh0, ow0, ods, ohs, ows;
  const float* w;             // [Ng][K] K-contiguous, K = cd*ch*cw * C
  int Ng, K;
  float* y;                   // output, channels-last with Ng channels, storage grid Od x Oh x Ow
  int Od, Oh, Ow;
  int ysd, ysh, ysw, yod, yoh, yow;   // output voxel = g * ys + yo
  int accumulate;
  float* stats;               // [tiles_m][2][Ng] per 128-row tile: column sum of y, sum of (y - tile mean)^2; or null
  int64_t M;
};

__device__ __forceinline__ int divq(int x, int d, float inv) {
  // x / d for 0 <= x < 2^24 by a float reciprocal and one correction step (24-bit multiply: full
  // rate, where v_mul_lo_u32 is a quarter-rate instruction)
  int q = (int)((float)x * inv);
  int r = x - (int)__umul24(q, d);
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}
__device__ __forceinline__ int mul24(int a, int b) { return (int)__umul24(a, b); }  // a, b in [0, 2^24)
// 16-B load through a raw buffer resource: an offset past num_records (kOob) returns zeros with no
// exec-mask branch or zeroing moves (the host keeps every operand below 2^31 bytes)
constexpr uint32_t kOob = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t conv_rsrc(const float* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// f32 MFMA operand images: row-major [rows][k], 34-float rows (conflict-free ds_read_b32 of 16 rows x
// 2 k per 32-lane half: bank = 2 row + k), filled by two ds_write_b64 per gathered float4
constexpr int kLdA = 34;

__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(Igemm g) {
  constexpr int BM = 128, BN = 64, BK = 32, LD = kLdA;
  constexpr int SA = BM * LD, SB = BN * LD, STAGE = SA + SB;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int tiles_n = g.Ng / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tiles_n, nt = bid % tiles_n;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int chunk = tid & 7;  // float4 index along k of this thread's operand loads

  // the 4 A rows of this thread (rows tid/8 + 32 s): voxel coordinates of the gathered input and the
  // voxel index of the row's tap-(0,0,0) origin.  Operand offsets are 32-bit (the host checks the
  // gathered volume x C < 2^31): the int64 index chain and the two integer divisions of the tap
  // were 31 v_mul_lo_u32 + 12 64-bit multiply-adds (quarter rate) per k step
  int rz[4], ry[4], rx[4], rvb[4];
  bool rok[4];
  {
    const float ihw = 1.0f / (float)g.Gw, ihh = 1.0f / (float)g.Gh, ihd = 1.0f / (float)g.Gd;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t m = m0 + (tid >> 3) + 32 * s;
      rok[s] = m < g.M;
      const int mm = rok[s] ? (int)m : 0;
      const int q1 = divq(mm, g.Gw, ihw), gw = mm - mul24(q1, g.Gw);
      const int q2 = divq(q1, g.Gh, ihh), gh = q1 - mul24(q2, g.Gh);
      const int n = divq(q2, g.Gd, ihd), gd = q2 - mul24(n, g.Gd);
      rz[s] = gd * g.sd;
      ry[s] = gh * g.sh;
      rx[s] = gw * g.sw;
      rvb[s] = ((n * g.Di + rz[s]) * g.Hi + ry[s]) * g.Wi + rx[s];
    }
  }
  const int chw = g.ch * g.cw;
  const float ichw = 1.0f / (float)chw, icw = 1.0f / (float)g.cw;
  const auto rsx = conv_rsrc(g.x, (g.N * g.Di * g.Hi * g.Wi) << (g.cshift + 2));
  const auto rsw = conv_rsrc(g.w, g.Ng * g.K * 4);
  auto load_a = [&](float4 (&ra)[4], int k0) {
    const int k = k0 + chunk * 4;
    const bool kok = k < g.K;
    const int tap = k >> g.cshift, c = k & (g.C - 1);
    const int jd = divq(tap, chw, ichw), jr = tap - mul24(jd, chw);
    const int jh = divq(jr, g.cw, icw), jw = jr - mul24(jh, g.cw);
    const int oz = g.od0 + __mul24(g.ods, jd), oy = g.oh0 + __mul24(g.ohs, jh), ox = g.ow0 + __mul24(g.ows, jw);
    const int toff = __mul24(__mul24(oz, g.Hi) + oy, g.Wi) + ox;  // voxel offset of the tap (may be < 0)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int z = rz[s] + oz, yy = ry[s] + oy, xx = rx[s] + ox;
      const bool ok = kok && rok[s] && (unsigned)z < (unsigned)g.Di && (unsigned)yy < (unsigned)g.Hi &&
                      (unsigned)xx < (unsigned)g.Wi;
      ra[s] = bload4(rsx, ok ? (uint32_t)(((rvb[s] + toff) << g.cshift) + c) * 4u : kOob);
    }
  };
  auto load_b = [&](float4 (&rb)[2], int k0) {
    const int k = k0 + chunk * 4;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int n = n0 + (tid >> 3) + 32 * s;
      rb[s] = bload4(rsw, k < g.K ? (uint32_t)(n * g.K + k) * 4u : kOob);
    }
  };
  auto store = [&](float* st, const float4 (&ra)[4], const float4 (&rb)[2]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float* d = st + ((tid >> 3) + 32 * s) * LD + chunk * 4;
      *(float2*)d = make_float2(ra[s].x, ra[s].y);
      *(float2*)(d + 2) = make_float2(ra[s].z, ra[s].w);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float* d = st + SA + ((tid >> 3) + 32 * s) * LD + chunk * 4;
      *(float2*)d = make_float2(rb[s].x, rb[s].y);
      *(float2*)(d + 2) = make_float2(rb[s].z, rb[s].w);
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  float4 ra[4], rb[2];
  load_a(ra, 0);
  load_b(rb, 0);
  store(smem, ra, rb);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const float* sa = smem + (t & 1) * STAGE;
    const float* sb = sa + SA;
    const bool more = t + 1 < nk;
    if (more) {
      load_a(ra, (t + 1) * BK);
      load_b(rb, (t + 1) * BK);
    }
#pragma unroll
    for (int sub = 0; sub < BK / 4; ++sub) {
      const int kk = 4 * sub + (lane >> 4);
      float af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = sa[(wr * 64 + i * 16 + (lane & 15)) * LD + kk];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = sb[(wc * 32 + j * 16 + (lane & 15)) * LD + kk];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(smem + ((t + 1) & 1) * STAGE, ra, rb);
    __syncthreads();
  }

  // epilogue: acc[i][j][r] = C[wr*64 + i*16 + 4*(lane>>4) + r][wc*32 + j*16 + (lane&15)]
  float csum[2] = {0.f, 0.f};
  {
    const float ihw = 1.0f / (float)g.Gw, ihh = 1.0f / (float)g.Gh, ihd = 1.0f / (float)g.Gd;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        const int mm = (int)m;
        const int q1 = divq(mm, g.Gw, ihw), gw = mm - q1 * g.Gw;
        const int q2 = divq(q1, g.Gh, ihh), gh = q1 - q2 * g.Gh;
        const int n = divq(q2, g.Gd, ihd), gd = q2 - n * g.Gd;
        const int64_t vox = (((int64_t)n * g.Od + gd * g.ysd + g.yod) * g.Oh + gh * g.ysh + g.yoh) * g.Ow +
                            gw * g.ysw + g.yow;
        float* dst = g.y + vox * g.Ng + n0 + wc * 32 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v = acc[i][j][r];
          if (g.accumulate) v += dst[j * 16];
          dst[j * 16] = v;
          acc[i][j][r] = v;  // the stored value, for the tile's second statistics pass
          csum[j] += v;
        }
      }
  }
  if (g.stats) {
    // BatchNorm partials per 128-row tile: the column sum S and the sum of squared deviations from
    // the TILE's own column mean, M2 = sum (y - S/n)^2 (two passes over the registers), merged later
    // with Chan's formula in f64.  A single-pass sum of y^2 loses the variance to cancellation in f32
    // when |mean| >> std (trained weights): E[y^2] - mean^2.
    __shared__ float red[2][2][64];
    __syncthreads();  // (smem reads done; red is a separate array written once)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v = csum[j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red[wr][0][wc * 32 + j * 16 + lane] = v;
    }
    __syncthreads();
    const int64_t nrows = g.M - m0 < BM ? g.M - m0 : BM;
    const float inv_n = 1.0f / (float)nrows;
    float csq[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = wc * 32 + j * 16 + (lane & 15);
      const float mu = (red[0][0][col] + red[1][0][col]) * inv_n;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t m = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + r;
          const float dv = acc[i][j][r] - mu;
          csq[j] += m < g.M ? dv * dv : 0.f;
        }
      float q = csq[j];
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) red[wr][1][wc * 32 + j * 16 + lane] = q;
    }
    __syncthreads();
    if (tid < 128) {
      const int which = tid >> 6, col = tid & 63;
      g.stats[((int64_t)mt * 2 + which) * g.Ng + n0 + col] = red[0][which][col] + red[1][which][col];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient: dw[o][k] (+)= sum_m dy[m][o] * gather(x)[m][k]
// ------------------------------------------------------------------------------------------------
struct ConvDw {
  const float* x;
  int N, Di, Hi, Wi, C, cshift;
  int Do, Ho, Wo;             // output (row) grid
  int sd, sh, sw, pd, ph, pw;
  int kd, kh, kw;
  const float* dy;            // [M][Co]
  int Co, K;                  // K = kd*kh*kw*C
  int64_t M;
  int splits, steps_per_split;  // rows of a split: steps_per_split * 32
  float* part;                // [splits][Co][Kp], Kp = tiles_k * 64
  int Kp;
};

// BKK = 64 or 128 k columns per tile: the wider tile reads the dy slab (the tile's A operand) half as
// often (the dy of one voxel row slab is re-read by every k tile of the product) but measured slower:
// 64 is the default (VS_KNOB_CONV_DW128)
// M32 (BKK = 64 only, VS_KNOB_CONV_MFMA = 1): v_mfma_f32_32x32x2_f32 on each wave's 32 x 32 output block
// instead of four v_mfma_f32_16x16x4_f32: the same MACs and operand reads (one A and one B dword per lane
// per 2 k) with half the MFMA instructions (half the issue slots the matrix pipe takes from the gather's
// VALU / LDS work).  Measured SLOWER at C4 (conv dW 37.3 vs 32.5 ms/step, profiles/r06_r3d_ab_mfma.json:
// one dependent 64-cycle accumulation chain per wave instead of four independent 32-cycle ones)
template <int BKK, bool M32 = false>
__global__ __launch_bounds__(256, 2) void conv_dw_kernel(ConvDw g) {
  static_assert(!M32 || BKK == 64, "M32: one 32 x 32 block per wave");
  constexpr int BO = 64, BM = 32, LDO = 80, LD = BKK + 16;   // row strides % 32 == 16: conflict-free b32 reads
  constexpr int SO = BM * LDO, STAGE = SO + BM * LD;
  constexpr int KCH = BKK / 4, XR = 256 / KCH, XS = BM / XR;  // x gather: float4 chunks per row, rows per pass, passes
  constexpr int NJ = BKK / 32;                                // 16-column fragments per wave (2 waves along k)
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int tiles_o = g.Co / BO, tiles_k = g.Kp / BKK;  // Kp: K rounded up to BKK
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / (tiles_o * tiles_k), rem = bid % (tiles_o * tiles_k);
  const int ot = rem / tiles_k, kt = rem % tiles_k;
  const int o0 = ot * BO, k0 = kt * BKK;
  const int64_t mb = (int64_t)split * g.steps_per_split * BM;
  int64_t me = mb + (int64_t)g.steps_per_split * BM;
  if (me > g.M) me = g.M;
  const int nsteps = me > mb ? (int)((me - mb + BM - 1) / BM) : 0;
  const int chunk = tid & 15;  // float4 index along o (dy)
  const int xchunk = tid % KCH;  // float4 index along k (gather)
  // the gather's k chunk: tap and channel are fixed for the whole launch of this thread
  const int k = k0 + xchunk * 4;
  const bool kok = k < g.K;
  const int tap = k >> g.cshift, c = k & (g.C - 1);
  const int khw = g.kh * g.kw;
  const int td = tap / khw, tr = tap - td * khw, th = tr / g.kw, tw = tr - th * g.kw;
  const int oz = td - g.pd, oy = th - g.ph, ox = tw - g.pw;
  const float ihw = 1.0f / (float)g.Wo, ihh = 1.0f / (float)g.Ho, ihd = 1.0f / (float)g.Do;

  // Operand addresses as 32-bit element offsets (the host checks M < 2^24, M Co < 2^31 and the input
  // volume x C < 2^31).  The gather's voxel coordinates are advanced incrementally: each thread keeps
  // the (n, z0 = gd sd, y0 = gh sh, x0 = gw sw) of its row slots and adds the mixed-radix digits of
  // one step (32 rows) with one conditional carry per digit, instead of three divisions per row and
  // step (the int64 index chains with three float-reciprocal divisions per row were ~200 VALU per
  // step, VALU : MFMA 6.5 : 1 in the counters, profiles/r05_pmc_convdw.json)
  const int me32 = (int)me, mb32 = (int)mb;
  const auto rsx = conv_rsrc(g.x, (g.N * g.Di * g.Hi * g.Wi) << (g.cshift + 2));
  const auto rsdy = conv_rsrc(g.dy, (int)g.M * g.Co * 4);
  const int XW = g.Wo * g.sw, YH = g.Ho * g.sh, ZD = g.Do * g.sd;
  int cW, cH, cD, cN;  // the step's digits (x0, y0, z0 strides; n count)
  {
    int q = BM;
    cW = (q % g.Wo) * g.sw; q /= g.Wo;
    cH = (q % g.Ho) * g.sh; q /= g.Ho;
    cD = (q % g.Do) * g.sd; q /= g.Do;
    cN = q;
  }
  int sx0[XS], sy0[XS], sz0[XS], sn[XS];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int m = mb32 + tid / KCH + XR * s;
    const int mm = m < me32 ? m : 0;  // (a slot past the split end only ever loads zeros)
    const int q1 = divq(mm, g.Wo, ihw), gw = mm - mul24(q1, g.Wo);
    const int q2 = divq(q1, g.Ho, ihh), gh = q1 - mul24(q2, g.Ho);
    const int n = divq(q2, g.Do, ihd), gd = q2 - mul24(n, g.Do);
    sx0[s] = gw * g.sw;
    sy0[s] = gh * g.sh;
    sz0[s] = gd * g.sd;
    sn[s] = n;
  }
  auto advance = [&]() {
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      int x0 = sx0[s] + cW;
      const bool cw = x0 >= XW;
      x0 -= cw ? XW : 0;
      int y0 = sy0[s] + cH + (cw ? g.sh : 0);
      const bool ch = y0 >= YH;
      y0 -= ch ? YH : 0;
      int z0 = sz0[s] + cD + (ch ? g.sd : 0);
      const bool cd = z0 >= ZD;
      z0 -= cd ? ZD : 0;
      sx0[s] = x0;
      sy0[s] = y0;
      sz0[s] = z0;
      sn[s] += cN + (cd ? 1 : 0);
    }
  };
  // load(step) reads the slots' current coordinates: called for steps 0, 1, 2, ... in order, each
  // call followed by advance()
  auto load = [&](float4 (&rd)[2], float4 (&rx)[XS], int step) {
    const int mstep = mb32 + step * BM;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int m = mstep + (tid >> 4) + 16 * s;
      const bool ok = m < me32;
      rd[s] = bload4(rsdy, ok ? (uint32_t)(mul24(m, g.Co) + o0 + chunk * 4) * 4u : kOob);
    }
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      const int m = mstep + tid / KCH + XR * s;
      const int z = sz0[s] + oz, yy = sy0[s] + oy, xx = sx0[s] + ox;
      const bool in = m < me32 && kok && (unsigned)z < (unsigned)g.Di && (unsigned)yy < (unsigned)g.Hi &&
                      (unsigned)xx < (unsigned)g.Wi;
      const int vox = mul24(mul24(mul24(sn[s], g.Di) + z, g.Hi) + yy, g.Wi) + xx;
      rx[s] = bload4(rsx, in ? (uint32_t)((vox << g.cshift) + c) * 4u : kOob);
    }
    advance();
  };

  auto store = [&](float* st, const float4 (&rd)[2], const float4 (&rx)[XS]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) *(float4*)(st + ((tid >> 4) + 16 * s) * LDO + chunk * 4) = rd[s];
#pragma unroll
    for (int s = 0; s < XS; ++s) *(float4*)(st + SO + (tid / KCH + XR * s) * LD + xchunk * 4) = rx[s];
  };

  // blocked accumulation: the MFMA chain runs over 16 steps (512 voxels), then folds into tot —
  // one f32 chain over a whole split (up to ~40k voxels at 16 clips) lets rounding grow with its
  // length, and these sums cancel strongly (the gradient of a conv feeding a BatchNorm)
  f32x4 acc[2][NJ], tot[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x16 acc32, tot32;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc32[r] = tot32[r] = 0.f;
  float4 rd[2], rx[XS];
  if (nsteps > 0) {
    load(rd, rx, 0);
    store(smem, rd, rx);
  }
  if constexpr (!M32) {
    // Two steps of global loads in flight (round 6): step t+2's dy / gather rows are loaded into the
    // register set not being stored this step, so a load has a whole step of MFMAs plus the next
    // step's to land before its LDS store (one step ahead, the stores waited on L2 / HBM latency:
    // wait_inst 0.62 of wave cycles, profiles/r05_pmc_convdw.json).  The two sets alternate by unrolling.
    float4 rdb[2], rxb[XS];
    if (nsteps > 1) load(rd, rx, 1);
    __syncthreads();
    constexpr int NS = BM / 4, HS = NS / 2;
    auto body = [&](int t, float4 (&sd1)[2], float4 (&sx1)[XS], float4 (&ld2)[2], float4 (&lx2)[XS]) {
      const float* sd_ = smem + (t & 1) * STAGE;
      const float* sx = sd_ + SO;
      if (t + 2 < nsteps) load(ld2, lx2, t + 2);
      float af[NS][2], bfr[NS][NJ];
      auto rd_ops = [&](int sub) {
        const int mrow = 4 * sub + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 2; ++i) af[sub][i] = sd_[mrow * LDO + wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[sub][j] = sx[mrow * LD + wc * (BKK / 2) + j * 16 + (lane & 15)];
      };
      auto mm_ops = [&](int sub) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[sub][i], bfr[sub][j], acc[i][j], 0, 0, 0);
      };
#pragma unroll
      for (int sub = 0; sub < HS; ++sub) rd_ops(sub);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = HS; sub < NS; ++sub) rd_ops(sub);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = 0; sub < HS; ++sub) mm_ops(sub);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = HS; sub < NS; ++sub) mm_ops(sub);
      if (t + 1 < nsteps) store(smem + ((t + 1) & 1) * STAGE, sd1, sx1);
      if ((t & 15) == 15) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            tot[i][j] += acc[i][j];
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
      __syncthreads();
    };
    for (int t = 0; t < nsteps; t += 2) {
      body(t, rd, rx, rdb, rxb);                     // stores step t+1 from (rd, rx), loads t+2 into (rdb, rxb)
      if (t + 1 < nsteps) body(t + 1, rdb, rxb, rd, rx);
    }
  }
  if constexpr (M32) __syncthreads();
  for (int t = 0; M32 && t < nsteps; ++t) {
    const float* sd_ = smem + (t & 1) * STAGE;
    const float* sx = sd_ + SO;
    const bool more = t + 1 < nsteps;
    if (more) load(rd, rx, t + 1);
    // operand fragments read a half-step (4 sub-steps) ahead of their MFMAs: reading each sub-step's
    // 4 values right before its 4 MFMAs (hipcc's choice, reusing 4 registers) serialised every
    // sub-step behind an LDS round trip (conv dW 34.0 -> 32.5 ms/step at C4; the same change in
    // conv_igemm_kernel, 146 VGPRs, measured slower: fwd 25.1 -> 26.2, dX 26.0 -> 26.9)
    if constexpr (M32) {
      // 16 two-row sub-steps: A = dy^T (o = lane & 31, m = 2 sub + lane / 32), B = the gather (k = lane & 31)
      constexpr int NS2 = BM / 2, HS2 = NS2 / 2;
      float a2[NS2], b2[NS2];
      auto rd2 = [&](int sub) {
        const int mrow = 2 * sub + (lane >> 5);
        a2[sub] = sd_[mrow * LDO + wr * 32 + (lane & 31)];
        b2[sub] = sx[mrow * LD + wc * 32 + (lane & 31)];
      };
#pragma unroll
      for (int sub = 0; sub < HS2; ++sub) rd2(sub);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = HS2; sub < NS2; ++sub) rd2(sub);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = 0; sub < HS2; ++sub) acc32 = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[sub], b2[sub], acc32, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sub = HS2; sub < NS2; ++sub) acc32 = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[sub], b2[sub], acc32, 0, 0, 0);
      if (more) store(smem + ((t + 1) & 1) * STAGE, rd, rx);
      if ((t & 15) == 15) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          tot32[r] += acc32[r];
          acc32[r] = 0.f;
        }
      }
      __syncthreads();
      continue;
    }
    constexpr int NS = BM / 4, HS = NS / 2;
    float af[NS][2], bfr[NS][NJ];
    auto rd_ops = [&](int sub) {
      const int mrow = 4 * sub + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) af[sub][i] = sd_[mrow * LDO + wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[sub][j] = sx[mrow * LD + wc * (BKK / 2) + j * 16 + (lane & 15)];
    };
    auto mm_ops = [&](int sub) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[sub][i], bfr[sub][j], acc[i][j], 0, 0, 0);
    };
#pragma unroll
    for (int sub = 0; sub < HS; ++sub) rd_ops(sub);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sub = HS; sub < NS; ++sub) rd_ops(sub);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sub = 0; sub < HS; ++sub) mm_ops(sub);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sub = HS; sub < NS; ++sub) mm_ops(sub);
    if (more) store(smem + ((t + 1) & 1) * STAGE, rd, rx);
    if ((t & 15) == 15) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          tot[i][j] += acc[i][j];
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] += tot[i][j];
  // partial tile (plain stores; the reduce adds the splits in order)
  float* pt = g.part + (int64_t)split * g.Co * g.Kp;
  if constexpr (M32) {
    // 32 x 32 accumulator layout: register r = row 8 (r / 4) + 4 (lane / 32) + r % 4, column lane & 31
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + wr * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
      const int kk = k0 + wc * 32 + (lane & 31);
      pt[(int64_t)o * g.Kp + kk] = acc32[r] + tot32[r];
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wr * 32 + i * 16 + 4 * (lane >> 4) + r;
        const int kk = k0 + wc * (BKK / 2) + j * 16 + (lane & 15);
        pt[(int64_t)o * g.Kp + kk] = acc[i][j][r];
      }
}

// dw[o][k] (=|+=) sum_s part[s][o][k] for k < K (float4 over k when K % 4 == 0)
__global__ __launch_bounds__(256) void conv_dw_reduce(const float* __restrict__ part, int splits, int Co, int K,
                                                      int Kp, float* __restrict__ dw, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)Co * K;
  if (i >= n) return;
  const int o = (int)(i / K), k = (int)(i % K);
  const int64_t src = (int64_t)o * Kp + k, plane = (int64_t)Co * Kp;
  float s = 0.f;
  for (int sp = 0; sp < splits; ++sp) s += part[sp * plane + src];
  dw[i] = accumulate ? dw[i] + s : s;
}

// dX weights of one parity class: wd[ci][(jd, jh, jw)][co] = w[co][td][th][tw][ci], t = t0 + tstep j
__global__ __launch_bounds__(256) void conv_dx_weights(const float* __restrict__ w, int Co, int Ci, int kd, int kh,
                                                       int kw, int cd, int ch, int cw, int t0d, int t0h, int t0w,
                                                       int tsd, int tsh, int tsw, float* __restrict__ wd) {
  const int T = cd * ch * cw;
  const int64_t n = (int64_t)Ci * T * Co;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int co = (int)(i % Co);
  const int64_t q = i / Co;
  const int j = (int)(q % T), ci = (int)(q / T);
  const int jd = j / (ch * cw), jr = j % (ch * cw), jh = jr / cw, jw = jr % cw;
  const int td = t0d + tsd * jd, th = t0h + tsh * jh, tw = t0w + tsw * jw;
  wd[i] = w[((((int64_t)co * kd + td) * kh + th) * kw + tw) * Ci + ci];
}

// ------------------------------------------------------------------------------------------------
// BatchNorm3d
// ------------------------------------------------------------------------------------------------
// The partials are per 128-row tile t (rows [128 t, min(128 t + 128, count))): S_t = sum y and
// M2_t = sum (y - S_t / n_t)^2.  Merged in f64 in a fixed order with Chan's formula: over a set of
// tiles, S = sum S_t, mean = S / n, M2 = sum M2_t + sum n_t (S_t / n_t - mean)^2.
constexpr int kBnTile = 128;
__device__ __forceinline__ double bn_tile_n(int64_t t, int64_t count) {
  const int64_t r = count - t * kBnTile;
  return (double)(r < kBnTile ? r : kBnTile);
}

// level 1: tiles [r0, r0 + 256) of the [rows][2][C] partials, 64 channels per block -> (S_b, M2_b)
__global__ __launch_bounds__(256) void bn_stats_l1(const float* __restrict__ part, int64_t rows, int C,
                                                   int64_t count, double* __restrict__ out) {
  __shared__ double red[2][4][64];
  __shared__ double mean_b[64];
  const int l = threadIdx.x & 63, c = blockIdx.y * 64 + l, grp = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int64_t r1 = r0 + 256 < rows ? r0 + 256 : rows;
  double s = 0.0;
  if (c < C)
    for (int64_t r = r0 + grp; r < r1; r += 4) s += (double)part[(r * 2) * C + c];
  red[0][grp][l] = s;
  __syncthreads();
  if (grp == 0) {
    const double n_b = fmin((double)(r1 - r0) * kBnTile, (double)(count - r0 * kBnTile));
    mean_b[l] = (((red[0][0][l] + red[0][1][l]) + red[0][2][l]) + red[0][3][l]) / n_b;
  }
  __syncthreads();
  const double mu = mean_b[l];
  double q = 0.0;
  if (c < C)
    for (int64_t r = r0 + grp; r < r1; r += 4) {
      const double n_t = bn_tile_n(r, count);
      const double d = (double)part[(r * 2) * C + c] / n_t - mu;
      q += (double)part[(r * 2 + 1) * C + c] + n_t * d * d;
    }
  red[1][grp][l] = q;
  __syncthreads();
  if (grp == 0 && c < C) {
    out[((int64_t)blockIdx.x * 2) * C + c] = ((red[0][0][l] + red[0][1][l]) + red[0][2][l]) + red[0][3][l];
    out[((int64_t)blockIdx.x * 2 + 1) * C + c] = ((red[1][0][l] + red[1][1][l]) + red[1][2][l]) + red[1][3][l];
  }
}

__global__ __launch_bounds__(256) void bn_stats_l2(const double* __restrict__ l1, int nblk, int C, int64_t count,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float eps, float momentum, float* mean, float* rstd, float* scale,
                                                   float* shift, float* rmean, float* rvar) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += l1[((int64_t)b * 2) * C + c];
  const double mu = s / (double)count;
  double m2 = 0.0;
  for (int b = 0; b < nblk; ++b) {   // block b holds tiles [256 b, 256 b + 256): rows [32768 b, ...)
    const int64_t rem = count - (int64_t)b * 256 * kBnTile;
    const double n_b = (double)(rem < 256 * kBnTile ? rem : 256 * kBnTile);
    const double d = l1[((int64_t)b * 2) * C + c] / n_b - mu;
    m2 += l1[((int64_t)b * 2 + 1) * C + c] + n_b * d * d;
  }
  double var = m2 / (double)count;
  if (var < 0.0) var = 0.0;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)mu;
  rstd[c] = rs;
  const float sc = gamma[c] * rs;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mu * sc;
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mu;
  if (rvar) {
    const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
  }
}

__global__ __launch_bounds__(256) void bn_apply_kernel(int64_t n4, int C, const float4* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float4* __restrict__ res, int relu,
                                                       float4* __restrict__ out) {
  // the grid stride (gridDim * 1024 floats) is a multiple of C (the host checks it), so a thread's
  // channel offset is loop-invariant: no 64-bit modulo per element
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = (int)((i0 * 4) % C);
  const float4 a = *(const float4*)(scale + c), b = *(const float4*)(shift + c);
  for (int64_t i = i0; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = y[i];
    v.x = fmaf(v.x, a.x, b.x); v.y = fmaf(v.y, a.y, b.y); v.z = fmaf(v.z, a.z, b.z); v.w = fmaf(v.w, a.w, b.w);
    if (res) {
      const float4 r = res[i];
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    if (relu) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    out[i] = v;
  }
}

// backward, pass 1: per block over a contiguous row range, per channel sum g and sum g xhat
// (g = dout masked by out > 0 under ReLU); partial rows [blocks][2][C] in f64.  The sums are kept in
// f64 from the first add: mean(g) and mean(g xhat) are subtracted from EVERY element's gradient, so
// their rounding is a coherent error that the next conv's weight-gradient sum over ~10^6 voxels
// accumulates instead of averaging out (f32 running sums here put 6e-3 of the norm on layer1's dW
// at 16 clips, against 1e-3 at 2 clips: r05)
__global__ __launch_bounds__(256) void bn_bwd_reduce(int64_t M, int C, const float* __restrict__ dout,
                                                     const float* __restrict__ out, int relu,
                                                     const float* __restrict__ y, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, int64_t rows_per_blk,
                                                     double* __restrict__ part) {
  __shared__ double red[2][4][256];
  const int groups = C / 4;                  // float4 channel groups per row
  const int rpi = 256 / groups;              // rows per iteration (C <= 1024)
  const int t = threadIdx.x, cg = t % groups, ro = t / groups;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  int64_t r1 = r0 + rows_per_blk;
  if (r1 > M) r1 = M;
  double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
  const float4 mu = *(const float4*)(mean + cg * 4), rs = *(const float4*)(rstd + cg * 4);
  // two rows per iteration, every load of both issued before the first f64 add (the adds stay in
  // row order r, r + rpi, ...)
  auto load = [&](int64_t r, float4& gv, float4& yv) {
    const int64_t i = r * C + cg * 4;
    gv = *(const float4*)(dout + i);
    if (relu) {
      const float4 o = *(const float4*)(out + i);
      gv.x = o.x > 0.f ? gv.x : 0.f; gv.y = o.y > 0.f ? gv.y : 0.f;
      gv.z = o.z > 0.f ? gv.z : 0.f; gv.w = o.w > 0.f ? gv.w : 0.f;
    }
    yv = *(const float4*)(y + i);
  };
  auto acc = [&](const float4& gv, const float4& yv) {
    s[0] += gv.x; s[1] += gv.y; s[2] += gv.z; s[3] += gv.w;
    q[0] += (double)gv.x * ((yv.x - mu.x) * rs.x);
    q[1] += (double)gv.y * ((yv.y - mu.y) * rs.y);
    q[2] += (double)gv.z * ((yv.z - mu.z) * rs.z);
    q[3] += (double)gv.w * ((yv.w - mu.w) * rs.w);
  };
  if (ro < rpi) {
    int64_t r = r0 + ro;
    for (; r + rpi < r1; r += 2 * rpi) {
      float4 g0, y0, g1, y1;
      load(r, g0, y0);
      load(r + rpi, g1, y1);
      acc(g0, y0);
      acc(g1, y1);
    }
    if (r < r1) {
      float4 g0, y0;
      load(r, g0, y0);
      acc(g0, y0);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[0][k][t] = s[k];
    red[1][k][t] = q[k];
  }
  __syncthreads();
  if (t < groups) {       // fixed order over the row offsets
    double a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = red[0][k][t];
      b[k] = red[1][k][t];
    }
    for (int o = 1; o < rpi; ++o)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] += red[0][k][o * groups + t];
        b[k] += red[1][k][o * groups + t];
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      part[((int64_t)blockIdx.x * 2) * C + t * 4 + k] = a[k];
      part[((int64_t)blockIdx.x * 2 + 1) * C + t * 4 + k] = b[k];
    }
  }
}

// pass 2: per channel the totals (f64, block order), dgamma / dbeta (+=), and the apply coefficients
// coef[0][c] = gamma rstd, coef[1][c] = gamma rstd mean(g), coef[2][c] = gamma rstd mean(g xhat)
// 64 channels per workgroup, the partial rows split over 16 thread groups (rows b = grp mod 16, in
// order) and the 16 group sums added in a fixed order: one thread per channel walking all the rows was
// a 116-us latency chain per call (r05 rocprof)
__global__ __launch_bounds__(1024) void bn_bwd_finalize(const double* __restrict__ part, int nblk, int C, int64_t M,
                                                        const float* __restrict__ gamma, const float* __restrict__ rstd,
                                                        float* dgamma, float* dbeta, float* __restrict__ coef,
                                                        int batch_stats) {
  constexpr int NG = 16;  // thread groups over the partial rows (rows b = grp mod NG, in order)
  __shared__ double red[2][NG][64];
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6, c = blockIdx.x * 64 + l;
  double s0 = 0.0, q0 = 0.0;
  if (c < C) {
    int b = grp;
    for (; b + 7 * NG < nblk; b += 8 * NG) {  // 8 rows' loads in flight, added in row order
      double vs[8], vq[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        vs[u] = part[((int64_t)(b + u * NG) * 2) * C + c];
        vq[u] = part[((int64_t)(b + u * NG) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s0 += vs[u];
        q0 += vq[u];
      }
    }
    for (; b < nblk; b += NG) {
      s0 += part[((int64_t)b * 2) * C + c];
      q0 += part[((int64_t)b * 2 + 1) * C + c];
    }
  }
  red[0][grp][l] = s0;
  red[1][grp][l] = q0;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double s = red[0][0][l], q = red[1][0][l];
#pragma unroll
  for (int k = 1; k < NG; ++k) {
    s += red[0][k][l];
    q += red[1][k][l];
  }
  if (dgamma) dgamma[c] += (float)q;
  if (dbeta) dbeta[c] += (float)s;
  const double a = (double)gamma[c] * (double)rstd[c];
  coef[c] = (float)a;
  // batch statistics (training mode): the mean and xhat terms of d(batch mean, batch var); running
  // statistics (eval mode) are constants, so dy = gamma rstd g
  coef[C + c] = batch_stats ? (float)(a * (s / (double)M)) : 0.f;
  coef[2 * C + c] = batch_stats ? (float)(a * (q / (double)M)) : 0.f;
}

// pass 3: dy = a g - b - c xhat;  dres = g
__global__ __launch_bounds__(256) void bn_bwd_apply(int64_t n4, int C, const float4* __restrict__ dout,
                                                    const float4* __restrict__ out, int relu,
                                                    const float4* __restrict__ y, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, const float* __restrict__ coef,
                                                    float4* __restrict__ dy, float4* __restrict__ dres) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // loop-invariant channel (as bn_apply_kernel)
  const int c = (int)((i0 * 4) % C);
  const float4 mu = *(const float4*)(mean + c), rs = *(const float4*)(rstd + c);
  const float4 a = *(const float4*)(coef + c), b = *(const float4*)(coef + C + c),
               cc = *(const float4*)(coef + 2 * C + c);
  for (int64_t i = i0; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 gv = dout[i];
    if (relu) {
      const float4 o = out[i];
      gv.x = o.x > 0.f ? gv.x : 0.f; gv.y = o.y > 0.f ? gv.y : 0.f;
      gv.z = o.z > 0.f ? gv.z : 0.f; gv.w = o.w > 0.f ? gv.w : 0.f;
    }
    if (dres) dres[i] = gv;
    const float4 yv = y[i];
    float4 o;
    o.x = fmaf(a.x, gv.x, -b.x) - cc.x * ((yv.x - mu.x) * rs.x);
    o.y = fmaf(a.y, gv.y, -b.y) - cc.y * ((yv.y - mu.y) * rs.y);
    o.z = fmaf(a.z, gv.z, -b.z) - cc.z * ((yv.z - mu.z) * rs.z);
    o.w = fmaf(a.w, gv.w, -b.w) - cc.w * ((yv.w - mu.w) * rs.w);
    dy[i] = o;
  }
}

// ------------------------------------------------------------------------------------------------
// layout and pooling helpers
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void to_channels_last_kernel(int64_t vox, int64_t HW, int C, int Cp,
                                                               const float* __restrict__ x,
                                                               float* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;  // voxel index over (B, T, H, W)
  if (v >= vox) return;
  const int64_t bt = v / HW, hw = v % HW;
  float o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = c < C ? x[(bt * C + c) * HW + hw] : 0.f;
  float* dst = out + v * Cp;
  *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
  if (Cp == 8) *(float4*)(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

__global__ __launch_bounds__(256) void avgpool_kernel(int64_t S, int C, const float* __restrict__ x,
                                                      float* __restrict__ pooled) {
  const int n = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float* p = x + (int64_t)n * S * C + c;
  float s = 0.f;
  for (int64_t i = 0; i < S; ++i) s += p[i * C];
  pooled[(int64_t)n * C + c] = s / (float)S;
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int64_t total, int64_t S, int C,
                                                          const float* __restrict__ dpool, float* __restrict__ dx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const int64_t n = i / ((int64_t)S * C);
  dx[i] = dpool[n * C + c] / (float)S;
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int ilog2(int64_t v) {
  int s = 0;
  while ((1ll << s) < v) ++s;
  return (1ll << s) == v ? s : -1;
}

static bool desc_ok(const vs_conv3d_desc* d) {
  if (!d || d->N <= 0 || d->Ci <= 0 || d->Co <= 0) return false;
  if (d->kd < 1 || d->kh < 1 || d->kw < 1 || d->sd < 1 || d->sh < 1 || d->sw < 1) return false;
  if (d->pd < 0 || d->ph < 0 || d->pw < 0) return false;
  return d->Do == (d->Di + 2 * d->pd - d->kd) / d->sd + 1 && d->Ho == (d->Hi + 2 * d->ph - d->kh) / d->sh + 1 &&
         d->Wo == (d->Wi + 2 * d->pw - d->kw) / d->sw + 1 && d->Do > 0 && d->Ho > 0 && d->Wo > 0;
}

static double conv_flops(const vs_conv3d_desc* d) {
  return 2.0 * (double)(d->N * d->Do * d->Ho * d->Wo) * (double)d->Co * (double)(d->kd * d->kh * d->kw * d->Ci);
}

static int launch_igemm(const Igemm& g, hipStream_t s) {
  VS_REQUIRE((int64_t)g.N * g.Di * g.Hi * g.Wi * g.C < (1ll << 29) && (int64_t)g.Ng * g.K < (1ll << 29) &&
                 g.M < (1ll << 24) && g.K < (1 << 24),
             "conv3d: gathered volume too large (operands must stay below 2^31 bytes)");
  const int64_t tiles_m = (g.M + 127) / 128;
  const int64_t nwg = tiles_m * (g.Ng / 64);
  VS_REQUIRE(nwg < (1ll << 31), "conv3d: grid too large");
  count_path(VS_PATH_CONV_IGEMM);
  hipLaunchKernelGGL(conv_igemm_kernel, dim3((unsigned)nwg), dim3(256), 0, s, g);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

}  // namespace vs

using namespace vs;

extern "C" size_t vs_conv3d_stats_rows(const vs_conv3d_desc* d) {
  if (!desc_ok(d)) return 0;
  return (size_t)((d->N * d->Do * d->Ho * d->Wo + 127) / 128);
}

extern "C" int vs_conv3d_fwd(const vs_conv3d_desc* d, const float* x, const float* w, float* y, float* stats,
                             void* stream) {
  VS_REQUIRE(desc_ok(d), "vs_conv3d_fwd: inconsistent geometry (Do = (Di + 2 pd - kd) / sd + 1, ...)");
  VS_REQUIRE(x && w && y, "vs_conv3d_fwd: null pointer");
  const int cs = ilog2(d->Ci);
  VS_REQUIRE(cs >= 2 && d->Co % 64 == 0, "vs_conv3d_fwd: Ci must be a power of two >= 4, Co a multiple of 64");
  VS_REQUIRE(aligned16(x) && aligned16(w) && aligned16(y), "vs_conv3d_fwd: pointers must be 16-byte aligned");
  const int64_t M = d->N * d->Do * d->Ho * d->Wo;
  VS_REQUIRE(M < (1ll << 24) && d->N * d->Di * d->Hi * d->Wi < (1ll << 31), "vs_conv3d_fwd: volume too large");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_CONV_FWD, s, conv_flops(d));
  Igemm g = {};
  g.x = x; g.N = (int)d->N; g.Di = (int)d->Di; g.Hi = (int)d->Hi; g.Wi = (int)d->Wi; g.C = (int)d->Ci; g.cshift = cs;
  g.Gd = (int)d->Do; g.Gh = (int)d->Ho; g.Gw = (int)d->Wo;
  g.sd = d->sd; g.sh = d->sh; g.sw = d->sw;
  g.cd = d->kd; g.ch = d->kh; g.cw = d->kw;
  g.od0 = -d->pd; g.oh0 = -d->ph; g.ow0 = -d->pw; g.ods = 1; g.ohs = 1; g.ows = 1;
  g.w = w; g.Ng = (int)d->Co; g.K = d->kd * d->kh * d->kw * (int)d->Ci;
  g.y = y; g.Od = (int)d->Do; g.Oh = (int)d->Ho; g.Ow = (int)d->Wo;
  g.ysd = g.ysh = g.ysw = 1;
  g.accumulate = 0;
  g.stats = stats;
  g.M = M;
  return launch_igemm(g, s);
}

// the parity classes of a dX launch: per dim the first tap, tap step, class count and the offsets
struct DxDim {
  int ncls;            // 1 (stride 1) or 2 (stride 2)
  int cnt[2], t0[2], ts[2], o0[2], os[2], start[2], step;
};
static DxDim dx_dim(int k, int s, int p) {
  DxDim r = {};
  if (s == 1) {    // dX[i] = sum_t dy[i + p - t] w[t]
    r.ncls = 1;
    r.cnt[0] = k; r.t0[0] = 0; r.ts[0] = 1; r.o0[0] = p; r.os[0] = -1; r.start[0] = 0;
    r.step = 1;
    return r;
  }
  // stride 2: i = 2 j + par; taps t with (par + p - t) even; dy index j + (par + p - t) / 2
  r.ncls = 2;
  r.step = 2;
  for (int par = 0; par < 2; ++par) {
    const int t0 = (par + p) & 1;
    r.t0[par] = t0;
    r.ts[par] = 2;
    r.cnt[par] = t0 < k ? (k - 1 - t0) / 2 + 1 : 0;
    r.o0[par] = (par + p - t0) / 2;
    r.os[par] = -1;
    r.start[par] = par;
  }
  return r;
}

extern "C" size_t vs_conv3d_dx_workspace_bytes(const vs_conv3d_desc* d) {
  if (!desc_ok(d)) return 0;
  return (size_t)d->Ci * d->kd * d->kh * d->kw * d->Co * 4 + 256;
}

extern "C" int vs_conv3d_dx(const vs_conv3d_desc* d, const float* dy, const float* w, float* dx, int32_t accumulate,
                            void* workspace, int64_t workspace_bytes, void* stream) {
  VS_REQUIRE(desc_ok(d), "vs_conv3d_dx: inconsistent geometry");
  VS_REQUIRE(dy && w && dx && workspace, "vs_conv3d_dx: null pointer");
  const int cs = ilog2(d->Co);
  VS_REQUIRE(cs >= 2 && d->Ci % 64 == 0, "vs_conv3d_dx: Co must be a power of two >= 4, Ci a multiple of 64");
  VS_REQUIRE(d->sd <= 2 && d->sh <= 2 && d->sw <= 2, "vs_conv3d_dx: stride 1 or 2");
  VS_REQUIRE((size_t)workspace_bytes >= vs_conv3d_dx_workspace_bytes(d), "vs_conv3d_dx: workspace too small");
  VS_REQUIRE(aligned16(dy) && aligned16(w) && aligned16(dx) && aligned16(workspace),
             "vs_conv3d_dx: pointers must be 16-byte aligned");
  VS_REQUIRE(d->N * d->Di * d->Hi * d->Wi < (1ll << 24), "vs_conv3d_dx: volume too large");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_CONV_DX, s, conv_flops(d));
  const DxDim zd = dx_dim(d->kd, d->sd, d->pd), yd = dx_dim(d->kh, d->sh, d->ph), xd = dx_dim(d->kw, d->sw, d->pw);
  float* wd = (float*)workspace;
  for (int a = 0; a < zd.ncls; ++a)
    for (int b = 0; b < yd.ncls; ++b)
      for (int c = 0; c < xd.ncls; ++c) {
        // the positions of this class: i = start + step * j, j < G
        const int Gd = (int)((d->Di - zd.start[a] + zd.step - 1) / zd.step);
        const int Gh = (int)((d->Hi - yd.start[b] + yd.step - 1) / yd.step);
        const int Gw = (int)((d->Wi - xd.start[c] + xd.step - 1) / xd.step);
        if (Gd <= 0 || Gh <= 0 || Gw <= 0) continue;
        const int T = zd.cnt[a] * yd.cnt[b] * xd.cnt[c];
        if (T == 0) {   // no tap reaches these positions: their gradient is zero
          if (!accumulate) {
            Igemm g = {};   // a K = 0 GEMM writes zeros through the same epilogue
            g.x = dy; g.N = (int)d->N; g.Di = (int)d->Do; g.Hi = (int)d->Ho; g.Wi = (int)d->Wo; g.C = (int)d->Co;
            g.cshift = cs; g.Gd = Gd; g.Gh = Gh; g.Gw = Gw; g.sd = g.sh = g.sw = 1; g.cd = g.ch = g.cw = 1;
            g.w = wd; g.Ng = (int)d->Ci; g.K = 0;
            g.y = dx; g.Od = (int)d->Di; g.Oh = (int)d->Hi; g.Ow = (int)d->Wi;
            g.ysd = zd.step; g.ysh = yd.step; g.ysw = xd.step; g.yod = zd.start[a]; g.yoh = yd.start[b];
            g.yow = xd.start[c];
            g.M = d->N * (int64_t)Gd * Gh * Gw;
            VS_CALL(launch_igemm(g, s));
          }
          continue;
        }
        const int64_t nw = d->Ci * (int64_t)T * d->Co;
        hipLaunchKernelGGL(conv_dx_weights, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)d->Co,
                           (int)d->Ci, d->kd, d->kh, d->kw, zd.cnt[a], yd.cnt[b], xd.cnt[c], zd.t0[a], yd.t0[b],
                           xd.t0[c], zd.ts[a], yd.ts[b], xd.ts[c], wd);
        VS_LAUNCH_CHECK();
        Igemm g = {};
        g.x = dy; g.N = (int)d->N; g.Di = (int)d->Do; g.Hi = (int)d->Ho; g.Wi = (int)d->Wo; g.C = (int)d->Co;
        g.cshift = cs;
        g.Gd = Gd; g.Gh = Gh; g.Gw = Gw;
        g.sd = g.sh = g.sw = 1;
        g.cd = zd.cnt[a]; g.ch = yd.cnt[b]; g.cw = xd.cnt[c];
        g.od0 = zd.o0[a]; g.oh0 = yd.o0[b]; g.ow0 = xd.o0[c];
        g.ods = zd.os[a]; g.ohs = yd.os[b]; g.ows = xd.os[c];
        g.w = wd; g.Ng = (int)d->Ci; g.K = T * (int)d->Co;
        g.y = dx; g.Od = (int)d->Di; g.Oh = (int)d->Hi; g.Ow = (int)d->Wi;
        g.ysd = zd.step; g.ysh = yd.step; g.ysw = xd.step;
        g.yod = zd.start[a]; g.yoh = yd.start[b]; g.yow = xd.start[c];
        g.accumulate = accumulate;
        g.M = d->N * (int64_t)Gd * Gh * Gw;
        VS_CALL(launch_igemm(g, s));
      }
  return VS_OK;
}

namespace vs {
struct DwPlanC {
  int tiles_o, tiles_k, Kp, splits, sps, bkk;
};
static DwPlanC plan_conv_dw(const vs_conv3d_desc* d) {
  DwPlanC p;
  const int K = d->kd * d->kh * d->kw * (int)d->Ci;
  // 128-wide k tiles halve the dy re-reads but measured slower (conv dW 40.9 vs 39.4 ms/step at C4)
  p.bkk = K >= 128 && knob(VS_KNOB_CONV_DW128) ? 128 : 64;
  p.tiles_o = (int)(d->Co / 64);
  p.tiles_k = (K + p.bkk - 1) / p.bkk;
  p.Kp = p.tiles_k * p.bkk;
  const int64_t M = d->N * d->Do * d->Ho * d->Wo;
  const int64_t steps = (M + 31) / 32;
  const int tiles = p.tiles_o * p.tiles_k;
  int64_t S = (1024 + tiles - 1) / tiles;        // ~4 workgroups per CU
  const int64_t smax = steps / 16 > 0 ? steps / 16 : 1;   // >= 16 row steps per split
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  p.sps = (int)((steps + S - 1) / S);
  p.splits = (int)((steps + p.sps - 1) / p.sps);
  return p;
}
}  // namespace vs

extern "C" size_t vs_conv3d_dw_workspace_bytes(const vs_conv3d_desc* d) {
  if (!desc_ok(d) || d->Co % 64) return 0;
  const DwPlanC p = plan_conv_dw(d);
  return (size_t)p.splits * d->Co * p.Kp * 4 + 256;
}

extern "C" int vs_conv3d_dw(const vs_conv3d_desc* d, const float* x, const float* dy, float* dw, int32_t accumulate,
                            void* workspace, int64_t workspace_bytes, void* stream) {
  VS_REQUIRE(desc_ok(d), "vs_conv3d_dw: inconsistent geometry");
  VS_REQUIRE(x && dy && dw && workspace, "vs_conv3d_dw: null pointer");
  const int cs = ilog2(d->Ci);
  VS_REQUIRE(cs >= 2 && d->Co % 64 == 0, "vs_conv3d_dw: Ci must be a power of two >= 4, Co a multiple of 64");
  VS_REQUIRE((size_t)workspace_bytes >= vs_conv3d_dw_workspace_bytes(d), "vs_conv3d_dw: workspace too small");
  VS_REQUIRE(aligned16(x) && aligned16(dy) && aligned16(workspace), "vs_conv3d_dw: pointers must be 16-byte aligned");
  const int64_t M = d->N * d->Do * d->Ho * d->Wo;
  VS_REQUIRE(M < (1ll << 24) && M * d->Co < (1ll << 29) && d->N * d->Di * d->Hi * d->Wi < (1ll << 24) &&
                 d->N * d->Di * d->Hi * d->Wi * d->Ci < (1ll << 29),
             "vs_conv3d_dw: volume too large (operands must stay below 2^31 bytes)");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_CONV_DW, s, conv_flops(d));
  const DwPlanC p = plan_conv_dw(d);
  ConvDw g = {};
  g.x = x; g.N = (int)d->N; g.Di = (int)d->Di; g.Hi = (int)d->Hi; g.Wi = (int)d->Wi; g.C = (int)d->Ci; g.cshift = cs;
  g.Do = (int)d->Do; g.Ho = (int)d->Ho; g.Wo = (int)d->Wo;
  g.sd = d->sd; g.sh = d->sh; g.sw = d->sw; g.pd = d->pd; g.ph = d->ph; g.pw = d->pw;
  g.kd = d->kd; g.kh = d->kh; g.kw = d->kw;
  g.dy = dy; g.Co = (int)d->Co; g.K = d->kd * d->kh * d->kw * (int)d->Ci;
  g.M = M; g.splits = p.splits; g.steps_per_split = p.sps; g.part = (float*)workspace; g.Kp = p.Kp;
  count_path(VS_PATH_CONV_DW);
  const int64_t nwg = (int64_t)p.splits * p.tiles_o * p.tiles_k;
  if (p.bkk == 128) hipLaunchKernelGGL((conv_dw_kernel<128, false>), dim3((unsigned)nwg), dim3(256), 0, s, g);
  else if (knob(VS_KNOB_CONV_MFMA) == 1)   // 32x32x2: measured slower (conv dW 37.3 vs 32.5 ms/step, r06)
    hipLaunchKernelGGL((conv_dw_kernel<64, true>), dim3((unsigned)nwg), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((conv_dw_kernel<64, false>), dim3((unsigned)nwg), dim3(256), 0, s, g);
  VS_LAUNCH_CHECK();
  const int64_t n = d->Co * (int64_t)g.K;
  hipLaunchKernelGGL(conv_dw_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float*)workspace,
                     p.splits, g.Co, g.K, p.Kp, dw, accumulate);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" size_t vs_bn3d_stats_workspace_bytes(int64_t rows, int64_t C) {
  return (size_t)((rows + 255) / 256) * 2 * C * sizeof(double) + 256;
}

extern "C" int vs_bn3d_stats(int64_t rows, int64_t C, const float* part, int64_t count, const float* gamma,
                             const float* beta, float eps, float momentum, float* mean, float* rstd, float* scale,
                             float* shift, float* running_mean, float* running_var, void* workspace, void* stream) {
  VS_REQUIRE(part && gamma && beta && mean && rstd && scale && shift && workspace, "vs_bn3d_stats: null pointer");
  VS_REQUIRE(rows > 0 && C > 0 && count > 0 && C % 4 == 0 && (count + kBnTile - 1) / kBnTile == rows,
             "vs_bn3d_stats: bad extents (rows = ceil(count / 128) tiles)");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)rows * 2.0 * (double)C * 4.0);
  const int64_t nblk = (rows + 255) / 256;
  double* l1 = (double*)workspace;   // level-1 f64 partial sums [nblk][2][C]
  hipLaunchKernelGGL(bn_stats_l1, dim3((unsigned)nblk, (unsigned)((C + 63) / 64)), dim3(256), 0, s, part, rows,
                     (int)C, count, l1);
  VS_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_stats_l2, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, (const double*)l1, (int)nblk,
                     (int)C, count, gamma, beta, eps, momentum, mean, rstd, scale, shift, running_mean, running_var);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

namespace vs {
// ~8K elements per workgroup (<= 2,048 partial rows): the old rows-only rule (1,024 rows per block,
// <= 512 blocks) gave the deep layers 4-196 workgroups with 128-392 serial row steps per thread
// (bn_bwd_reduce averaged 219 us per call at C4, 3.4x its bytes at the apply pass's rate)
static int64_t bn_bwd_blocks(int64_t M, int64_t C) {
  const int64_t b = (M * C + 8191) / 8192;
  return b < 2048 ? (b > 0 ? b : 1) : 2048;
}
// grid of the elementwise BN passes: <= 4096 workgroups, and a stride (blocks x 1024 floats) that is
// a multiple of C so each thread's channel offset is fixed (C <= 1024 divides 1024, or 1 round)
static int64_t bn_ew_blocks(int64_t n4, int64_t C) {
  const int64_t need = (n4 + 255) / 256;
  if (need <= 4096) return need;
  int64_t b = 4096;
  while (b > 1 && (b * 1024) % C != 0) --b;
  return b;
}
}  // namespace vs

extern "C" int vs_bn3d_apply(int64_t M, int64_t C, const float* y, const float* scale, const float* shift,
                             const float* residual, int32_t relu, float* out, void* stream) {
  VS_REQUIRE(y && scale && shift && out, "vs_bn3d_apply: null pointer");
  VS_REQUIRE(C % 4 == 0 && aligned16(y) && aligned16(out) && (!residual || aligned16(residual)) && aligned16(scale) &&
                 aligned16(shift),
             "vs_bn3d_apply: C % 4 == 0 and 16-byte aligned pointers");
  if (M <= 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)M * C * (residual ? 12.0 : 8.0));
  const int64_t n4 = M * C / 4;
  const int64_t blocks = bn_ew_blocks(n4, C);
  hipLaunchKernelGGL(bn_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n4, (int)C, (const float4*)y, scale,
                     shift, (const float4*)residual, relu, (float4*)out);
  VS_LAUNCH_CHECK();
  return VS_OK;
}


extern "C" size_t vs_bn3d_bwd_workspace_bytes(int64_t M, int64_t C) {
  return (size_t)bn_bwd_blocks(M, C) * 2 * C * 8 + (size_t)3 * C * 4 + 256;
}

static int bn3d_bwd(int64_t M, int64_t C, const float* dout, const float* out, int32_t relu, const float* y,
                    const float* mean, const float* rstd, const float* gamma, float* dy, float* dres, float* dgamma,
                    float* dbeta, void* workspace, void* stream, int batch_stats) {
  VS_REQUIRE(dout && y && mean && rstd && gamma && dy && workspace && (!relu || out), "vs_bn3d_bwd: null pointer");
  VS_REQUIRE(C % 4 == 0 && C <= 1024 && aligned16(dout) && aligned16(y) && aligned16(dy) &&
                 (!out || aligned16(out)) && (!dres || aligned16(dres)) && aligned16(workspace),
             "vs_bn3d_bwd: C % 4 == 0, C <= 1024, 16-byte aligned pointers");
  if (M <= 0) return VS_OK;
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)M * C * (4.0 * (relu ? 3 : 2) + 4.0 + (dres ? 4.0 : 0.0)));
  const int64_t nblk = bn_bwd_blocks(M, C);
  const int64_t rpb = (M + nblk - 1) / nblk;
  double* part = (double*)workspace;
  float* coef = (float*)(part + nblk * 2 * C);
  hipLaunchKernelGGL(bn_bwd_reduce, dim3((unsigned)nblk), dim3(256), 0, s, M, (int)C, dout, out, relu, y, mean, rstd,
                     rpb, part);
  VS_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3((unsigned)((C + 63) / 64)), dim3(1024), 0, s, (const double*)part,
                     (int)nblk, (int)C, M, gamma, rstd, dgamma, dbeta, coef, batch_stats);
  VS_LAUNCH_CHECK();
  const int64_t n4 = M * C / 4;
  const int64_t blocks = bn_ew_blocks(n4, C);
  hipLaunchKernelGGL(bn_bwd_apply, dim3((unsigned)blocks), dim3(256), 0, s, n4, (int)C, (const float4*)dout,
                     (const float4*)out, relu, (const float4*)y, mean, rstd, (const float*)coef, (float4*)dy,
                     (float4*)dres);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_bn3d_bwd(int64_t M, int64_t C, const float* dout, const float* out, int32_t relu, const float* y,
                           const float* mean, const float* rstd, const float* gamma, float* dy, float* dres,
                           float* dgamma, float* dbeta, void* workspace, void* stream) {
  return bn3d_bwd(M, C, dout, out, relu, y, mean, rstd, gamma, dy, dres, dgamma, dbeta, workspace, stream, 1);
}

extern "C" int vs_bn3d_bwd_eval(int64_t M, int64_t C, const float* dout, const float* out, int32_t relu,
                                const float* y, const float* mean, const float* rstd, const float* gamma, float* dy,
                                float* dres, float* dgamma, float* dbeta, void* workspace, void* stream) {
  return bn3d_bwd(M, C, dout, out, relu, y, mean, rstd, gamma, dy, dres, dgamma, dbeta, workspace, stream, 0);
}

extern "C" int vs_to_channels_last(int64_t B, int64_t T, int64_t C, int64_t H, int64_t W, int64_t Cp, const float* x,
                                   float* out, void* stream) {
  VS_REQUIRE(x && out && aligned16(out), "vs_to_channels_last: null / misaligned pointer");
  VS_REQUIRE(C >= 1 && C <= Cp && (Cp == 4 || Cp == 8), "vs_to_channels_last: C <= Cp, Cp = 4 or 8");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)B * T * H * W * (C + Cp) * 4.0);
  const int64_t vox = B * T * H * W;
  hipLaunchKernelGGL(to_channels_last_kernel, dim3((unsigned)((vox + 255) / 256)), dim3(256), 0, s, vox, H * W,
                     (int)C, (int)Cp, x, out);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_avgpool3d(int64_t N, int64_t S, int64_t C, const float* x, float* pooled, void* stream) {
  VS_REQUIRE(x && pooled && N > 0 && S > 0 && C > 0, "vs_avgpool3d: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)N * S * C * 4.0);
  hipLaunchKernelGGL(avgpool_kernel, dim3((unsigned)((C + 255) / 256), (unsigned)N), dim3(256), 0, s, S, (int)C, x,
                     pooled);
  VS_LAUNCH_CHECK();
  return VS_OK;
}

extern "C" int vs_avgpool3d_bwd(int64_t N, int64_t S, int64_t C, const float* dpool, float* dx, void* stream) {
  VS_REQUIRE(dpool && dx && N > 0 && S > 0 && C > 0, "vs_avgpool3d_bwd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  ScopedTimer timer(VS_TIMER_BN, s, (double)N * S * C * 4.0);
  const int64_t total = N * S * C;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, total, S, (int)C,
                     dpool, dx);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
