// preprocess.hip — on-device K0: the VideoMAE plugin's CPU preprocessing (videomae.py:18-25),
// frame gather + gray->RGB + HF VideoMAEImageProcessor resize/crop/rescale/normalise.
//
// Parity target: the reference runs the HF image processor on each selected frame.  Its frames
// are integer-valued floats, so HF casts them to uint8 and resizes with PIL (Image.resize,
// BILINEAR, reducing_gap None).  PIL's uint8 resample is reproduced bit for bit:
//   * coefficients (Pillow libImaging/Resample.c precompute_coeffs): per output index xx,
//     scale = in/out, filterscale = max(scale, 1), support = filterscale, center = (xx+0.5)*scale,
//     xmin = int(center - support + 0.5) >= 0, xmax = min(int(center + support + 0.5), in),
//     w(x) = tri((x + xmin - center + 0.5) / filterscale), normalised by their sum (double), then
//     fixed point kk = int(w * 2^22 +- 0.5) (normalize_coeffs_8bpc, PRECISION_BITS = 22);
//   * two passes, horizontal first into a uint8 image, then vertical:
//     out = clip8((1 << 21) + sum in * kk) with clip8(v) = v <= 0 ? 0 : v >= 255 << 22 ? 255 : v >> 22.
// Every double operation is written with an explicit round-to-nearest intrinsic so the device
// computes exactly the host C expression (no FMA contraction).  Then, as HF does: rescale in
// double, (double)u8 * (1/255) rounded to f32, and normalise in f32: (x - mean) / std.
//
// One thread per output pixel (frame, y, x): it recomputes its row's 3 horizontal taps for the
// 2-3 source rows the vertical pass needs (at most 9 uint8 reads, L1/L2-resident: a 128x128 frame
// is 16 KB) and writes the 3 channels.  Bound: HBM on the f32 output (12 B per output pixel).
#include <algorithm>

#include "common.h"

namespace vs {

constexpr int kPilBits = 22;  // Pillow PRECISION_BITS for 8-bit images (32 - 8 - 2)
constexpr int kMaxTaps = 16;  // ksize for in <= 7 * out

// Pillow precompute_coeffs for one output index (bilinear filter, support 1).
__device__ __forceinline__ int pil_coeffs(int in_size, int out_size, int xx, int* k) {
  const double scale = __ddiv_rn((double)in_size, (double)out_size);
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = filterscale;  // bilinear support 1.0 * filterscale
  const double center = __dmul_rn((double)xx + 0.5, scale);  // in0 = 0; xx + 0.5 is exact
  const double ss = __ddiv_rn(1.0, filterscale);
  int xmin = (int)__dadd_rn(__dsub_rn(center, support), 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)__dadd_rn(__dadd_rn(center, support), 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double w[kMaxTaps];
  double ww = 0.0;
  for (int x = 0; x < xmax && x < kMaxTaps; ++x) {
    double t = __dmul_rn(__dadd_rn(__dsub_rn((double)(x + xmin), center), 0.5), ss);
    if (t < 0.0) t = -t;
    const double v = t < 1.0 ? 1.0 - t : 0.0;
    w[x] = v;
    ww = __dadd_rn(ww, v);
  }
  for (int x = 0; x < xmax && x < kMaxTaps; ++x) {
    const double v = ww != 0.0 ? __ddiv_rn(w[x], ww) : w[x];
    const double f = __dmul_rn(v, (double)(1 << kPilBits));
    k[x] = v < 0 ? (int)__dadd_rn(-0.5, f) : (int)__dadd_rn(0.5, f);
  }
  k[kMaxTaps - 1] = xmin;  // packed return: taps in k[0 .. xmax), xmin in the last slot
  return xmax;
}

__device__ __forceinline__ int pil_clip8(int64_t v) {
  if (v >= ((int64_t)1 << kPilBits << 8)) return 255;
  if (v <= 0) return 0;
  return (int)(v >> kPilBits);
}

template <typename TI>
__device__ __forceinline__ int load_u8(const TI* p) {
  if constexpr (std::is_same<TI, uint8_t>::value) return *p;
  else return (int)(uint8_t)(int)(*p);  // numpy astype(uint8) of an integer-valued float
}

struct FrameIdx {
  int32_t v[64];
};
struct Norm3 {
  float mean[3], stdv[3];
};

template <typename TI>
__global__ __launch_bounds__(256) void video_preprocess_kernel(const TI* __restrict__ video, int64_t B, int T, int HW,
                                                               FrameIdx fidx, int F, int S, Norm3 nrm,
                                                               float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per_frame = (int64_t)S * S;
  if (t >= B * F * per_frame) return;
  const int x = (int)(t % S), y = (int)((t / S) % S);
  const int64_t bf = t / per_frame;
  const int f = (int)(bf % F);
  const int64_t b = bf / F;
  const TI* src = video + (b * T + fidx.v[f]) * (int64_t)HW * HW;

  int kx[kMaxTaps], ky[kMaxTaps];
  const int nx = pil_coeffs(HW, S, x, kx), xmin = kx[kMaxTaps - 1];
  const int ny = pil_coeffs(HW, S, y, ky), ymin = ky[kMaxTaps - 1];
  int64_t acc = (int64_t)1 << (kPilBits - 1);
  for (int j = 0; j < ny; ++j) {
    const TI* row = src + (int64_t)(ymin + j) * HW + xmin;
    int64_t h = (int64_t)1 << (kPilBits - 1);
    for (int i = 0; i < nx; ++i) h += (int64_t)load_u8(row + i) * kx[i];
    acc += (int64_t)pil_clip8(h) * ky[j];  // the uint8 intermediate image of the horizontal pass
  }
  const int u = pil_clip8(acc);
  const float r = (float)__dmul_rn((double)u, 1.0 / 255.0);  // HF rescale in double, then f32
  float* o = out + bf * 3 * per_frame + (int64_t)y * S + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c * per_frame] = __fdiv_rn(r - nrm.mean[c], nrm.stdv[c]);
}

}  // namespace vs

using namespace vs;

extern "C" int vs_video_preprocess(int32_t in_dtype, int64_t B, int64_t T, int64_t H, int64_t W, const void* video,
                                   const int32_t* frame_idx, int32_t n_frames, int64_t out_size, const float* mean,
                                   const float* std, float* out, void* stream) {
  VS_REQUIRE(in_dtype == VS_F32 || in_dtype == VS_U8, "vs_video_preprocess: in_dtype must be VS_F32 or VS_U8");
  VS_REQUIRE(video && frame_idx && mean && std && out, "vs_video_preprocess: null pointer");
  VS_REQUIRE(B >= 0 && T > 0 && H > 0 && H == W, "vs_video_preprocess: frames must be square (H == W)");
  VS_REQUIRE(n_frames > 0 && n_frames <= 64, "vs_video_preprocess: 1..64 frames");
  VS_REQUIRE(out_size > 0 && H <= 7 * out_size && out_size <= 4096, "vs_video_preprocess: bad out_size");
  FrameIdx fi;
  for (int i = 0; i < n_frames; ++i) {
    VS_REQUIRE(frame_idx[i] >= 0 && frame_idx[i] < T, "vs_video_preprocess: frame index out of range");
    fi.v[i] = frame_idx[i];
  }
  Norm3 nrm;
  for (int c = 0; c < 3; ++c) {
    VS_REQUIRE(std[c] != 0.f, "vs_video_preprocess: std must be non-zero");
    nrm.mean[c] = mean[c];
    nrm.stdv[c] = std[c];
  }
  if (B == 0) return VS_OK;
  const int64_t n = B * n_frames * out_size * out_size;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)cdiv(n, 256));
  if (in_dtype == VS_U8)
    hipLaunchKernelGGL(video_preprocess_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)video, B, (int)T,
                       (int)H, fi, (int)n_frames, (int)out_size, nrm, out);
  else
    hipLaunchKernelGGL(video_preprocess_kernel<float>, grid, dim3(256), 0, s, (const float*)video, B, (int)T, (int)H,
                       fi, (int)n_frames, (int)out_size, nrm, out);
  VS_LAUNCH_CHECK();
  return VS_OK;
}
