// common.h — shared device helpers for libvspike (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vspike.h"

typedef uint16_t bf16_t;  // bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short short4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define VS_LDS __attribute__((address_space(3)))

namespace vs {

// ---- host-side error plumbing ------------------------------------------------------------
void set_error(const char* msg);
#define VS_REQUIRE(cond, msg)       \
  do {                              \
    if (!(cond)) {                  \
      ::vs::set_error(msg);         \
      return VS_EINVAL;             \
    }                               \
  } while (0)
#define VS_LAUNCH_CHECK()                              \
  do {                                                 \
    hipError_t _e = hipGetLastError();                 \
    if (_e != hipSuccess) return (int)_e;              \
  } while (0)
#define VS_CALL(expr)               \
  do {                              \
    int _r = (expr);                \
    if (_r != VS_OK) return _r;     \
  } while (0)

inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t esize(int dtype) { return dtype == VS_BF16 ? 2 : 4; }

// ---- kernel timers ------------------------------------------------------------------------
struct ScopedTimer {
  int timer;
  hipStream_t stream;
  void* ev_end;
  ScopedTimer(int t, hipStream_t s);
  ~ScopedTimer();
};

// ---- device conversions -------------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int dtype = VS_F32;
  __device__ static __forceinline__ float load(const float* p) { return *p; }
  __device__ static __forceinline__ void store(float* p, float v) { *p = v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int dtype = VS_BF16;
  __device__ static __forceinline__ float load(const bf16_t* p) { return bf2f(*p); }
  __device__ static __forceinline__ void store(bf16_t* p, float v) { *p = f2bf(v); }
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware block remap for a 1D grid of nwg workgroups.  The dispatcher deals workgroup
// ids round-robin over the 8 XCDs (id % 8); this returns a logical index such that the workgroups
// of one XCD get CONSECUTIVE logical indices, so blocks that share operands (e.g. the query blocks
// of one (batch, head)) share that XCD's L2 instead of being fetched into eight of them.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

}  // namespace vs
