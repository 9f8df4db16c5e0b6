// common.h — shared device helpers for libvspike (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include "vspike.h"

typedef uint16_t bf16_t;  // bf16 storage
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short short4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4v;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;

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

// A/B and test knobs (VS_KNOB_*): read from the environment once, overridable by vs_knob_set
int knob(int id);
// dispatch counters (VS_PATH_*): one relaxed host-side add per launch of a path
void count_path(int id);

inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t esize(int dtype) { return dtype == VS_BF16 ? 2 : 4; }

// ---- kernel timers ------------------------------------------------------------------------
struct ScopedTimer {
  int timer;
  hipStream_t stream;
  void* ev_end;
  ScopedTimer(int t, hipStream_t s, double algorithmic_bytes = 0.0);
  ~ScopedTimer();
};
// The timer a nested vs_gemm call is charged to, set by the block executor around each product
// (-1: the call's own class).  Thread-local: executors on different threads do not interfere.
extern thread_local int g_timer_tag;
// dgamma[c] += sum_b part[b][c], dbeta[c] += sum_b part[b][cols + c] in a fixed order (norm.hip)
void launch_ln_partsum(const float* part, int nblk, int cols, float* dgamma, float* dbeta, hipStream_t s);
struct TimerTag {
  int prev;
  explicit TimerTag(int t) : prev(g_timer_tag) { g_timer_tag = t; }
  ~TimerTag() { g_timer_tag = prev; }
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

// bf16-path GELU: Phi(x) from Abramowitz & Stegun 7.1.26 (|erf error| <= 1.5e-7, far below bf16's
// 2^-9), evaluated as a tail so Phi(x < 0) keeps relative accuracy; its exp(-x^2/2) factor is also
// the Gaussian density of GELU' (one exp for both).  ~15 VALU vs ~46 for erff (+8 for the exp).
__device__ __forceinline__ float phi_fast(float x, float& g) {  // returns Phi(x); g = exp(-x^2/2)
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  g = __builtin_amdgcn_exp2f(-(x * x) * 0.72134752044448170f);  // exp(-x^2/2) = 2^(-x^2 log2(e)/2)
  const float tail = 0.5f * (t * p) * g;                       // = 0.5 * erfc(|x|/sqrt 2)
  return x >= 0.f ? 1.f - tail : tail;
}
__device__ __forceinline__ float gelu_fast(float x) {
  float g;
  return x * phi_fast(x, g);
}
__device__ __forceinline__ float gelu_fast_grad(float x) {
  float g;
  const float cdf = phi_fast(x, g);
  return fmaf(x * 0.39894228040143268f, g, cdf);
}
// gelu(x) and gelu'(x) from one Phi / exp evaluation (the fc1 forward that stores gelu')
__device__ __forceinline__ float gelu_fast_both(float x, float& grad) {
  float g;
  const float cdf = phi_fast(x, g);
  grad = fmaf(x * 0.39894228040143268f, g, cdf);
  return x * cdf;
}

// The same on a pair of values in packed f32 VALU (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per
// instruction; only the rcp and exp2 stay scalar): bitwise the single-value results (the same fused
// operations in the same order).  For epilogues that run with no MFMA beside them, where packed VALU
// halves the issue count (beside MFMAs it is an anti-lever: MI355X_MICROARCH.md issue-cost rows).
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v phi_fast2(f32x2v x, f32x2v& g) {
  const f32x2v z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2v d = __builtin_elementwise_fma((f32x2v)0.3275911f, z, (f32x2v)1.0f);
  const f32x2v t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2v p = __builtin_elementwise_fma(t, (f32x2v)1.061405429f, (f32x2v)-1.453152027f);
  p = __builtin_elementwise_fma(t, p, (f32x2v)1.421413741f);
  p = __builtin_elementwise_fma(t, p, (f32x2v)-0.284496736f);
  p = __builtin_elementwise_fma(t, p, (f32x2v)0.254829592f);
  const f32x2v q = -(x * x) * 0.72134752044448170f;
  g = f32x2v{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2v tail = 0.5f * (t * p) * g;
  return f32x2v{x.x >= 0.f ? 1.f - tail.x : tail.x, x.y >= 0.f ? 1.f - tail.y : tail.y};
}
__device__ __forceinline__ f32x2v gelu_fast_both2(f32x2v x, f32x2v& grad) {
  f32x2v g;
  const f32x2v cdf = phi_fast2(x, g);
  grad = __builtin_elementwise_fma(x * 0.39894228040143268f, g, cdf);
  return x * cdf;
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

// compile-time integer tag (unrolled loops over LDS stages)
template <int I>
using IC = std::integral_constant<int, I>;

// ---- LDS-DMA (global_load_lds): one wave-instruction writes 64 x size bytes to a wave-uniform
// LDS base + lane * size; the source address is per lane.
// An opaque copy of a lane value: stops loop strength reduction from turning "uniform tile base +
// lane offset" into one loop-carried 64-bit pointer per DMA stream (30 VGPRs in the dK/dV kernel);
// the DMA then uses the SGPR-base + 32-bit VGPR-offset form.
__device__ __forceinline__ uint32_t vopaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ void glds16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src, (VS_LDS void*)dst, 16, 0, 0);
}
// The same DMA as inline asm, invisible to hipcc's waitcnt insertion.  Beside more in-flight
// LDS-DMA stores than it can track separately, hipcc waits vmcnt(0) before every LDS read and so
// drains a prefetch ring; a kernel using this form must order its own LDS reads after the DMA
// with counted s_waitcnt vmcnt + barriers, and must not mix it with compiler-visible loads in the
// same span.  M0 is saved and restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16_asm(const void* src, void* dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(VS_LDS void*)dst;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}
// The same with a wave-uniform 64-bit SGPR base and a 32-bit per-lane byte offset (saddr form:
// one VGPR per stream instead of a 64-bit address pair).
__device__ __forceinline__ void glds16_asm_so(const void* sbase, uint32_t voff, void* dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(VS_LDS void*)dst;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}
// 4 bytes per lane (64 lanes -> 256 B), SGPR base + per-lane 32-bit offset, invisible to hipcc's
// waitcnt tracking like glds16_asm_so
__device__ __forceinline__ void glds4_asm_so(const void* sbase, uint32_t voff, void* dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(VS_LDS void*)dst;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}
// Four 1-KiB pieces from one SGPR base (per-piece 32-bit lane offsets) to the LDS byte addresses
// l0..l3, already wave-uniform values: one M0 save / restore per four pieces and no generic -> LDS
// pointer conversion per piece (each glds16_asm_so pays a readfirstlane pair and a null check).
__device__ __forceinline__ void glds16x4_m0(const void* sbase, uint32_t o0, uint32_t o1, uint32_t o2, uint32_t o3,
                                            uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %6\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %5\n\t"
      "s_mov_b32 m0, %7\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %5\n\t"
      "s_mov_b32 m0, %8\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %5\n\t"
      "s_mov_b32 m0, %9\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %5\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(o0), "v"(o1), "v"(o2), "v"(o3), "s"(sbase), "s"(l0), "s"(l1), "s"(l2), "s"(l3)
      : "memory");
}
__device__ __forceinline__ void glds4(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src, (VS_LDS void*)dst, 4, 0, 0);
}


}  // namespace vs
