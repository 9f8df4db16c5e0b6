// runtime.hip — error reporting, version / build id, knobs, dispatch counters, kernel timers.
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <string.h>
#include <vector>

#include "common.h"

#ifndef VS_BUILD_ID
#define VS_BUILD_ID "unknown"
#endif

namespace vs {

static thread_local char g_err[512] = "";
thread_local int g_timer_tag = -1;

void set_error(const char* msg) {
  strncpy(g_err, msg, sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

// ---- knobs: environment read once (first use), then vs_knob_set overrides -------------------
struct KnobDef {
  const char* env;
  int dflt;
};
static const KnobDef kKnobs[VS_KNOB_COUNT] = {
    {"VSPIKE_DW_OLD", 0},      {"VSPIKE_NO_SKINNY", 0},    {"VSPIKE_NO_SLAB", 0},      {"VSPIKE_NO_BIG", 0},
    {"VSPIKE_NO_WRES", 0},     {"VSPIKE_WRES_GBWD", 0},    {"VSPIKE_NO_WSLAB", 0},     {"VSPIKE_WSLAB", 0},
    {"VSPIKE_WSLAB_G", 512},   {"VSPIKE_PANEL", 0},        {"VSPIKE_NO_PANEL", 0},     {"VSPIKE_PANEL_GRID", 512},
    {"VSPIKE_NO_FULLK", 0},    {"VSPIKE_NO_RING", 0},      {"VSPIKE_NO_LNF_FUSE", 0},  {"VSPIKE_NO_LN_FUSE", 0},
    {"VSPIKE_DW_BM", 0},       {"VSPIKE_DW_BN", 0},        {"VSPIKE_DW_SPLITS", 0},    {"VSPIKE_DW_STAGES", 0},
    {"VSPIKE_LN_BLOCKS", 0},   {"VSPIKE_DH_F32", 0},       {"VSPIKE_NO_PATCH_FUSED", 0}, {"VSPIKE_NO_DW_GROUP", 0},
    {"VSPIKE_ATTN_VARIANT", 0}, {"VSPIKE_SLAB_WV", 0}, {"VSPIKE_WRES_WV", 0}, {"VSPIKE_WRES_DBG", 0}, {"VSPIKE_G256", 0}, {"VSPIKE_G256_GRID", 0}, {"VSPIKE_G256_DBG", 0}, {"VSPIKE_NO_DW256", 0}, {"VSPIKE_G256_STAGGER", 0}, {"VSPIKE_CONV_DW128", 0},
    {"VSPIKE_CONV_MFMA", 0}, {"VSPIKE_G256_A3", 0}, {"VSPIKE_DW256_ALL", 0}, {"VSPIKE_LN_FWD_BLOCKS", 0},
    {nullptr, 0}};
static std::atomic<int> g_knob[VS_KNOB_COUNT];
static std::once_flag g_knob_once;
static void knob_init() {
  for (int i = 0; i < VS_KNOB_COUNT; ++i) {
    int v = kKnobs[i].dflt;
    if (kKnobs[i].env) {
      const char* e = getenv(kKnobs[i].env);
      if (e && e[0]) v = (int)strtol(e, nullptr, 0);  // decimal or 0x hex
    }
    g_knob[i].store(v, std::memory_order_relaxed);
  }
}
int knob(int id) {
  std::call_once(g_knob_once, knob_init);
  return g_knob[id].load(std::memory_order_relaxed);
}

static std::atomic<int64_t> g_dispatch[VS_PATH_COUNT];
void count_path(int id) { g_dispatch[id].fetch_add(1, std::memory_order_relaxed); }

// Event pairs recorded around tracked launches while timing is enabled.  Events are pooled and
// only read back in vs_timing_collect(), so recording never synchronises the stream.
struct TimerState {
  std::mutex mu;
  unsigned mask = 0;  // bit t set: timer t records
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pairs[VS_TIMER_COUNT];
  double bytes[VS_TIMER_COUNT] = {};
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
};
static TimerState g_t;

ScopedTimer::ScopedTimer(int t, hipStream_t s, double algorithmic_bytes) : timer(t), stream(s), ev_end(nullptr) {
  if (!((g_t.mask >> t) & 1u)) return;
  std::lock_guard<std::mutex> lk(g_t.mu);
  g_t.bytes[t] += algorithmic_bytes;
  hipEvent_t a = g_t.get(), b = g_t.get();
  (void)hipEventRecord(a, s);
  g_t.pairs[t].push_back({a, b});
  ev_end = (void*)b;
}
ScopedTimer::~ScopedTimer() {
  if (ev_end) (void)hipEventRecord((hipEvent_t)ev_end, stream);
}

}  // namespace vs

// 2: vs_vit_layer_grad.flags; 3: .chain; 4: bf16-mode a_pre holds gelu'(pre), d_h may be bf16,
// knobs / dispatch counters / build id; 5: a_pre == NULL selects the fused MLP (vs_mlp_*);
// 6: vs_vit_layer.fp8_ws / fp8_ws_bytes and dtype VS_FP8 (MX-FP8 forward products);
// 7: vs_vit_layer.next_ln_* / ln1_ready (the next block's LayerNorm1 in the fused MLP epilogue)
extern "C" int vs_version(void) { return 7; }
extern "C" const char* vs_build_id(void) { return VS_BUILD_ID; }

extern "C" int vs_knob_get(int k) {
  VS_REQUIRE(k >= 0 && k < VS_KNOB_COUNT, "vs_knob_get: unknown knob");
  return vs::knob(k);
}
extern "C" int vs_knob_set(int k, int value) {
  VS_REQUIRE(k >= 0 && k < VS_KNOB_COUNT, "vs_knob_set: unknown knob");
  const int prev = vs::knob(k);
  vs::g_knob[k].store(value, std::memory_order_relaxed);
  return prev;
}
extern "C" int vs_knob_default(int k) {
  VS_REQUIRE(k >= 0 && k < VS_KNOB_COUNT, "vs_knob_default: unknown knob");
  return vs::kKnobs[k].dflt;
}
extern "C" int vs_debug_knobs(void) {
#ifdef VS_DEBUG_KNOBS
  return 1;
#else
  return 0;
#endif
}
extern "C" int vs_dispatch_counts(int64_t* out, int n) {
  for (int i = 0; i < n && i < VS_PATH_COUNT; ++i) out[i] = vs::g_dispatch[i].load(std::memory_order_relaxed);
  return VS_PATH_COUNT;
}
extern "C" int vs_dispatch_reset(void) {
  for (auto& c : vs::g_dispatch) c.store(0, std::memory_order_relaxed);
  return VS_OK;
}

extern "C" int vs_struct_size(int which) {
  switch (which) {
    case 0: return (int)sizeof(vs_gemm_desc);
    case 1: return (int)sizeof(vs_vit_layer);
    case 2: return (int)sizeof(vs_vit_layer_grad);
    case 3: return (int)sizeof(vs_conv3d_desc);
    default: return -1;
  }
}
extern "C" const char* vs_last_error(void) { return vs::g_err; }

extern "C" int vs_device_arch(char* buf, int n) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t p;
  e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return (int)e;
  strncpy(buf, p.gcnArchName, n - 1);
  buf[n - 1] = 0;
  return VS_OK;
}

extern "C" int vs_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(vs::g_t.mu);
  vs::g_t.mask = (unsigned)on;
  if (!on) {
    for (auto& v : vs::g_t.pairs) {
      for (auto& p : v) {
        vs::g_t.pool.push_back(p.first);
        vs::g_t.pool.push_back(p.second);
      }
      v.clear();
    }
    for (auto& b : vs::g_t.bytes) b = 0.0;
  }
  return VS_OK;
}

extern "C" int vs_timing_bytes(int timer, double* algorithmic_bytes) {
  VS_REQUIRE(timer >= 0 && timer < VS_TIMER_COUNT, "vs_timing_bytes: bad timer id");
  std::lock_guard<std::mutex> lk(vs::g_t.mu);
  if (algorithmic_bytes) *algorithmic_bytes = vs::g_t.bytes[timer];
  return VS_OK;
}

extern "C" int vs_timing_collect(int timer, int64_t* launches, double* total_ms) {
  VS_REQUIRE(timer >= 0 && timer < VS_TIMER_COUNT, "vs_timing_collect: bad timer id");
  std::lock_guard<std::mutex> lk(vs::g_t.mu);
  double tot = 0.0;
  int64_t n = 0;
  for (auto& p : vs::g_t.pairs[timer]) {
    hipError_t e = hipEventSynchronize(p.second);
    if (e != hipSuccess) return (int)e;
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, p.first, p.second);
    if (e != hipSuccess) return (int)e;
    tot += ms;
    ++n;
    vs::g_t.pool.push_back(p.first);
    vs::g_t.pool.push_back(p.second);
  }
  vs::g_t.pairs[timer].clear();
  vs::g_t.bytes[timer] = 0.0;
  if (launches) *launches = n;
  if (total_ms) *total_ms = tot;
  return VS_OK;
}
