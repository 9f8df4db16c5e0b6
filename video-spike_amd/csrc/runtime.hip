// runtime.hip — error reporting, version, kernel timers (bench instrumentation).
#include <mutex>
#include <string.h>
#include <vector>

#include "common.h"

namespace vs {

static thread_local char g_err[512] = "";
thread_local int g_timer_tag = -1;

void set_error(const char* msg) {
  strncpy(g_err, msg, sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

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

extern "C" int vs_version(void) { return 3; }  // 2: vs_vit_layer_grad.flags; 3: .chain

extern "C" int vs_struct_size(int which) {
  switch (which) {
    case 0: return (int)sizeof(vs_gemm_desc);
    case 1: return (int)sizeof(vs_vit_layer);
    case 2: return (int)sizeof(vs_vit_layer_grad);
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
