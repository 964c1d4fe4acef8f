// enflow_timing.hip -- per-kernel HIP-event timing of the library's own launches.
//
// Off by default (one relaxed atomic load per launch).  When enabled
// (enflow_timing_enable(1)) every launch site wrapped in ENFLOW_TIMED records a
// hipEvent pair on the stream the kernel is launched on; enflow_timing_collect()
// waits for the recorded events and accumulates elapsed milliseconds per kernel
// name.  bench.py reads these to price each dominant kernel against its roofline
// (the event pair brackets exactly one kernel, on its own stream, which
// torch.cuda.Event on torch's current stream cannot guarantee).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "enflow_hip.h"
#include "enflow_timing.h"

namespace {
struct Rec {
  int name;
  hipEvent_t e0, e1;
};
std::atomic<bool> g_on{false};
std::mutex g_mu;
std::vector<std::string> g_names;
std::vector<double> g_ms;
std::vector<long long> g_count;
std::vector<Rec> g_pending;
std::vector<hipEvent_t> g_pool;

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int name_id(const char* n) {
  for (size_t i = 0; i < g_names.size(); ++i)
    if (g_names[i] == n) return (int)i;
  g_names.emplace_back(n);
  g_ms.push_back(0.0);
  g_count.push_back(0);
  return (int)g_names.size() - 1;
}

int collect_locked() {
  for (const Rec& r : g_pending) {
    float ms = 0.f;
    if (r.e0 && r.e1 && hipEventSynchronize(r.e1) == hipSuccess &&
        hipEventElapsedTime(&ms, r.e0, r.e1) == hipSuccess) {
      g_ms[r.name] += ms;
      g_count[r.name] += 1;
    }
    if (r.e0) g_pool.push_back(r.e0);
    if (r.e1) g_pool.push_back(r.e1);
  }
  g_pending.clear();
  return (int)g_names.size();
}
}  // namespace

int enflow_tm_begin(const char* name, hipStream_t st) {
  if (!g_on.load(std::memory_order_relaxed)) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  Rec r{name_id(name), take_event(), take_event()};
  if (r.e0) (void)hipEventRecord(r.e0, st);
  g_pending.push_back(r);
  return (int)g_pending.size() - 1;
}

void enflow_tm_end(int slot, hipStream_t st) {
  if (slot < 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (slot < (int)g_pending.size() && g_pending[slot].e1) (void)hipEventRecord(g_pending[slot].e1, st);
}

extern "C" {

int enflow_timing_enable(int on) {
  g_on.store(on != 0);
  return 0;
}

int enflow_timing_collect(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return collect_locked();
}

int enflow_timing_entry(int i, char* name, int name_len, double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (i < 0 || i >= (int)g_names.size()) return -1;
  if (name && name_len > 0) {
    std::strncpy(name, g_names[i].c_str(), (size_t)name_len - 1);
    name[name_len - 1] = '\0';
  }
  if (total_ms) *total_ms = g_ms[i];
  if (launches) *launches = g_count[i];
  return 0;
}

int enflow_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  collect_locked();
  for (size_t i = 0; i < g_ms.size(); ++i) {
    g_ms[i] = 0.0;
    g_count[i] = 0;
  }
  return 0;
}

}  // extern "C"
