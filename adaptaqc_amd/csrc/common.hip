// Library-wide state: error strings, device selection, per-family kernel timing.
#include <map>
#include <mutex>

#include "aqc_internal.h"

namespace aqc {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

namespace {
struct PendingEvent {
  std::string family;
  hipEvent_t start, stop;
  double bytes, flops;
};
struct FamilyStats {
  double ms = 0, bytes = 0, flops = 0;
  int64_t launches = 0;
};
std::mutex g_timing_mutex;
bool g_timing = false;
std::vector<PendingEvent> g_pending;
std::vector<size_t> g_open;  // indices of begun-not-ended events
std::map<std::string, FamilyStats> g_stats;

void drain_locked() {
  for (auto& p : g_pending) {
    hipEventSynchronize(p.stop);
    float ms = 0.f;
    hipEventElapsedTime(&ms, p.start, p.stop);
    auto& s = g_stats[p.family];
    s.ms += ms;
    s.bytes += p.bytes;
    s.flops += p.flops;
    s.launches += 1;
    hipEventDestroy(p.start);
    hipEventDestroy(p.stop);
  }
  g_pending.clear();
  g_open.clear();
}
}  // namespace

void KernelTimer::begin(hipStream_t stream, const char* family, double bytes, double flops) {
  if (!g_timing) return;
  std::lock_guard<std::mutex> lk(g_timing_mutex);
  PendingEvent p;
  p.family = family;
  p.bytes = bytes;
  p.flops = flops;
  hipEventCreate(&p.start);
  hipEventCreate(&p.stop);
  hipEventRecord(p.start, stream);
  g_pending.push_back(p);
  g_open.push_back(g_pending.size() - 1);
}

void KernelTimer::end(hipStream_t stream) {
  if (!g_timing) return;
  std::lock_guard<std::mutex> lk(g_timing_mutex);
  if (g_open.empty()) return;
  size_t i = g_open.back();
  g_open.pop_back();
  hipEventRecord(g_pending[i].stop, stream);
  if (g_pending.size() > 4096) drain_locked();
}

}  // namespace aqc

extern "C" {

const char* aqc_last_error(void) { return aqc::g_last_error.c_str(); }

int aqc_version(void) { return 1; }

int aqc_init(int device) {
  int count = 0;
  AQC_HIP_CHECK(hipGetDeviceCount(&count));
  AQC_REQUIRE(device >= 0 && device < count, "aqc_init: device index out of range");
  AQC_HIP_CHECK(hipSetDevice(device));
  return AQC_OK;
}

int aqc_finalize(void) {
  std::lock_guard<std::mutex> lk(aqc::g_timing_mutex);
  aqc::drain_locked();
  return AQC_OK;
}

int aqc_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(aqc::g_timing_mutex);
  if (!on) aqc::drain_locked();
  aqc::g_timing = on != 0;
  return AQC_OK;
}

int aqc_timing_query(const char* name, double* total_ms, int64_t* launches, double* bytes,
                     double* flops) {
  std::lock_guard<std::mutex> lk(aqc::g_timing_mutex);
  aqc::drain_locked();
  auto it = aqc::g_stats.find(name ? name : "");
  if (it == aqc::g_stats.end()) {
    if (total_ms) *total_ms = 0;
    if (launches) *launches = 0;
    if (bytes) *bytes = 0;
    if (flops) *flops = 0;
    return AQC_OK;
  }
  if (total_ms) *total_ms = it->second.ms;
  if (launches) *launches = it->second.launches;
  if (bytes) *bytes = it->second.bytes;
  if (flops) *flops = it->second.flops;
  return AQC_OK;
}

int aqc_timing_reset(void) {
  std::lock_guard<std::mutex> lk(aqc::g_timing_mutex);
  aqc::drain_locked();
  aqc::g_stats.clear();
  return AQC_OK;
}

}  // extern "C"
