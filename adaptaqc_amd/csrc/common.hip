// Library-wide state: error strings, device selection, per-family kernel timing, teardown.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "aqc_internal.h"

namespace aqc {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

namespace {
std::mutex g_fin_mutex;
std::vector<void (*)()> g_fin;         // cleanups, in registration order
std::atomic<unsigned long long> g_devs{0};  // bit d: device d was used
}  // namespace

void on_finalize(void (*fn)()) {
  std::lock_guard<std::mutex> lk(g_fin_mutex);
  for (auto f : g_fin)
    if (f == fn) return;
  g_fin.push_back(fn);
}

namespace {
__global__ __launch_bounds__(256) void k_upload(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16,
                                                int tail) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < tail)
    reinterpret_cast<unsigned char*>(dst + n16)[threadIdx.x] = reinterpret_cast<const unsigned char*>(src + n16)[threadIdx.x];
}
}  // namespace

int upload_async(void* dst, const void* pinned_src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return AQC_OK;
  // Below AQC_UPLOAD_MIN_KB (default 16) hipMemcpyAsync stays: the runtime's small-copy path was
  // ~20 us faster per single MPS evaluation than the kernel; above it the runtime switches to the
  // copy engine.  AQC_UPLOAD=memcpy: hipMemcpyAsync everywhere (A/B).
  static const size_t min_bytes = [] {
    const char* e = std::getenv("AQC_UPLOAD");
    if (e && std::strcmp(e, "memcpy") == 0) return ~(size_t)0;
    const char* k = std::getenv("AQC_UPLOAD_MIN_KB");
    return (size_t)(k ? std::max(0, std::atoi(k)) : 16) << 10;
  }();
  if (bytes < min_bytes || (((uintptr_t)dst | (uintptr_t)pinned_src) & 15)) {
    AQC_HIP_CHECK(hipMemcpyAsync(dst, pinned_src, bytes, hipMemcpyHostToDevice, st));
    return AQC_OK;
  }
  const size_t n16 = bytes / 16;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(1024, (n16 + 255) / 256));
  hipLaunchKernelGGL(k_upload, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const uint4*>(pinned_src),
                     reinterpret_cast<uint4*>(dst), n16, (int)(bytes % 16));
  AQC_HIP_CHECK(hipGetLastError());
  return AQC_OK;
}

void note_device(int dev) {
  if (dev >= 0 && dev < 64) g_devs.fetch_or(1ull << dev);
}

namespace {
std::mutex g_pool_mutex;
struct PoolKey {
  int dev;
  size_t bytes;
  bool operator<(const PoolKey& o) const { return dev != o.dev ? dev < o.dev : bytes < o.bytes; }
};
std::map<PoolKey, std::vector<void*>> g_pool_free;  // cached blocks
std::map<void*, PoolKey> g_pool_live;               // blocks handed out
size_t g_pool_cached = 0, g_pool_limit = 0;
unsigned long long g_pool_hits = 0, g_pool_misses = 0;

void pool_release_locked() {
  int cur = 0;
  const bool have = hipGetDevice(&cur) == hipSuccess;
  for (auto& kv : g_pool_free) {
    if (kv.second.empty()) continue;
    (void)hipSetDevice(kv.first.dev);
    for (void* p : kv.second) (void)hipFree(p);
    kv.second.clear();
  }
  if (have) (void)hipSetDevice(cur);
  g_pool_free.clear();
  g_pool_cached = 0;
}

void pool_release() {
  std::lock_guard<std::mutex> lk(g_pool_mutex);
  pool_release_locked();
}
}  // namespace

void* dev_alloc(size_t bytes) {
  const size_t b = (std::max<size_t>(bytes, 1) + 4095) & ~(size_t)4095;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mutex);
  if (g_pool_limit == 0) {
    const char* e = std::getenv("AQC_POOL_MB");
    g_pool_limit = (size_t)(e ? std::max(0.0, std::atof(e)) : 8192.0) * (1ull << 20) + 1;
    on_finalize(pool_release);
  }
  const PoolKey key{dev, b};
  void* p = nullptr;
  auto it = g_pool_free.find(key);
  if (it != g_pool_free.end() && !it->second.empty()) {
    p = it->second.back();
    it->second.pop_back();
    g_pool_cached -= b;
    ++g_pool_hits;
  } else if (++g_pool_misses, hipMalloc(&p, b) != hipSuccess) {
    (void)hipGetLastError();
    pool_release_locked();
    (void)hipSetDevice(dev);
    if (hipMalloc(&p, b) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  g_pool_live[p] = key;
  note_device(dev);
  return p;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pool_mutex);
  auto it = g_pool_live.find(p);
  if (it == g_pool_live.end()) {  // (not from dev_alloc)
    (void)hipFree(p);
    return;
  }
  const PoolKey key = it->second;
  g_pool_live.erase(it);
  if (g_pool_cached + key.bytes < g_pool_limit) {
    g_pool_free[key].push_back(p);
    g_pool_cached += key.bytes;
  } else {
    int cur = 0;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    (void)hipSetDevice(key.dev);
    (void)hipFree(p);
    if (have) (void)hipSetDevice(cur);
  }
}

namespace {
// Fatal-signal report: the signal and a native backtrace on stderr, then the previous handler
// (Python's faulthandler, the default action) runs as if we had never been there.  Installed when
// the library is loaded unless AQC_CRASH_TRACE=0.
struct sigaction g_old_segv, g_old_bus, g_old_abrt;
void crash_handler(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  char msg[128];
  const int n = snprintf(msg, sizeof(msg), "libaqchip: fatal signal %d (fault address %p), native backtrace:\n", sig,
                         si ? si->si_addr : nullptr);
  if (n > 0) (void)!write(2, msg, (size_t)n);
  void* frames[64];
  const int nf = backtrace(frames, 64);
  backtrace_symbols_fd(frames, nf, 2);
  const struct sigaction* old = sig == SIGSEGV ? &g_old_segv : sig == SIGBUS ? &g_old_bus : &g_old_abrt;
  sigaction(sig, old, nullptr);
  raise(sig);
}
__attribute__((constructor)) void install_crash_handler() {
  const char* e = std::getenv("AQC_CRASH_TRACE");
  if (e && std::strcmp(e, "0") == 0) return;
  void* warm[2];
  (void)backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = crash_handler;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_old_segv);
  sigaction(SIGBUS, &sa, &g_old_bus);
  sigaction(SIGABRT, &sa, &g_old_abrt);
}
}  // namespace

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

// Test load: every workgroup holds its CU for a staggered time (block b: (b % 16 + 1) / 16 of
// `ticks`), so that kernels queued behind it on other streams get their workgroups dispatched one
// CU at a time -- the late-start case of the multi-workgroup exchanges (gram_big.hip).
__global__ __launch_bounds__(256) void k_hog(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long lim = ticks * (unsigned long long)(blockIdx.x % 16 + 1) / 16ull;
  while (__builtin_amdgcn_s_memrealtime() - t0 < lim) __builtin_amdgcn_s_sleep(8);
}

namespace {
hipStream_t g_hog_stream[64] = {nullptr};
void release_hog_streams() {
  for (auto& s : g_hog_stream)
    if (s) (void)hipStreamDestroy(s), s = nullptr;
}
}  // namespace

}  // namespace aqc

extern "C" {

int aqc_debug_hog(int nblocks, double ms) {
  AQC_REQUIRE(nblocks > 0 && nblocks <= 65536 && ms >= 0 && ms <= 1000, "aqc_debug_hog: bad arguments");
  int dev = 0;
  AQC_HIP_CHECK(hipGetDevice(&dev));
  AQC_REQUIRE(dev >= 0 && dev < 64, "aqc_debug_hog: device index out of range");
  if (!aqc::g_hog_stream[dev]) {
    AQC_HIP_CHECK(hipStreamCreateWithFlags(&aqc::g_hog_stream[dev], hipStreamNonBlocking));
    aqc::note_device(dev);
    aqc::on_finalize(aqc::release_hog_streams);
  }
  hipLaunchKernelGGL(aqc::k_hog, dim3(nblocks), dim3(256), 0, aqc::g_hog_stream[dev],
                     (unsigned long long)(ms * 1e5));
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

int aqc_pool_stats(double* out) {
  AQC_REQUIRE(out, "aqc_pool_stats: null out");
  std::lock_guard<std::mutex> lk(aqc::g_pool_mutex);
  size_t live = 0;
  for (const auto& kv : aqc::g_pool_live) live += kv.second.bytes;
  out[0] = (double)aqc::g_pool_cached;
  out[1] = (double)live;
  out[2] = (double)aqc::g_pool_live.size();
  out[3] = (double)aqc::g_pool_hits;
  out[4] = (double)aqc::g_pool_misses;
  return AQC_OK;
}

const char* aqc_last_error(void) { return aqc::g_last_error.c_str(); }

int aqc_version(void) { return 1; }

int aqc_init(int device) {
  int count = 0;
  AQC_HIP_CHECK(hipGetDeviceCount(&count));
  AQC_REQUIRE(device >= 0 && device < count, "aqc_init: device index out of range");
  AQC_HIP_CHECK(hipSetDevice(device));
  aqc::note_device(device);
  return AQC_OK;
}

int aqc_finalize(void) {
  {
    std::lock_guard<std::mutex> lk(aqc::g_timing_mutex);
    aqc::drain_locked();
  }
  // every device the library used: drain all its streams (the side streams' kernels are ordered
  // only by events), then release the lazily created objects
  int cur = 0;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  const unsigned long long devs = aqc::g_devs.load();
  int rc = AQC_OK;
  for (int d = 0; d < 64; ++d) {
    if (!(devs >> d & 1ull)) continue;
    if (hipSetDevice(d) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      aqc::set_error("aqc_finalize: device synchronisation failed");
      rc = AQC_ERR_HIP;
    }
  }
  if (have_cur) (void)hipSetDevice(cur);
  std::vector<void (*)()> fin;
  {
    std::lock_guard<std::mutex> lk(aqc::g_fin_mutex);
    fin.swap(aqc::g_fin);
  }
  for (auto it = fin.rbegin(); it != fin.rend(); ++it) (*it)();
  return rc;
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
