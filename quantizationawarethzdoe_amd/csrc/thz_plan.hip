// Host side of the FFT engine: factorisation, twiddle tables (double precision on the
// host, stored fp32 on the device), per-device cache, error reporting, and the
// generic batched row-FFT entry point.
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "thz_common.hpp"

namespace thz {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

static std::vector<int> factorise(int n) {
  std::vector<int> r;
  while (n % 16 == 0) { r.push_back(16); n /= 16; }
  if (n % 8 == 0) { r.push_back(8); n /= 8; }
  if (n % 4 == 0) { r.push_back(4); n /= 4; }
  if (n % 2 == 0) { r.push_back(2); n /= 2; }
  for (int p : {3, 5, 7}) {
    while (n % p == 0) { r.push_back(p); n /= p; }
  }
  for (int p = 11; n > 1 && p * p <= n; p += 2) {
    while (n % p == 0) { r.push_back(p); n /= p; }
  }
  if (n > 1) r.push_back(n);
  return r;
}

struct TwEntry {
  float2* dev = nullptr;
};

static std::mutex g_mu;
static std::map<std::pair<int, int>, TwEntry> g_tw;  // (device, n)

int get_plan(int n, FftPlan* out) {
  if (n < 1 || n > FFT_MAX_N) return fail(THZ_E_UNSUPPORTED, "FFT length %d outside [1, %d]", n, FFT_MAX_N);
  std::vector<int> f = factorise(n);
  if ((int)f.size() > FFT_MAX_STAGES) return fail(THZ_E_UNSUPPORTED, "FFT length %d: too many stages", n);
  int dev = 0;
  THZ_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_pair(dev, n);
  auto it = g_tw.find(key);
  if (it == g_tw.end()) {
    std::vector<float2> h(n);
    for (int t = 0; t < n; ++t) {
      // exp(-2 pi i t / n) with exact octant symmetry to keep the table accurate
      double a = -2.0 * M_PI * (double)t / (double)n;
      h[t] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    float2* d = nullptr;
    THZ_HIP_CHECK(hipMalloc(&d, sizeof(float2) * n));
    THZ_HIP_CHECK(hipMemcpy(d, h.data(), sizeof(float2) * n, hipMemcpyHostToDevice));
    it = g_tw.emplace(key, TwEntry{d}).first;
  }
  out->n = n;
  out->nst = (int)f.size();
  for (int s = 0; s < FFT_MAX_STAGES; ++s) out->radix[s] = s < (int)f.size() ? f[s] : 1;
  out->tw = it->second.dev;
  return THZ_OK;
}

// ---------------------------------------------------------------------------------------------
// per-kernel event timing
// ---------------------------------------------------------------------------------------------
struct Pending {
  std::string name;
  hipEvent_t a, b;
};
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<Pending> g_pending;
static std::vector<hipEvent_t> g_pool;
static std::map<std::string, std::pair<double, long>> g_acc;

static hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

KernelTimer::KernelTimer(const char* n, hipStream_t s) : name(n), stream(s) {
  std::lock_guard<std::mutex> lk(g_tmu);
  if (!g_timing) return;
  start = take_event();
  if (start) (void)hipEventRecord(start, stream);
}

void KernelTimer::stop() {
  if (!start) return;
  std::lock_guard<std::mutex> lk(g_tmu);
  hipEvent_t e = take_event();
  if (!e) return;
  (void)hipEventRecord(e, stream);
  g_pending.push_back(Pending{name, start, e});
  start = nullptr;
}

static int drain() {
  for (auto& p : g_pending) {
    THZ_HIP_CHECK(hipEventSynchronize(p.b));
    float ms = 0.f;
    THZ_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
    auto& acc = g_acc[p.name];
    acc.first += ms;
    acc.second += 1;
    g_pool.push_back(p.a);
    g_pool.push_back(p.b);
  }
  g_pending.clear();
  return THZ_OK;
}

}  // namespace thz

extern "C" int thz_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(thz::g_tmu);
  thz::g_timing = on != 0;
  return THZ_OK;
}

extern "C" int thz_timing_reset(void) {
  std::lock_guard<std::mutex> lk(thz::g_tmu);
  int e = thz::drain();
  thz::g_acc.clear();
  return e;
}

extern "C" int thz_timing_read(const char* kernel, double* total_ms, long* launches) {
  std::lock_guard<std::mutex> lk(thz::g_tmu);
  int e = thz::drain();
  if (e) return e;
  auto it = thz::g_acc.find(kernel ? kernel : "");
  if (total_ms) *total_ms = it == thz::g_acc.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == thz::g_acc.end() ? 0 : it->second.second;
  return THZ_OK;
}

extern "C" const char* thz_version(void) { return "thzdoe 0.4.0 gfx950"; }
extern "C" int thz_abi_version(void) { return THZ_ABI_VERSION; }
extern "C" const char* thz_last_error(void) { return thz::g_err.c_str(); }
