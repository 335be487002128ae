// Internal host-side helpers shared by the libthzdoe translation units:
// thread-local error text, HIP error mapping, per-device FFT plan cache.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/thzdoe.h"
#include "thz_fft.hpp"

namespace thz {

void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define THZ_HIP_CHECK(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return ::thz::fail(THZ_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                         __FILE__, __LINE__);                                                \
  } while (0)

#define THZ_LAUNCH_CHECK() THZ_HIP_CHECK(hipGetLastError())

constexpr int FFT_MAX_N = 16384;

// Factorise n and return a plan whose twiddle table lives on the current device.
// Returns THZ_OK or an error code (message set).
int get_plan(int n, FftPlan* out);

// Optional per-kernel HIP-event timing (thz_timing_*): when enabled, every launch is
// bracketed by two events recorded on the launch stream.
struct KernelTimer {
  const char* name;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  KernelTimer(const char* n, hipStream_t s);
  void stop();
};

// Threads per workgroup for a length-n LDS transform.
// FFT_MAXV values per thread -> n/16 threads (512 for n = 8192, 1024 for n = 16384).
// rows in-place-capable transforms of length n at row stride `stride` elements (thz_asm.hip)
int fft_rows_strided(const void* in, void* out, int rows, int n, size_t stride, int inverse, hipStream_t s);

inline int fft_threads(int n) {
  int t = (n + FFT_MAXV - 1) / FFT_MAXV;
  t = (t + 63) / 64 * 64;
  if (t < 64) t = 64;
  return t;
}
// data rows + the two-level twiddle table of the power-of-two kernels
inline size_t fft_lds_bytes(int n) { return (size_t)(lds_floats2(n) + tw_lds_count(n)) * sizeof(float2); }
// LDS of a row / column workgroup that runs fft_pow2_run: the split-exchange image (one float
// per element) for the compile-time power-of-two sizes, the complex image for runtime plans
inline size_t fft_lds_bytes_io(int n) {
  const bool pow2 = n >= 1024 && n <= 16384 && (n & (n - 1)) == 0;
  if (pow2) return (size_t)(lds_split_f2(n) + tw_lds_count(n)) * sizeof(float2);
  return fft_lds_bytes(n);
}

}  // namespace thz
