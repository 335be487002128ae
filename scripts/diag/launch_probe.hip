// Per-kernel floor of small launches in a replayed HIP graph: the thz
// training steps' trivial kernels (thz_step_fetch, thz_adam_step, the loss finish) take 4.5-5 us
// each under rocprofv3 while the ATen trivial kernels in the same trace take 1.8-2.7 us.  This
// probe separates the candidates: the same empty kernel with a 4-byte and an AsmArgs-sized (1.7 KB)
// argument block, a kernel that stores one int, one that reads pinned host memory, one that
// counts arrivals with a device atomic, and the library's thz_step_fetch / thz_adam_step -- each
// as a chain of 20 nodes in one captured graph (replayed 50 times) and, for comparison, the empty
// kernel and thz_step_fetch launched eagerly.  Run under rocprofv3 --kernel-trace --stats; the
// probe also prints the wall time per node from events.
//
//   hipcc --offload-arch=gfx950 -O3 -o launch_probe launch_probe.hip -I../../include \
//         -L../../quantizationawarethzdoe_amd -lthzdoe -Wl,-rpath,$PWD/../../quantizationawarethzdoe_amd
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "thzdoe.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)
#define CT(x)                                                                              \
  do {                                                                                     \
    int e_ = (x);                                                                          \
    if (e_) {                                                                              \
      std::fprintf(stderr, "%s:%d %s: thz error %d\n", __FILE__, __LINE__, #x, e_);        \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

struct Big {
  int v[432];  // 1728 bytes, about sizeof(thz::AsmArgs)
};

template <int TAG>
__global__ void k_empty(int x) {
  if (x == 12345678) __builtin_trap();
}
__global__ void k_big(Big b) {
  if (b.v[0] == 12345678) __builtin_trap();
}
__global__ void k_store(int* p) {
  if (threadIdx.x == 0) p[0] = 1;
}
__global__ void k_hostread(const volatile int* host, int* p) {
  if (threadIdx.x == 0) p[1] = host[0];
}
__global__ void k_count(unsigned* c) {
  if (threadIdx.x == 0) atomicAdd(c, 1u);
}

static const int CHAIN = 20, REPLAYS = 50;

template <class F>
static double graph_chain(hipStream_t s, const char* name, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < CHAIN; ++i) launch(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));  // warm-up
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < REPLAYS; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / (REPLAYS * CHAIN);
  std::printf("graph %-14s %7.2f us per node (wall, %d-node chain)\n", name, us, CHAIN);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return us;
}

template <class F>
static double eager_chain(hipStream_t s, const char* name, F launch) {
  for (int i = 0; i < CHAIN; ++i) launch(s);
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int r = 0; r < REPLAYS; ++r)
    for (int i = 0; i < CHAIN; ++i) launch(s);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / (REPLAYS * CHAIN);
  std::printf("eager %-14s %7.2f us per launch (wall)\n", name, us);
  return us;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* dev_i = nullptr;
  unsigned* dev_c = nullptr;
  CK(hipMalloc(&dev_i, 64 * sizeof(int)));
  CK(hipMalloc(&dev_c, sizeof(unsigned)));
  CK(hipMemset(dev_i, 0, 64 * sizeof(int)));
  int* host = nullptr;
  CK(hipHostMalloc(&host, 16 * 64 * sizeof(int), hipHostMallocMapped));
  for (int i = 0; i < 16 * 64; ++i) host[i] = i;
  int* host_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&host_dev, host, 0));
  // Adam over one 2,500-float parameter (the four-focal-spots weight)
  const int n = 2500;
  float *p, *g, *m, *v, *st;
  unsigned* done;
  CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&g, n * 4));
  CK(hipMalloc(&m, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&st, 4));
  CK(hipMalloc(&done, 4));
  CK(hipMemset(p, 0, n * 4));
  CK(hipMemset(g, 0, n * 4));
  CK(hipMemset(m, 0, n * 4));
  CK(hipMemset(v, 0, n * 4));
  CK(hipMemset(st, 0, 4));
  CK(hipMemset(done, 0, 4));
  thz_adam_desc ad{0.02, 0.9, 0.999, 1e-8, 0.0, 0, 1, done};
  thz_adam_param ap{p, g, m, v, st, n};
  Big big{};
  hipStream_t hs = s;
  int* state = dev_i + 8;

  graph_chain(s, "empty_4B", [&](hipStream_t q) { hipLaunchKernelGGL(k_empty<0>, dim3(1), dim3(64), 0, q, 1); });
  graph_chain(s, "empty_1728B", [&](hipStream_t q) { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, q, big); });
  graph_chain(s, "store", [&](hipStream_t q) { hipLaunchKernelGGL(k_store, dim3(1), dim3(64), 0, q, dev_i); });
  graph_chain(s, "host_read", [&](hipStream_t q) {
    hipLaunchKernelGGL(k_hostread, dim3(1), dim3(64), 0, q, (const volatile int*)host_dev, dev_i);
  });
  graph_chain(s, "atomic_count", [&](hipStream_t q) { hipLaunchKernelGGL(k_count, dim3(1), dim3(64), 0, q, dev_c); });
  graph_chain(s, "step_fetch", [&](hipStream_t q) { CT(thz_step_fetch(host_dev, 16, 8, state, dev_i + 32, (thz_stream_t)q)); });
  graph_chain(s, "adam_step", [&](hipStream_t q) { CT(thz_adam_step(&ad, &ap, (thz_stream_t)q)); });
  eager_chain(s, "empty_4B", [&](hipStream_t q) { hipLaunchKernelGGL(k_empty<1>, dim3(1), dim3(64), 0, q, 1); });
  eager_chain(hs, "step_fetch", [&](hipStream_t q) { CT(thz_step_fetch(host_dev, 16, 8, state, dev_i + 32, (thz_stream_t)q)); });
  CK(hipStreamSynchronize(s));
  std::printf("probe done\n");
  return 0;
}
