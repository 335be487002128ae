// Workgroups resident per CU for a 512-thread kernel at a given dynamic LDS size: the runtime's
// occupancy answer and the measured one (each workgroup spins ~200 us and records its CU and its
// start / end wall clock; the host counts the most intervals overlapping on one CU).
// usage: lds_residency <lds_bytes> [threads]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <map>
#include <algorithm>

__global__ void __launch_bounds__(1024) spin(unsigned long long* rec) {
  extern __shared__ float lds[];
  const unsigned long long t0 = wall_clock64();
  lds[threadIdx.x] = (float)threadIdx.x;
  while (wall_clock64() - t0 < 20000) {  // 100 MHz: 200 us
  }
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    rec[3 * blockIdx.x] = ((unsigned long long)(xcc & 15) << 16) | (unsigned)__smid();
    rec[3 * blockIdx.x + 1] = t0;
    rec[3 * blockIdx.x + 2] = t1 + (unsigned long long)lds[0];
  }
}

int main(int argc, char** argv) {
  const int lds = argc > 1 ? atoi(argv[1]) : 0, th = argc > 2 ? atoi(argv[2]) : 512;
  hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  int per_cu = -1, cus = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, spin, th, lds);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int nb = cus * 4;
  unsigned long long* d;
  hipMalloc(&d, 3 * 8 * nb);
  hipLaunchKernelGGL(spin, dim3(nb), dim3(th), lds, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<unsigned long long> h(3 * nb);
  hipMemcpy(h.data(), d, 3 * 8 * nb, hipMemcpyDeviceToHost);
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
  for (int b = 0; b < nb; ++b) {
    ev[h[3 * b]].push_back({h[3 * b + 1], +1});
    ev[h[3 * b]].push_back({h[3 * b + 2], -1});
  }
  int best = 0;
  for (auto& kv : ev) {
    auto v = kv.second;
    std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
    int cur = 0;
    for (auto& e : v) best = std::max(best, cur += e.second);
  }
  printf("threads %d lds %d: occupancy API %d per CU, measured max %d per CU (%zu CUs seen)\n", th, lds, per_cu, best, ev.size());
  return 0;
}
