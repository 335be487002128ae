// Accuracy of the hardware v_sin_f32 / v_cos_f32 (input in revolutions) after an exact
// two-constant reduction, against double sincos, for phases up to ~2000 rad; compared with
// the software sincos_rad the kernels use.  Diagnostic only (run on the GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../../quantizationawarethzdoe_amd/csrc/thz_dev.hpp"

__global__ void k(int n, float* err_sw, float* err_hw) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float ph = 2000.0f * ((float)i / (float)n) - 1000.0f + 1e-3f * (float)(i % 97);
  double s, c;
  sincos((double)ph, &s, &c);
  float ss, cc;
  thz::sincos_rad(ph, &ss, &cc);
  err_sw[i] = fmaxf(fabsf(ss - (float)s), fabsf(cc - (float)c));
  // hardware: t = ph / (2 pi) split exactly, reduce to [-0.5, 0.5] revolutions
  const float C_HI = 0.15915494f;                 // fp32(1 / 2pi)
  const float C_LO = (float)(0.15915494309189535 - (double)0.15915494f);
  float t = ph * C_HI;
  float e = fmaf(ph, C_HI, -t) + ph * C_LO;
  float r = (t - rintf(t)) + e;
  float hs = __builtin_amdgcn_sinf(r), hc = __builtin_amdgcn_cosf(r);
  err_hw[i] = fmaxf(fabsf(hs - (float)s), fabsf(hc - (float)c));
}

int main() {
  const int n = 1 << 24;
  float *a, *b;
  hipMalloc(&a, n * 4);
  hipMalloc(&b, n * 4);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, n, a, b);
  float* ha = (float*)malloc(n * 4);
  float* hb = (float*)malloc(n * 4);
  hipMemcpy(ha, a, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, n * 4, hipMemcpyDeviceToHost);
  double ma = 0, mb = 0, sa = 0, sb = 0;
  for (int i = 0; i < n; ++i) { ma = fmax(ma, ha[i]); mb = fmax(mb, hb[i]); sa += ha[i]; sb += hb[i]; }
  printf("sw sincos_rad: max %.3e mean %.3e\nhw v_sin/v_cos: max %.3e mean %.3e\n", ma, sa / n, mb, sb / n);
  return 0;
}
