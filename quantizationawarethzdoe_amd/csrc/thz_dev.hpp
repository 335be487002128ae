// Device helpers shared by the propagator kernels (ASM, CZT, RSC) and the DOE kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace thz {

// Blocks b and b+8 share an XCD (MI355X_MICROARCH.md §Workgroup dispatch).  Map each run
// of 16 consecutive rows (one 128-B line of a column-major T/U column) onto one XCD so
// the strided 8-B accesses of K1/K3 combine in that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_rows(int b, int nb) {
  if (nb & 127) return b;
  const int xcd = b & 7, slot = b >> 3;
  return (((slot >> 4) << 3) + xcd) * 16 + (slot & 15);
}

// Contiguous chunk of block ids per XCD (the bijective form of cdna_hip_programming.md §5):
// consecutive logical ids land on one XCD and start close together in time.  Speed only.
__device__ __forceinline__ int xcd_chunk(int b, int nb) {
  const int xcd = b & 7, q = nb >> 3, r = nb & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Blocked column-major layout of the spectral intermediates T and U: element (c, row) of a
// plane lives at ((cb * rows + row) * CB + c % CB), cb = c / CB.  A row pass then touches CB
// consecutive columns as one 128-B segment (K1 stores, K3 gathers), and the column pass
// touches one 8-B element per segment; the CB column workgroups sharing a segment run on
// one XCD back to back (xcd_chunk) so the L2 merges their partial lines.
constexpr int CB = 16;
__device__ __forceinline__ size_t blk(int c, int row, int rows) {
  return ((size_t)(c / CB) * rows + row) * CB + (c % CB);
}


// sin/cos of a float angle (|ang| up to ~1e5 rad): 3-constant Cody-Waite reduction by pi/2
// (exact for the quadrant counts reached here), then minimax polynomials on [-pi/4, pi/4].
// ~1 ulp, a few registers -- ocml's large-argument sincosf path is avoided because it
// triples the register footprint of the column kernel.
__device__ __forceinline__ void sincos_rad(float ang, float* sn, float* cs) {
  const float q = rintf(ang * 0.636619772367581343f);
  float r = fmaf(-q, 1.5707963705062866f, ang);
  r = fmaf(-q, -4.3711388286737929e-08f, r);
  r = fmaf(-q, -1.7151245100059206e-15f, r);
  const float r2 = r * r;
  // sin(r) ~ r + r^3 (s1 + r^2 (s2 + r^2 s3)),  cos(r) ~ 1 + r^2 (c1 + r^2 (c2 + r^2 (c3 + r^2 c4)))
  float ps = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(r2, ps, -1.6666654611e-1f);
  const float sr = fmaf(r * r2, ps, r);
  float pc = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(r2, pc, 4.166664568298827e-2f);
  pc = fmaf(r2, pc, -0.5f);
  const float cr = fmaf(r2, pc, 1.0f);
  const int iq = (int)q;
  const bool swap = iq & 1;
  float s0 = swap ? cr : sr;
  float c0 = swap ? sr : cr;
  if (iq & 2) s0 = -s0;
  if ((iq + 1) & 2) c0 = -c0;
  *sn = s0;
  *cs = c0;
}


// Complex exp(i phase) for a phase held in double (chirps of the CZT); reduced in double,
// evaluated in fp32.
__device__ __forceinline__ float2 cis_d(double ph) {
  const double tw = 6.283185307179586476925;
  ph -= tw * rint(ph / tw);
  float sn, cs;
  sincos_rad((float)ph, &sn, &cs);
  return make_float2(cs, sn);
}

__device__ __forceinline__ int freq_index(int i, int n) { return i < n - n / 2 ? i : i - n; }

}  // namespace thz
