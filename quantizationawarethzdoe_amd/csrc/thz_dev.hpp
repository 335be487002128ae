// Device helpers shared by the propagator kernels (ASM, CZT, RSC) and the DOE kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/thzdoe.h"

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
//
// The per-z intermediate U (column pass -> row pass) uses narrower blocks, CBU = 4 columns (the
// L2 writes back partially dirty sectors at a cost: measured K2 1.93 ms at 16 columns, 1.69 at
// 8, 1.39 at 4, 1.33 unblocked, while the row pass gathers K3 1.05 ms at 16, 1.22 at 4, 2.59
// unblocked; cfg2 sum per z-chunk lowest at 4), laid out as below.
constexpr int CB = 16;
#ifndef THZ_U_CBU
#define THZ_U_CBU 4
#endif
#ifndef THZ_U_URT
#define THZ_U_URT 4
#endif
constexpr int CBU = THZ_U_CBU;  // columns per U tile
constexpr int URT = THZ_U_URT;  // rows per U tile (CBU x URT x 8 B = one 128-B line)
static_assert(CBU * URT == 16, "a U tile is one 128-B line");
__device__ __forceinline__ size_t blk(int c, int row, int rows) {
  return ((size_t)(c / CB) * rows + row) * CB + (c % CB);
}
// U (the column pass's output, the inverse row pass's input) in 4 x 4 tiles of (column, row): a
// 32-B sector holds 4 consecutive ROWS of one column, so each store instruction of the column pass
// fills whole sectors itself (rows j..j+3 of one column come from one workgroup), and the row pass reads
// 8 B of each of 4 sectors of a 128-B line.  The row-major CBU-column blocking it replaced had its
// 32-B sectors written by the 4 column workgroups of a block: 1.65x U in WRITE_SIZE and K2 4.39 ->
// 4.17 ms at cfg2 on the same box (profiles/r05_experiments.txt).  U's rows are padded to a
// multiple of URT (u_rows).  Taller tiles give the column pass more of each line (2 x 8: K2 -8 %,
// 1 x 16: whole lines, K2 -8..-10 %) and cost the row pass more (K3 +33 %, +134 %:
// profiles/r06_experiments.txt 9), so 4 x 4 stays.
__host__ __device__ constexpr int u_rows(int rows) { return (rows + URT - 1) / URT * URT; }
__device__ __forceinline__ size_t blk_u(int c, int row, int rows) {
  return ((size_t)(c / CBU) * u_rows(rows) + (row & ~(URT - 1))) * CBU + (c % CBU) * URT + (row & (URT - 1));
}
// offset of row r from row 0 of the same column of U
__device__ __forceinline__ size_t u_roff(int r) { return (size_t)(r & ~(URT - 1)) * CBU + (r & (URT - 1)); }


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

// exp(i ph) for a phase in double, evaluated in double and rounded to fp32 once per component
// (error <= 6e-8 per component): the per-plane step factor of the column pass's plane recurrence,
// whose phase error accumulates over the planes of a chunk.  Quadrant reduction by a two-part pi/2,
// Taylor polynomials on [-pi/4, pi/4] (truncation < 5e-17).
__device__ __forceinline__ float2 cis_dd(double ph) {
  const double q = rint(ph * 0.63661977236758134308);
  double r = fma(-q, 1.5707963267948966192, ph);
  r = fma(-q, 6.1232339957367658e-17, r);
  const double r2 = r * r;
  // sin r = r + r^3 ps(r^2), ps = -1/3! + r^2/5! - r^4/7! + ... - r^12/15!
  double ps = -1.0 / 1307674368000.0;
  ps = fma(r2, ps, 1.0 / 6227020800.0);
  ps = fma(r2, ps, -1.0 / 39916800.0);
  ps = fma(r2, ps, 1.0 / 362880.0);
  ps = fma(r2, ps, -1.0 / 5040.0);
  ps = fma(r2, ps, 1.0 / 120.0);
  ps = fma(r2, ps, -1.0 / 6.0);
  const double s = fma(r * r2, ps, r);
  double pc = 1.0 / 20922789888000.0;  // 1/16!
  pc = fma(r2, pc, -1.0 / 87178291200.0);
  pc = fma(r2, pc, 1.0 / 479001600.0);
  pc = fma(r2, pc, -1.0 / 3628800.0);
  pc = fma(r2, pc, 1.0 / 40320.0);
  pc = fma(r2, pc, -1.0 / 720.0);
  pc = fma(r2, pc, 1.0 / 24.0);
  pc = fma(r2, pc, -0.5);
  const double c = fma(r2, pc, 1.0);
  const int iq = (int)q;
  double sn = (iq & 1) ? c : s;
  double cs = (iq & 1) ? s : c;
  if (iq & 2) sn = -sn;
  if ((iq + 1) & 2) cs = -cs;
  return make_float2((float)cs, (float)sn);
}

__device__ __forceinline__ int freq_index(int i, int n) { return i < n - n / 2 ? i : i - n; }

// Aperture masks (Components/Aperture.py:44-136): the aperture kernel and the ASM window mask
// (thz_asm_desc.window_mask) evaluate the same test.
struct ApertureArgs {
  int BC, H, W, kind;  // THZ_APERTURE_*
  float ax0, ax1, ay0, ay1;  // linspace end points of the two grid axes
  float half_w, half_h, radius;
};

__host__ __device__ inline ApertureArgs aperture_args(const thz_aperture_desc* d, int H, int W) {
  ApertureArgs a{};
  a.BC = d->BC; a.H = H; a.W = W; a.kind = d->kind;
  if (d->kind == THZ_APERTURE_RECT) {
    a.ax0 = (-d->dx * (float)W) / 2.0f;  // x over W with dx (Aperture.py:115)
    a.ax1 = (d->dx * (float)W) / 2.0f;
    a.ay0 = (-d->dy * (float)H) / 2.0f;  // y over H with dy (:116)
    a.ay1 = (d->dy * (float)H) / 2.0f;
  } else {
    a.ax0 = (-d->dx * (float)H) / 2.0f;  // x over H with dx (:76)
    a.ax1 = (d->dx * (float)H) / 2.0f;
    a.ay0 = (-d->dy * (float)W) / 2.0f;
    a.ay1 = (d->dy * (float)W) / 2.0f;
  }
  a.half_w = d->half_w;
  a.half_h = d->half_h;
  a.radius = d->radius;
  return a;
}

// RS kernel exp(ikr) z/(2 pi r^2) (1/r - ik) (Props/CZT_Prop.py:44-57).  The amplitude is
// fp32 in the reference's operation order; the phase k r (thousands of radians) is formed as
// (k|z| mod 2 pi, from double) + k rho^2 / (r + |z|) -- the exact identity r - |z| =
// rho^2/(r + |z|) keeps the fp32 part small, so the phase error drops from ~2e-4 rad (fp32
// k*r, which the reference pays and which costs it ~4e-3 rel-L2 on the test_czt.py case)
// to ~3e-5 rad.
struct RsPhase {
  float kzmod;  // (k |z|) mod 2 pi, k = 2 pi / lambda, evaluated in double
  float k;
};
__device__ __forceinline__ RsPhase rs_phase(float lam, float z) {
  const double k = 6.283185307179586476925 / (double)lam;
  double kz = k * fabs((double)z);
  kz -= 6.283185307179586476925 * floor(kz / 6.283185307179586476925);
  RsPhase p;
  p.kzmod = (float)kz;
  p.k = (float)k;
  return p;
}

#pragma clang fp contract(off)
__device__ __forceinline__ float2 rs_kernel(float x, float y, float z, float k, const RsPhase& ph) {
  const float rho2 = x * x + y * y;
  const float r = sqrtf(rho2 + z * z);
  const float f = 0.15915494309189535f * z / (r * r);
  const float fr = f * (1.0f / r), fi = -(f * k);
  float sn, cs;
  sincos_rad(ph.kzmod + ph.k * (rho2 / (r + fabsf(z))), &sn, &cs);
  return make_float2(cs * fr - sn * fi, cs * fi + sn * fr);
}

// sin/cos of an fp32 angle through the transcendental unit (v_sin_f32 / v_cos_f32 take
// revolutions): ang / 2 pi split exactly into t + e with a two-constant product, reduced to
// [-0.5, 0.5] revolutions.  Max abs error 1.8e-7 over |ang| <= 1000 rad against double
// (sincos_rad: 6e-8; scripts/diag/hw_sincos_check.hip), at about half the instructions.
__device__ __forceinline__ void sincos_hw(float ang, float* sn, float* cs) {
  const float C_HI = 0.15915494f;          // fp32(1 / 2 pi)
  const float C_LO = 6.4206383e-09f;       // 1 / 2 pi - C_HI
  const float t = ang * C_HI;
  const float e = __builtin_fmaf(ang, C_HI, -t) + ang * C_LO;
  const float r = (t - __builtin_rintf(t)) + e;
  *sn = __builtin_amdgcn_sinf(r);
  *cs = __builtin_amdgcn_cosf(r);
}

// The RS kernel of rs_kernel with the amplitude from the hardware rsqrt and the phase from a
// Newton-refined reciprocal and sincos_hw: about 25 instructions instead of three IEEE divisions,
// a square root and the polynomial sincos.  The phase k rho^2 / (r + |z|) (thousands of radians)
// keeps ~1 ulp, the fp32 floor of its representation; the amplitude carries a few ulp.  Used by
// the overlap-add CZT kernels, whose parity is measured against the fp64 oracle (1e-3 rel-L2).
__device__ __forceinline__ float2 rs_kernel_fast(float x, float y, float z, float k, const RsPhase& ph) {
  const float rho2 = x * x + y * y;
  const float r2 = rho2 + z * z;
  const float ir = __builtin_amdgcn_rsqf(r2);
  const float r = r2 * ir;
  const float f = (0.15915494309189535f * z) * (ir * ir);
  const float fr = f * ir, fi = -(f * k);
  const float d = r + fabsf(z);
  float rc = __builtin_amdgcn_rcpf(d);
  rc = __builtin_fmaf(rc, __builtin_fmaf(-d, rc, 1.0f), rc);
  float sn, cs;
  sincos_hw(ph.kzmod + ph.k * (rho2 * rc), &sn, &cs);
  return make_float2(cs * fr - sn * fi, cs * fi + sn * fr);
}

// torch.linspace(start, end, n)[i] in fp32 (symmetric two-sided form of ATen's CPU kernel)
// i < n/2: start + step i; else end - step (n - 1 - i), written as end + step (i - (n - 1)) -- the
// same IEEE operations (integers below 2^24 convert exactly) without a divergent branch
__device__ __forceinline__ float lin(float start, float end, int n, int i) {
  if (n == 1) return start;
  const float step = (end - start) / (float)(n - 1);
  const bool lo = i < n / 2;
  return (lo ? start : end) + step * (float)(lo ? i : i - (n - 1));
}

// pixel (i, j) of an H x W field open under the aperture (the reference's grids and fp32 tests)
__device__ __forceinline__ bool aperture_open(const ApertureArgs& a, int i, int j) {
  if (a.kind == THZ_APERTURE_RECT) {
    // meshgrid(x over W, y over H, indexing='xy'): X[i, j] = x[j], Y[i, j] = y[i]
    const float X = lin(a.ax0, a.ax1, a.W, j), Y = lin(a.ay0, a.ay1, a.H, i);
    return fabsf(X) <= a.half_w && fabsf(Y) <= a.half_h;
  }
  // circ: meshgrid(x over H, y over W) 'ij'
  const float X = lin(a.ax0, a.ax1, a.H, i), Y = lin(a.ay0, a.ay1, a.W, j);
  return sqrtf(X * X + Y * Y) <= a.radius;
}
#pragma clang fp contract(on)



// Two consecutive pixels per lane (16-byte loads and stores when HW is even, so every pair is
// aligned), one channel plane per blockIdx.y and a stride over the batch in blockIdx.z: the
// elementwise kernels stream B C HW complex values with the per-pixel factor evaluated once per
// (channel, pixel).  fac(p) gives the factor of pixel p (p < HW); out = in * factor.
constexpr int EW_THREADS = 256;
template <class Fac>
__device__ __forceinline__ void ew_scale_pairs(const float2* __restrict__ in, float2* __restrict__ out, int B, int C,
                                               int HW, Fac fac) {
  const int c = blockIdx.y;
  const int p0 = 2 * (blockIdx.x * EW_THREADS + (int)threadIdx.x);
  if (p0 >= HW) return;
  const bool two = p0 + 1 < HW;
  const float2 t0 = fac(p0), t1 = two ? fac(p0 + 1) : make_float2(0.f, 0.f);
  const bool vec = (HW & 1) == 0;
  // fields of 64 MB and more stream through the caches (read once, written once, and larger
  // than the L2s); smaller ones (the P = 300 layers' fields) stay cache-resident for their consumer
  const bool stream = (size_t)B * C * HW >= ((size_t)8 << 20);
  for (int b = blockIdx.z; b < B; b += gridDim.z) {
    const size_t i = ((size_t)b * C + c) * HW + p0;
    if (vec) {
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      if (stream) {
        const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in + i));
        const float2 r0 = cmul(make_float2(v.x, v.y), t0), r1 = cmul(make_float2(v.z, v.w), t1);
        __builtin_nontemporal_store(f32x4{r0.x, r0.y, r1.x, r1.y}, reinterpret_cast<f32x4*>(out + i));
        continue;
      }
      const float4 v = *reinterpret_cast<const float4*>(in + i);
      const float2 r0 = cmul(make_float2(v.x, v.y), t0), r1 = cmul(make_float2(v.z, v.w), t1);
      *reinterpret_cast<float4*>(out + i) = make_float4(r0.x, r0.y, r1.x, r1.y);
    } else {
      out[i] = cmul(in[i], t0);
      if (two) out[i + 1] = cmul(in[i + 1], t1);
    }
  }
}
inline dim3 ew_grid(int HW, int C, int B) {
  return dim3((unsigned)((HW + 2 * EW_THREADS - 1) / (2 * EW_THREADS)), (unsigned)C, (unsigned)(B < 16 ? B : 16));
}

// ---------------------------------------------------------------------------------------------
// DOE transmission (Components/QuantizedDOE.py:47-126), shared by the modulate kernels
// (thz_doe.hip) and the ASM row pass that applies it in its loader (thz_asm.hip, the fused
// DOE -> ASM step).  fp32 in the reference's operation order.
// ---------------------------------------------------------------------------------------------
constexpr float DOE_BASE_PLANE = 2e-3f;  // BASE_PLANE_THICKNESS (:23)

#pragma clang fp contract(off)
// nearest source index of torch.nn.functional.interpolate(mode='nearest'), fp32 scale (:102-107)
__device__ __forceinline__ int doe_nearest_src(int dst, int in, int out) {
  if (in == out) return dst;
  const float scale = (float)in / (float)out;
  return min((int)floorf((float)dst * scale), in - 1);
}

// Counter-based draws for graph-replayed training (the trainers' device_rng): every value is a
// hash of (seed, step, stream, index) -- stateless, so a forward and its backward regenerate the
// same draw, and each replay of a captured graph draws afresh from the step its host updates in
// the device state rng = [seed, step].  splitmix64 finalisation of the packed counter.
__device__ __forceinline__ unsigned long long rng_bits(const unsigned* rng, unsigned stream, unsigned idx) {
  unsigned long long x = ((unsigned long long)(rng[0] ^ (stream * 0x9E3779B9u)) << 32) | rng[1];
  x ^= (unsigned long long)idx * 0xD1B54A32D192ED03ull;
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// U[0, 1) with 24 random bits (torch.rand's support)
__device__ __forceinline__ float rng_u01(const unsigned* rng, unsigned stream, unsigned idx) {
  return (float)(unsigned)(rng_bits(rng, stream, idx) >> 40) * (1.0f / 16777216.0f);
}
// Exp(1) = -log(u), u = (b + 1) / 2^24 in (0, 1] (Tensor.exponential_).  The top bin (u = 1,
// probability 2^-24) would give E = 0 and a Gumbel draw -log(E) = +inf, which turns gumbel_softmax
// into NaN (a 6,000-iteration v3 / naive-Gumbel run draws ~10^7-10^8 values).  torch's CUDA
// transformation::exponential maps every u >= 1 - eps/2 to log = -eps/2, i.e. E = 2^-24 for fp32;
// the same floor here (u = 1 - 2^-24 already gives -logf(u) = 2^-24).
__device__ __forceinline__ float rng_exp1(const unsigned* rng, unsigned stream, unsigned idx) {
  const float e = -logf((float)((unsigned)(rng_bits(rng, stream, idx) >> 40) + 1u) * (1.0f / 16777216.0f));
  return fmaxf(e, 5.96046448e-8f);
}

// noisy height at a source pixel: h + (u - 0.5) * 2 * tol  (:85); u == nullptr: the device
// generator when rng is set, else no noise
__device__ __forceinline__ float doe_noisy_h(const float* h, const float* u, int idx, float tol,
                                             const unsigned* rng = nullptr, unsigned stream = 0) {
  float v = h[idx];
  if (u) v = v + ((u[idx] - 0.5f) * 2.0f) * tol;
  else if (rng) v = v + ((rng_u01(rng, stream, (unsigned)idx) - 0.5f) * 2.0f) * tol;
  return v;
}

// t_c(h) and gamma_c = dt/dh / t (:73-77)
__device__ __forceinline__ float2 doe_transmission(float hv, float lam, float eps, float tand, float2* gamma) {
  const float k = 6.283185307179586f / lam;
  const float hb = hv + DOE_BASE_PLANE;
  const float se = sqrtf(eps);
  const float ga = ((-0.5f * k) * tand) * se;  // d(log loss)/dh
  const float loss = expf(((-0.5f * k) * hb * tand) * se);
  const float gb = -k * (se - 1.0f);           // d(phase)/dh
  const float ph = (-k * hb) * (se - 1.0f);
  float sn, cs;
  sincos_rad(ph, &sn, &cs);
  if (gamma) *gamma = make_float2(ga, gb);
  return make_float2(loss * cs, loss * sn);
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------------------------
// |E|^2 -> normalize -> MSE as one-pass sums (experiment_four_focal_spots.ipynb:336-370,
// utils/Helper_Functions.py:185-193).  With m_b = max_i I_i of batch item b,
//   sum_i (I_i / m_b - T_i)^2 = S_II / m_b^2 - 2 S_IT / m_b + S_TT,
// so one pass accumulating S_II, S_IT, S_TT (fp64) and the max key per b replaces the two passes
// (max, then residuals) of a direct restatement.  The max key is (fp32 bits of I) << 32 |
// (0xffffffff - index): I >= 0 orders as its bits, ties go to the first index (torch.max).
// The backward statistic S_b = sum_i r_i I_i (r_i = I_i / m_b - T_i) is S_II / m_b - S_IT.
//
// Each producing workgroup stores its partial sums in its own slot (no atomics: a device-scope
// atomic per workgroup serialises a large batch on a few memory-side lines); loss_finish_kernel
// (thz_optics.hip) reduces the per_b slots of each b in a fixed order and the last of its
// workgroups sums the B terms, so the loss is bitwise reproducible.  Stats buffer layout
// (thz_intensity_mse_workspace_size): floats [0, 3B) = {m, argmax bits, S} per b; at byte 16 B:
// LossPart [B][per_b]; fp64 terms [B]; u64 finished-workgroup counter (zeroed by the producer).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float loss_intensity(float2 e) {
  const float m = hypotf(e.x, e.y);  // torch.abs(E) ** 2
  return m * m;
}

struct LossPart {
  double ii, it, tt;
  unsigned long long key;
};

struct LossAcc {
  double ii = 0.0, it = 0.0, tt = 0.0;
  unsigned long long key = 0ull;
  __device__ __forceinline__ void add(float2 v, float t, unsigned idx) {
    const float I = loss_intensity(v);
    const double di = I, dt = t;
    ii = fma(di, di, ii);
    it = fma(di, dt, it);
    tt = fma(dt, dt, tt);
    const unsigned long long k = ((unsigned long long)__float_as_uint(I) << 32) | (0xffffffffu - idx);
    key = k > key ? k : key;
  }
  __device__ __forceinline__ static LossAcc of(const LossPart& p) {
    LossAcc a;
    a.ii = p.ii;
    a.it = p.it;
    a.tt = p.tt;
    a.key = p.key;
    return a;
  }
  __device__ __forceinline__ LossPart part() const { return LossPart{ii, it, tt, key}; }
  __device__ __forceinline__ void merge(const LossAcc& o) {
    ii += o.ii;
    it += o.it;
    tt += o.tt;
    key = o.key > key ? o.key : key;
  }
};

struct LossSink {
  const float* target;        // [tB][tC][H][W]
  float* loss;                // [1]
  float* stats;               // [B][3] + the slots above
  int B, tB, tC;
  int per_b;                  // producer slots per batch item
  double inv_n;               // planes / (B C H W)
  __host__ __device__ static size_t part_offset(int B) { return 16 * (size_t)B; }  // bytes
  __host__ __device__ static size_t bytes(int B, int per_b) {
    return part_offset(B) + sizeof(LossPart) * (size_t)B * per_b + 8 * (size_t)B + 8;
  }
  __device__ LossPart* parts() const { return (LossPart*)((char*)stats + part_offset(B)); }
  __device__ double* terms() const { return (double*)(parts() + (size_t)B * per_b); }
  __device__ unsigned long long* counter() const { return (unsigned long long*)(terms() + B); }
};

// planes > 1: the loss items are Z planes x B (plane-major) and the loss is the sum of the planes'
// means (the multi-plane notebooks' summed MSEs)
inline LossSink loss_sink(const thz_loss_desc* d, const float* target, float* loss, float* stats, int per_b,
                          int planes = 1) {
  LossSink ls;
  ls.target = target;
  ls.loss = loss;
  ls.stats = stats;
  ls.B = d->B;
  ls.tB = d->tB;
  ls.tC = d->tC;
  ls.per_b = per_b;
  ls.inv_n = (double)planes / ((double)d->B * d->C * d->H * d->W);
  return ls;
}

// Workgroup reduction of the accumulators (fixed order), stored by thread 0 in slot (b, slot).
// Workgroup (0, 0) also zeroes the finish kernel's counter (it runs after this launch).
__device__ __forceinline__ void loss_store_part(LossAcc acc, const LossSink& ls, int b, int slot) {
  __shared__ LossPart s_a[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  for (int o = 32; o > 0; o >>= 1) {
    LossAcc t;
    t.ii = __shfl_xor(acc.ii, o);
    t.it = __shfl_xor(acc.it, o);
    t.tt = __shfl_xor(acc.tt, o);
    t.key = __shfl_xor(acc.key, o);
    acc.merge(t);
  }
  if (nw > 1) {
    __syncthreads();
    if (lane == 0) s_a[wid] = acc.part();
    __syncthreads();
    if (threadIdx.x == 0)
      for (int w = 1; w < nw; ++w) acc.merge(LossAcc::of(s_a[w]));
  }
  if (threadIdx.x == 0) {
    ls.parts()[(size_t)b * ls.per_b + slot] = LossPart{acc.ii, acc.it, acc.tt, acc.key};
    if (blockIdx.x == 0 && blockIdx.y == 0) *ls.counter() = 0ull;
  }
}

// loss_finish_kernel launch (thz_optics.hip): B workgroups
int launch_loss_finish(const LossSink& ls, hipStream_t s);

}  // namespace thz
