// Wave-level 1024-point Stockham FFT for gfx950: ONE wavefront (64 lanes x 16 values) owns a
// transform.  The two data exchanges go through a per-wave LDS image of floats (real parts, then
// imaginary parts), so a workgroup's waves never wait on each other: no workgroup barriers, only
// wave-scope ordering of the LDS accesses (a wave's LDS instructions execute in issue order; the
// fences keep the compiler from reordering them across lanes' data).
//
// Used by the overlap-add Bluestein kernels of the chirp-z propagator (thz_czt.hip): per line,
// several forward transforms of zero-padded half blocks (HALF_IN: inputs 512..1023 are zero) are
// accumulated in registers against filter spectra and finished by one inverse transform of which
// only the upper half of the outputs is kept.
//
// Forward schedule 16 (L=1), 16 (L=16), 4 (L=256): the result X[j], j = i + 256 q, sits in lane
// i % 64 as reg[i / 64][q] (i < 256, q < 4).  The inverse starts with radix 4 on exactly those
// registers, then 16 (L=4), 16 (L=64): output j = lane + 64 q, q < 16.
// Twiddles: per workgroup in LDS (shared by its waves), one table per read pattern so that every
// twiddle read of a 32-lane group is conflict-free (ds_read_b64, bank = dword mod 64; the model is
// scripts/wfft_bank_sim.py): w1024^t (t < 768: the forward's last stage reads k and 3k, odd strides),
// w1024^(2k) (k < 256), w256^(r k) as a 16 x 16 [r][k] table, w64^t, and the inverse's last stage
// w1024^(lane r) as a 15 x 64 [r - 1][lane] table (the flat w1024^(lane r) put 2 to 8 distinct
// slots on one bank for even r).
#pragma once
#include <hip/hip_runtime.h>

#include "thz_fft.hpp"

namespace thz {
namespace wf {

constexpr int N = 1024;
constexpr int LANES = 64;
constexpr int IMG = N + 2 * (N / 32);  // floats per wave image: pad2(1023) = 1023 + 2 * 31
constexpr int T1024 = 0, T512 = 768, T256 = 1024, T64 = 1280, TINV = 1344;
constexpr int TAB = TINV + 15 * 64;  // float2 twiddle entries per workgroup
struct Tabs {
  const float2* t1024;  // w1024^t, t < 768
  const float2* t512;   // w1024^(2 k), k < 256
  const float2* t256;   // [r][k] = w256^(r k)
  const float2* t64;    // w64^t
  const float2* tinv;   // [r - 1][lane] = w1024^(lane r)
};
// image padding, one per exchange (the write and the read of an exchange share it):
// pad1(j) = j + (j >> 5) for the first exchange of either transform, pad2(j) = j + 2 (j >> 5) for the
// second.  Every read pattern (x[lane + 64 r], x[lane + 64 m + 256 r]) walks 32 consecutive
// elements of one 32-aligned run, so any such pad keeps it conflict-free on the 32 banks of
// ds_read_b32; the writes need the slope: the forward's second exchange writes 16-element runs of
// two 256-apart groups (pad1 folds them 8 banks apart, a 2-way conflict on every write), the
// inverse's writes runs of 4 lanes 64 apart (pad2 spreads them over all 32 banks).
// (MI355X_MICROARCH.md §LDS; scripts/wfft_bank_sim.py)
__device__ __forceinline__ int pad(int j) { return j + (j >> 5); }
__device__ __forceinline__ int pad2(int j) { return j + 2 * (j >> 5); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the workgroup's twiddle tables (all threads; barrier before use): every entry is a root of the
// 1024-point plan table tw1024[t] = exp(-2 pi i t / 1024) (fp64-rounded on the host), gathered
// from L2 -- w1024^(2k) = tw1024[2 k], w256^e = tw1024[4 e], w64^e = tw1024[16 e]
__device__ __forceinline__ int tab_source(int t) {
  if (t < T512) return t;                                        // w1024^t
  if (t < T256) return 2 * (t - T512);                           // w1024^(2 k)
  if (t < T64) return 4 * ((t - T256) >> 4) * ((t - T256) & 15);  // [r][k] = w256^(r k)
  if (t < TINV) return 16 * (t - T64);                           // w64^t
  const int q = t - TINV;                                        // [r - 1][lane] = w1024^(lane r)
  return (q & 63) * ((q >> 6) + 1);
}
__device__ __forceinline__ Tabs fill_tables(float2* tab, const float2* __restrict__ tw1024, int tid, int nt) {
  for (int t = tid; t < TAB; t += nt) tab[t] = tw1024[tab_source(t)];
  return Tabs{tab + T1024, tab + T512, tab + T256, tab + T64, tab + TINV};
}
// The same fill by a workgroup of NT threads with every load issued before the first LDS write (the
// loop form waits out one L2 round trip per entry it writes)
template <int NT>
__device__ __forceinline__ Tabs fill_tables(float2* tab, const float2* __restrict__ tw1024, int tid) {
  constexpr int K = (TAB + NT - 1) / NT;
  float2 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int t = tid + k * NT;
    v[k] = t < TAB ? tw1024[tab_source(t)] : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int t = tid + k * NT;
    if (t < TAB) tab[t] = v[k];
  }
  return Tabs{tab + T1024, tab + T512, tab + T256, tab + T64, tab + TINV};
}

// This wave's float image behind the workgroup's tables.  Its offset is made opaque so the
// compiler keeps the (large, constant) image base in the address register: every exchange access
// is then that register plus a per-lane term and a small immediate, instead of one address add
// per access (the base alone exceeds the 8-bit dword offsets of ds_write2 / ds_read2).
__device__ __forceinline__ float* wave_image(float2* lds, int wave) {
  int off = 2 * TAB + wave * IMG;
  asm volatile("" : "+v"(off));
  return reinterpret_cast<float*>(lds) + off;
}

// Exchange: this lane's values v[a] go to the PADDED image position wpos(a); then
// nx[b] = image[rpos(b)] (padded too).  The callers write each padded position as a per-lane base
// plus a compile-time term (pad() distributes over the schedule's index forms for lane < 64), so
// every access is one address register and an immediate offset.
template <int NA, int NB, class WPos, class RPos>
__device__ __forceinline__ void exchange(float* img, const float2 (&v)[NA], WPos wpos, float2 (&nx)[NB], RPos rpos) {
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int a = 0; a < NA; ++a) img[wpos(a)] = part ? v[a].y : v[a].x;
    wave_sync();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float x = img[rpos(b)];
      if (part) nx[b].y = x;
      else nx[b].x = x;
    }
    wave_sync();
  }
}

// Forward transform of x[idx] = ld(idx) (HALF_IN: ld is only called for idx < N/2, the rest is
// zero).  Result: out(m * 4 + q, X[lane + 64 m + 256 q]) for m, q < 4.
template <bool HALF_IN, class Ld, class Out>
__device__ __forceinline__ void forward(float* img, const Tabs& tw, int lane, Ld& ld, Out& out) {
  float2 v[16];
  // stage 0: radix 16, L = 1, butterfly i = lane: inputs x[i + 64 r]
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = (!HALF_IN || r < 8) ? ld(lane + 64 * r) : make_float2(0.f, 0.f);
  dft16<false, HALF_IN>(v);
  float2 x1[16];
  // outputs y[16 i + q] -> stage 1 inputs x[i + 64 r]
  // pad(16 lane + q) = 16 lane + (lane >> 1) + q;  pad(lane + 64 r) = pad(lane) + 66 r
  const int pl = pad(lane), w0 = 16 * lane + (lane >> 1);
  exchange(img, v, [&](int q) { return w0 + q; }, x1, [&](int r) { return pl + 66 * r; });
  // stage 1: radix 16, L = 16, k = lane & 15: twiddle w256^(k r)
  const int k1 = lane & 15;
#pragma unroll
  for (int r = 1; r < 16; ++r) x1[r] = cmul(x1[r], tw.t256[16 * r + k1]);
  dft16<false>(x1);
  // outputs y[(i - k) 16 + k + 16 q] -> stage 2 inputs x[i2 + 256 r], i2 = lane + 64 m
  // pad2((lane - k) 16 + k + 16 q) = (lane - k) 16 + k + 16 (lane >> 4) + 16 q + 2 (q >> 1);
  // pad2(lane + 64 r) = pad2(lane) + 68 r
  float2 x2[16];
  const int w1 = (lane - k1) * 16 + k1 + 16 * (lane >> 4);
  const int pl2 = pad2(lane);
  exchange(img, x1, [&](int q) { return w1 + 16 * q + 2 * (q >> 1); }, x2,
           [&](int b) { return pl2 + 68 * ((b >> 2) + 4 * (b & 3)); });
  // stage 2: radix 4, L = 256, k = i2: twiddle w1024^(k r) (k and 3 k: odd strides; 2 k from its
  // own table)
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int k = lane + 64 * m;
    float2* q = &x2[4 * m];
    q[1] = cmul(q[1], tw.t1024[k]);
    q[2] = cmul(q[2], tw.t512[k]);
    q[3] = cmul(q[3], tw.t1024[3 * k]);
    dft4<false>(q[0], q[1], q[2], q[3]);
#pragma unroll
    for (int r = 0; r < 4; ++r) out(4 * m + r, q[r]);
  }
}

// Inverse (unnormalised) transform of the registers a forward() left: in[m * 4 + q] = X[lane + 64 m
// + 256 q].  sv(q, j, v) receives output j = lane + 64 q for q in [Q0, 16) only.
template <int Q0, class Sv>
__device__ __forceinline__ void inverse(float* img, const Tabs& tw, int lane, float2 (&in)[16], Sv& sv) {
  // stage 0: radix 4, L = 1, butterflies i = lane + 64 m: inputs x[i + 256 r] = in[4 m + r]
#pragma unroll
  for (int m = 0; m < 4; ++m) dft4<true>(in[4 * m], in[4 * m + 1], in[4 * m + 2], in[4 * m + 3]);
  // outputs y[4 i + q] -> stage 1 inputs x[lane + 64 r]
  // pad(4 (lane + 64 m) + q) = 4 lane + (lane >> 3) + 264 m + q;  pad(lane + 64 r) = pad(lane) + 66 r
  float2 x1[16];
  const int pl = pad(lane), w0 = 4 * lane + (lane >> 3);
  exchange(img, in, [&](int a) { return w0 + 264 * (a >> 2) + (a & 3); }, x1, [&](int r) { return pl + 66 * r; });
  // stage 1: radix 16, L = 4, k = lane & 3: conj twiddle w64^(k r)
  const int k1 = lane & 3;
#pragma unroll
  for (int r = 1; r < 16; ++r) x1[r] = cmulc(x1[r], tw.t64[k1 * r]);
  dft16<true>(x1);
  // outputs y[(i - k) 16 + k + 4 q] -> stage 2 inputs x[lane + 64 r]
  // pad2((lane - k) 16 + k + 4 q) = (lane - k) 16 + k + 4 (lane >> 2) + 4 q + 2 (q >> 3);
  // pad2(lane + 64 r) = pad2(lane) + 68 r
  float2 x2[16];
  const int w1 = (lane - k1) * 16 + k1 + 4 * (lane >> 2);
  const int pl2 = pad2(lane);
  exchange(img, x1, [&](int q) { return w1 + 4 * q + 2 * (q >> 3); }, x2, [&](int r) { return pl2 + 68 * r; });
  // stage 2: radix 16, L = 64, k = lane: conj twiddle w1024^(k r) from the [r - 1][lane] table;
  // outputs y[lane + 64 q]
#pragma unroll
  for (int r = 1; r < 16; ++r) x2[r] = cmulc(x2[r], tw.tinv[64 * (r - 1) + lane]);
  dft16<true>(x2);
#pragma unroll
  for (int q = Q0; q < 16; ++q) sv(q, lane + 64 * q, x2[q]);
}

}  // namespace wf
}  // namespace thz
