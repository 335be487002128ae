// LDS-resident mixed-radix Stockham FFT engine for gfx950 (CDNA4, wave64).
//
// One workgroup transforms one (or several) length-N complex rows held in LDS in
// natural order.  Radices 2/4/8/16 (and 3/5/7) run as in-register butterflies; any
// other factor (large primes such as 67, 101, 251 that the reference's
// P = N + 2*floor(s*N/2) padding produces) runs through a generic DFT stage that
// reads the twiddle table directly, so every length is supported.
//
// Stockham autosort, stage with current sub-transform length L and radix R:
//   butterfly i in [0, N/R), k = i mod L:
//     v_r = x[i + r*N/R] * w^(r*k),  w = exp(-+2 pi i /(L R))
//     y[(i-k)*R + k + q*L] = DFT_R(v)_q
// The twiddle table holds exp(-2 pi i t / N), t in [0, N), computed in double on
// the host (thz_plan.cpp) and read through L1/L2 (a few KiB, always cache-resident).
//
// LDS addressing pads one float2 every 16 (PADX) so power-of-two strides spread
// over the 64 LDS banks.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

namespace thz {

constexpr int FFT_MAX_STAGES = 24;
// Split-exchange row kernels of 8192 / 16384 points: the LDS image allows 8 waves / SIMD, so
// hold them to 64 VGPRs (the smaller sizes are LDS-limited below 8 and would only spill).
__host__ __device__ constexpr int row_waves_per_eu(int n) { return n >= 8192 ? 8 : 1; }
#define THZ_ROW_ATTR __attribute__((amdgpu_waves_per_eu(row_waves_per_eu(PN))))
constexpr int FFT_MAXV = 16;  // complex values held per thread per stage (N <= 16 * threads)
// Power-of-two path: 16 values (= the largest radix) per thread, T = N / 16 threads per transform.
// (8 values per thread measured slower on cfg2: one more LDS exchange costs more than the doubled
// occupancy hides)
__host__ __device__ constexpr int pow2_v(int) { return 16; }
constexpr int pow2_log(int v) { return v <= 1 ? 0 : 1 + pow2_log(v >> 1); }

struct FftPlan {
  int n;                       // transform length
  int nst;                     // number of stages
  int radix[FFT_MAX_STAGES];   // radix of each stage (product == n)
  const float2* tw;            // n roots exp(-2 pi i t / n)
};

__device__ __forceinline__ int padx(int a) { return a + (a >> 4); }
__host__ __device__ constexpr int lds_floats2(int n) { return n + (n >> 4) + 1; }

// Complex arithmetic on scalar fp32 (a packed v_pk_* form measured no faster: a packed op holds the
// SIMD for both halves, and its aligned register pairs push the column pass into spills).
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// The fused multiply-adds are written out: with a * b + c * d left to contraction, which product the
// compiler keeps rounded differs between instantiations of one transform (a window folded as a
// compile-time constant changed 10 % of the cfg2 outputs by an ulp), so every kernel that runs the
// same butterflies now rounds them the same way.
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  return make_float2(__builtin_fmaf(a.x, b.x, a.y * b.y), __builtin_fmaf(a.y, b.x, -(a.x * b.y)));
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 add_mfwd(float2 a, float2 d) { return make_float2(a.x + d.y, a.y - d.x); }
__device__ __forceinline__ float2 sub_mfwd(float2 a, float2 d) { return make_float2(a.x - d.y, a.y + d.x); }
// a * w (forward) or a * conj(w) (inverse): twiddles are stored and combined unconjugated
template <bool INV>
__device__ __forceinline__ float2 cmul_tw(float2 a, float2 w) { return INV ? cmulc(a, w) : cmul(a, w); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
  return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}
// a + m d and a - m d with m = -i (forward) or +i (inverse): one packed add each
template <bool INV>
__device__ __forceinline__ float2 add_mi(float2 a, float2 d) { return INV ? sub_mfwd(a, d) : add_mfwd(a, d); }
template <bool INV>
__device__ __forceinline__ float2 sub_mi(float2 a, float2 d) { return INV ? add_mfwd(a, d) : sub_mfwd(a, d); }

// ---------------------------------------------------------------------------------------------
// In-register DFTs: y_q = sum_r v_r exp(-+2 pi i r q / R)
// ---------------------------------------------------------------------------------------------
template <bool INV>
__device__ __forceinline__ void dft2(float2& a, float2& b) {
  float2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
  float2 t2 = cadd(a1, a3), d = csub(a1, a3);
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = add_mi<INV>(t1, d);
  a3 = sub_mi<INV>(t1, d);
}
// dft4 of (a0, a1, m a2, a3) with m = -i (forward) / +i (inverse): the twiddle of the radix-16
// element (2, 2) folded into the first butterfly
template <bool INV>
__device__ __forceinline__ void dft4_m2(float2& a0, float2& a1, float2& a2, float2& a3) {
  float2 t0 = add_mi<INV>(a0, a2), t1 = sub_mi<INV>(a0, a2);
  float2 t2 = cadd(a1, a3), d = csub(a1, a3);
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = add_mi<INV>(t1, d);
  a3 = sub_mi<INV>(t1, d);
}

template <bool INV>
__device__ __forceinline__ void dft8(float2* v) {
  // even/odd split: E = DFT4(v0,v2,v4,v6), O = DFT4(v1,v3,v5,v7)
  float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
  dft4<INV>(e0, e1, e2, e3);
  dft4<INV>(o0, o1, o2, o3);
  const float c = 0.70710678118654752440f;
  // w8^1 o1 = c (o1 + m o1), w8^3 o3 = -c (o3 - m o3), w8^2 o2 = m o2 (m = -+i)
  const float2 t1 = cscale(add_mi<INV>(o1, o1), c);
  const float2 t3 = cscale(sub_mi<INV>(o3, o3), -c);
  v[0] = cadd(e0, o0);
  v[4] = csub(e0, o0);
  v[1] = cadd(e1, t1);
  v[5] = csub(e1, t1);
  v[2] = add_mi<INV>(e2, o2);
  v[6] = sub_mi<INV>(e2, o2);
  v[3] = cadd(e3, t3);
  v[7] = csub(e3, t3);
}

// HALF_IN: inputs 8..15 are zero (a zero-padded half transform's first stage), so the first DFT4
// layer is two-input.
template <bool INV, bool HALF_IN = false>
__device__ __forceinline__ void dft16(float2* v) {
  // 16 = 4 x 4: B[r2][q1] = DFT4_{r1}(v[r2 + 4 r1]); B *= w16^(r2 q1); y[q1 + 4 q2] = DFT4_{r2}(B[.][q1])
  float2 b[4][4];
#pragma unroll
  for (int r2 = 0; r2 < 4; ++r2) {
    if constexpr (HALF_IN) {
      const float2 a0 = v[r2], a1 = v[r2 + 4];
      b[r2][0] = cadd(a0, a1);
      b[r2][2] = csub(a0, a1);
      b[r2][1] = add_mi<INV>(a0, a1);
      b[r2][3] = sub_mi<INV>(a0, a1);
    } else {
      b[r2][0] = v[r2];
      b[r2][1] = v[r2 + 4];
      b[r2][2] = v[r2 + 8];
      b[r2][3] = v[r2 + 12];
      dft4<INV>(b[r2][0], b[r2][1], b[r2][2], b[r2][3]);
    }
  }
  const float s = INV ? 1.f : -1.f;
  // w16^k = cos(2 pi k/16) + s i sin(2 pi k/16), k = r2*q1 in {1,2,3,4,6,9}
  const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
  const float c2 = 0.70710678118654752440f;
  // w16^2 = c2 (1 + m), w16^6 = -c2 (1 - m) with m = -+i; w16^4 = m (folded into dft4_m2)
  b[1][1] = cmul(b[1][1], make_float2(c1, s * s1));
  b[1][2] = cscale(add_mi<INV>(b[1][2], b[1][2]), c2);
  b[1][3] = cmul(b[1][3], make_float2(s1, s * c1));
  b[2][1] = cscale(add_mi<INV>(b[2][1], b[2][1]), c2);
  b[2][3] = cscale(sub_mi<INV>(b[2][3], b[2][3]), -c2);
  b[3][1] = cmul(b[3][1], make_float2(s1, s * c1));
  b[3][2] = cscale(sub_mi<INV>(b[3][2], b[3][2]), -c2);
  b[3][3] = cmul(b[3][3], make_float2(-c1, -s * s1));
#pragma unroll
  for (int q1 = 0; q1 < 4; ++q1) {
    float2 a0 = b[0][q1], a1 = b[1][q1], a2 = b[2][q1], a3 = b[3][q1];
    if (q1 == 2) dft4_m2<INV>(a0, a1, a2, a3);
    else dft4<INV>(a0, a1, a2, a3);
    v[q1] = a0;
    v[q1 + 4] = a1;
    v[q1 + 8] = a2;
    v[q1 + 12] = a3;
  }
}

template <bool INV>
__device__ __forceinline__ void dft3(float2* v) {
  const float c = -0.5f, s = (INV ? 1.f : -1.f) * 0.86602540378443864676f;
  float2 t = cadd(v[1], v[2]);
  float2 d = csub(v[1], v[2]);
  float2 m = make_float2(v[0].x + c * t.x, v[0].y + c * t.y);
  float2 js = make_float2(-s * d.y, s * d.x);  // i*s*d
  v[0] = cadd(v[0], t);
  v[1] = cadd(m, js);
  v[2] = csub(m, js);
}

template <bool INV>
__device__ __forceinline__ void dft5(float2* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float sg = INV ? 1.f : -1.f;
  const float s1 = sg * 0.95105651629515357212f, s2 = sg * 0.58778525229247312917f;
  float2 a = cadd(v[1], v[4]), b = csub(v[1], v[4]);
  float2 c = cadd(v[2], v[3]), d = csub(v[2], v[3]);
  float2 x0 = v[0];
  float2 m1 = make_float2(x0.x + c1 * a.x + c2 * c.x, x0.y + c1 * a.y + c2 * c.y);
  float2 m2 = make_float2(x0.x + c2 * a.x + c1 * c.x, x0.y + c2 * a.y + c1 * c.y);
  // n1 = i*(s1 b + s2 d), n2 = i*(s2 b - s1 d)
  float2 p1 = make_float2(s1 * b.x + s2 * d.x, s1 * b.y + s2 * d.y);
  float2 p2 = make_float2(s2 * b.x - s1 * d.x, s2 * b.y - s1 * d.y);
  float2 n1 = make_float2(-p1.y, p1.x), n2 = make_float2(-p2.y, p2.x);
  v[0] = make_float2(x0.x + a.x + c.x, x0.y + a.y + c.y);
  v[1] = cadd(m1, n1);
  v[4] = csub(m1, n1);
  v[2] = cadd(m2, n2);
  v[3] = csub(m2, n2);
}

template <bool INV>
__device__ __forceinline__ void dft7(float2* v) {
  const float sg = INV ? 1.f : -1.f;
  const float c1 = 0.62348980185873353053f, c2 = -0.22252093395631440429f, c3 = -0.90096886790241912624f;
  const float s1 = sg * 0.78183148246802980871f, s2 = sg * 0.97492791218182360702f,
              s3 = sg * 0.43388373911755812048f;
  float2 a1 = cadd(v[1], v[6]), b1 = csub(v[1], v[6]);
  float2 a2 = cadd(v[2], v[5]), b2 = csub(v[2], v[5]);
  float2 a3 = cadd(v[3], v[4]), b3 = csub(v[3], v[4]);
  float2 x0 = v[0];
  float2 m1 = make_float2(x0.x + c1 * a1.x + c2 * a2.x + c3 * a3.x, x0.y + c1 * a1.y + c2 * a2.y + c3 * a3.y);
  float2 m2 = make_float2(x0.x + c2 * a1.x + c3 * a2.x + c1 * a3.x, x0.y + c2 * a1.y + c3 * a2.y + c1 * a3.y);
  float2 m3 = make_float2(x0.x + c3 * a1.x + c1 * a2.x + c2 * a3.x, x0.y + c3 * a1.y + c1 * a2.y + c2 * a3.y);
  float2 p1 = make_float2(s1 * b1.x + s2 * b2.x + s3 * b3.x, s1 * b1.y + s2 * b2.y + s3 * b3.y);
  float2 p2 = make_float2(s2 * b1.x - s3 * b2.x - s1 * b3.x, s2 * b1.y - s3 * b2.y - s1 * b3.y);
  float2 p3 = make_float2(s3 * b1.x - s1 * b2.x + s2 * b3.x, s3 * b1.y - s1 * b2.y + s2 * b3.y);
  v[0] = make_float2(x0.x + a1.x + a2.x + a3.x, x0.y + a1.y + a2.y + a3.y);
  v[1] = make_float2(m1.x - p1.y, m1.y + p1.x);
  v[6] = make_float2(m1.x + p1.y, m1.y - p1.x);
  v[2] = make_float2(m2.x - p2.y, m2.y + p2.x);
  v[5] = make_float2(m2.x + p2.y, m2.y - p2.x);
  v[3] = make_float2(m3.x - p3.y, m3.y + p3.x);
  v[4] = make_float2(m3.x + p3.y, m3.y - p3.x);
}

template <int R, bool INV>
__device__ __forceinline__ void dftR(float2* v) {
  if constexpr (R == 2) dft2<INV>(v[0], v[1]);
  else if constexpr (R == 3) dft3<INV>(v);
  else if constexpr (R == 4) dft4<INV>(v[0], v[1], v[2], v[3]);
  else if constexpr (R == 5) dft5<INV>(v);
  else if constexpr (R == 7) dft7<INV>(v);
  else if constexpr (R == 8) dft8<INV>(v);
  else if constexpr (R == 16) dft16<INV>(v);
  else static_assert(R == 0, "no in-register DFT of this radix");
}

// ---------------------------------------------------------------------------------------------
// One Stockham stage with a register butterfly, in place in LDS (read all, barrier, write all)
// ---------------------------------------------------------------------------------------------
template <int R, bool INV>
__device__ __noinline__ void stage_reg(float2* lds, int n, int L, const float2* __restrict__ tw, int tid,
                                          int nthr) {
  constexpr int MAXB = (FFT_MAXV + R - 1) / R;
  const int nb = n / R;
  const int twstep = n / (L * R);
  float2 v[MAXB][R];
#pragma unroll
  for (int m = 0; m < MAXB; ++m) {
    const int i = tid + m * nthr;
    if (i < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[m][r] = lds[padx(i + r * nb)];
      if (L > 1) {
        const int k = i % L;
        const float2 w = tw[k * twstep];
        float2 wr = w;
#pragma unroll
        for (int r = 1; r < R; ++r) {
          v[m][r] = cmul_tw<INV>(v[m][r], wr);
          if (r + 1 < R) wr = cmul(wr, w);
        }
      }
      dftR<R, INV>(v[m]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MAXB; ++m) {
    const int i = tid + m * nthr;
    if (i < nb) {
      const int k = i % L;
      const int j = (i - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) lds[padx(j + r * L)] = v[m][r];
    }
  }
  __syncthreads();
}

// Generic-radix stage (any R): each thread computes FFT_MAXV outputs straight from the table.
template <bool INV>
__device__ __noinline__ void stage_generic(float2* lds, int n, int L, int R, const float2* __restrict__ tw,
                                           int tid, int nthr) {
  const int nb = n / R;
  const int LR = L * R;
  const int twstep = n / LR;
  float2 out[FFT_MAXV];
#pragma unroll
  for (int m = 0; m < FFT_MAXV; ++m) {
    const int o = tid + m * nthr;
    out[m] = make_float2(0.f, 0.f);
    if (o < n) {
      const int k = o % L;
      const int q = (o / L) % R;
      const int b = o / LR;
      const int i = b * L + k;
      const int e = k + q * L;  // exponent numerator over L*R
      float2 acc = make_float2(0.f, 0.f);
      int t = 0;                 // (r * e) mod LR
      for (int r = 0; r < R; ++r) {
        float2 w = tw[t * twstep];
        if (INV) w.y = -w.y;
        float2 x = lds[padx(i + r * nb)];
        acc.x += x.x * w.x - x.y * w.y;
        acc.y += x.x * w.y + x.y * w.x;
        t += e;
        if (t >= LR) t -= LR;
      }
      out[m] = acc;
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < FFT_MAXV; ++m) {
    const int o = tid + m * nthr;
    if (o < n) lds[padx(o)] = out[m];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Compile-time power-of-two path: N, the thread count T = N/FFT_MAXV and every stage's L
// and R are template constants, so index math is shifts/masks and loops fully unroll.
// Radix-16 stages first, then one 8/4/2 stage for the remainder.
// ---------------------------------------------------------------------------------------------
// Twiddles w^r, r = 1..R-1, of w = exp(-+2 pi i k / (L R)): powers of two straight from the
// table (independent loads), the rest by at most three dependent complex products.
//
// Twiddle sources: the global table (const float2*: L1/L2 loads, vmcnt waits) or a two-level
// copy in LDS (TwLds: w^t = A[t mod 64] * B[t / 64], 64 + N/64 entries, ds_reads that never
// wait behind the kernel's outstanding global stores).
struct TwLds {
  const float2* t;     // t[a] = w^a (a < 64), t[64 + b] = w^(64 b), w = exp(-2 pi i / N)
  // every twiddle of the L R = 256 stage as a 16 x 16 table, t256[16 r + k] = exp(-2 pi i r k / 256):
  // the 16 butterflies k of a half-wave read 16 consecutive slots for each r (conflict-free; the
  // flat table t[r k] put 2 to 4 distinct slots on one bank for r = 4, 8, 12)
  const float2* t256;
};
__device__ __forceinline__ float2 twat(const float2* __restrict__ p, int i) { return p[i]; }
__device__ __forceinline__ float2 twat(const TwLds& s, int i) { return cmul(s.t[i & 63], s.t[64 + (i >> 6)]); }

// LDS slots of the twiddle tables of a length-n transform (placed after the data rows)
__host__ __device__ constexpr int tw_lds_count(int n) { return n >= 1024 ? 64 + n / 64 + 256 : 0; }

// Fill the tables (visible after the first stage's barrier): a gather of 64 + N/64 + 256 entries
// of the plan's global table (tw[t] = w^t, L2-resident), issued ahead of the data loads.
template <int N>
__device__ __forceinline__ TwLds load_tw_lds(float2* dst, const float2* __restrict__ tw, int tid, int nt) {
  constexpr int N2 = 64 + N / 64;
  for (int i = tid; i < tw_lds_count(N); i += nt) {
    const int q = i - N2;
    const int t = i < 64 ? i : (i < N2 ? (i - 64) * 64 : (q >> 4) * (q & 15) * (N / 256));
    dst[i] = tw[t];
  }
  return TwLds{dst, dst + N2};
}

// The same fill in two halves, so the table's global loads can be issued ahead of a kernel's data
// loads and written to LDS after them (tw_fetch -> data loads -> tw_store, before the first barrier
// that precedes a twiddle read): NT threads, each fetching ceil(count / NT) entries into registers.
template <int N, int NT>
struct TwFetch {
  static constexpr int K = (tw_lds_count(N) + NT - 1) / NT;
  float2 v[K];
};
template <int N, int NT>
__device__ __forceinline__ TwFetch<N, NT> tw_fetch(const float2* __restrict__ tw, int tid) {
  constexpr int N2 = 64 + N / 64;
  TwFetch<N, NT> f;
#pragma unroll
  for (int k = 0; k < TwFetch<N, NT>::K; ++k) {
    const int i = tid + k * NT;
    const int q = i - N2;
    const int t = i < 64 ? i : (i < N2 ? (i - 64) * 64 : (q >> 4) * (q & 15) * (N / 256));
    f.v[k] = i < tw_lds_count(N) ? tw[t] : make_float2(0.f, 0.f);
  }
  return f;
}
template <int N, int NT>
__device__ __forceinline__ void tw_store(float2* dst, const TwFetch<N, NT>& f, int tid) {
#pragma unroll
  for (int k = 0; k < TwFetch<N, NT>::K; ++k) {
    const int i = tid + k * NT;
    if (i < tw_lds_count(N)) dst[i] = f.v[k];
  }
}
template <int N>
__device__ __forceinline__ TwLds tw_lds_at(float2* dst) {
  return TwLds{dst, dst + 64 + N / 64};
}

template <int R, class Tw>
__device__ __forceinline__ void twiddle_powers(const Tw& tw, int kt, float2* w) {
  // w[r] for r = 1..R-1 (forward sign; the inverse applies them conjugated, cmul_tw);
  // kt = k * (N / (L R)) is the table index of w^1
  w[1] = twat(tw, kt);
  if constexpr (R >= 4) w[2] = twat(tw, 2 * kt);
  if constexpr (R >= 8) w[4] = twat(tw, 4 * kt);
  if constexpr (R >= 16) w[8] = twat(tw, 8 * kt);
  if constexpr (R >= 4) w[3] = cmul(w[1], w[2]);
  if constexpr (R >= 8) {
    w[5] = cmul(w[1], w[4]);
    w[6] = cmul(w[2], w[4]);
    w[7] = cmul(w[3], w[4]);
  }
  if constexpr (R >= 16) {
#pragma unroll
    for (int r = 9; r < 16; ++r) w[r] = cmul(w[r - 8], w[8]);
  }
}

// One compile-time stage with pluggable input and output.
//   IN_LDS : read x[i + r*NB] from LDS (base padx(i) + constant offsets); else ld(m, r, idx)
//   OUT_LDS: write y[j + r*L] to LDS (in place: barrier, write, barrier); else sv(m, r, idx, v)
// For power-of-two N >= 256 every LDS access is base + compile-time offset:
//   padx(i + r NB) = padx(i) + r NB + (r NB >> 4)       (NB % 16 == 0)
//   padx(j + r L)  = padx(j) + r L  + (r L >> 4)        (L | 16 or 16 | L, L R >= 16 or L == 1)
// Complex-image layouts per exchange (keyed by the writing stage's L): element j at float2
// j + C (j >> SH).  L == 1 keeps padx (the natural-order image fft_pow2's callers read and
// write); 1 < L < 16 uses (4 + log2 L, L); L >= 16 needs no padding.  Bank model of ds_read_b64
// (2 x 32 lanes, dword mod 64) and ds_write_b64 (4 x 16 lanes, dword mod 32): 1.33x the ideal
// LDS cycles on the L == 1 exchange, conflict-free on the others (scripts/lds_bank_sim.py
// layouts64), against 1.33x on every exchange for padx everywhere.
__host__ __device__ constexpr int c64_sh(int L) { return L == 1 ? 4 : (L < 16 ? 4 + pow2_log(L) : 0); }
__host__ __device__ constexpr int c64_c(int L) { return L == 1 ? 1 : (L < 16 ? L : 0); }
template <int L>
__host__ __device__ constexpr int c64_lay(int j) { return j + c64_c(L) * (j >> c64_sh(L)); }

// Butterfly order of a stage that reads the natural-order (padx) image: each 32-lane half reads
// x[i + r NB] for 32 butterflies, which under padx land on float2 slots i + (i >> 4): 32
// consecutive i put slot 0 and slot 32 of the run on one bank (2-way on every read).  Swapping
// bits 4 and 8 of the thread index gives each half the runs [16b, 16b + 16) and
// [16b + 256, 16b + 272), whose padded slots 17b + l and 17b + 272 + l cover the 64 banks once
// (17 * 16 = 272 = 16 mod 32).  Any butterfly order is valid for a stage whose results go back
// to LDS; the twiddle index i mod L is unchanged (L <= 16 in these stages).
template <int LIN, int T, int NB, bool OUT_LDS>
__device__ __forceinline__ int stage_order(int tid) {
  if constexpr (LIN == 1 && OUT_LDS && T % 512 == 0 && NB % 512 == 0)
    return (tid & ~0x110) | ((tid & 0x10) << 4) | ((tid & 0x100) >> 4);
  else
    return tid;
}

template <int R, bool INV, int N, int L, int T, bool IN_LDS, bool OUT_LDS, int LIN = 1, int LOUT = L, class Tw,
          class Ld, class Sv>
__device__ __forceinline__ void stage_x(float2* lds, const Tw& tw, int tid, Ld& ld, Sv& sv) {
  constexpr int NB = N / R;
  constexpr int MB = NB / T;  // butterflies per thread (exact)
  static_assert(MB * T == NB, "pow2 plan must tile exactly");
  static_assert(NB % 16 == 0, "constant-offset LDS addressing");
  constexpr int TWS = N / (L * R);
  const int bo = IN_LDS ? stage_order<LIN, T, NB, OUT_LDS>(tid) : tid;
  float2 v[MB][R];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int i = bo + m * T;
    if constexpr (IN_LDS) {
      const float2* src = lds + c64_lay<LIN>(i);
#pragma unroll
      for (int r = 0; r < R; ++r) v[m][r] = src[c64_lay<LIN>(m * T + r * NB) - c64_lay<LIN>(m * T)];
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) v[m][r] = ld(m, r, i + r * NB);
    }
    if constexpr (L > 1) {
      float2 w[R];
      if constexpr (L * R == 256 && std::is_same<Tw, TwLds>::value) {
        // w^r = exp(-2 pi i k r / 256): straight LDS reads of the 16 x 16 table, no products
        static_assert(L == 16, "the L R = 256 stage of a radix-16 schedule");
        const int k = i & (L - 1);
#pragma unroll
        for (int r = 1; r < R; ++r) w[r] = tw.t256[16 * r + k];
      } else {
        twiddle_powers<R>(tw, (i & (L - 1)) * TWS, w);
      }
#pragma unroll
      for (int r = 1; r < R; ++r) v[m][r] = cmul_tw<INV>(v[m][r], w[r]);
    }
    dftR<R, INV>(v[m]);
  }
  if constexpr (OUT_LDS) {
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int i = bo + m * T;
      const int k = i & (L - 1);
      const int i0 = m * T, k0 = i0 & (L - 1), j0 = (i0 - k0) * R + k0;  // thread 0: folds after unrolling
      float2* dst = lds + c64_lay<LOUT>((i - k) * R + k);
#pragma unroll
      for (int r = 0; r < R; ++r) dst[c64_lay<LOUT>(j0 + r * L) - c64_lay<LOUT>(j0)] = v[m][r];
    }
    __syncthreads();
  } else {
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int i = bo + m * T;
      const int k = L * R == N ? i : i & (L - 1);  // last stage: i < N / R = L
      const int j = (i - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) sv(m, r, j + r * L, v[m][r]);
    }
  }
}

// Radix schedule of a power-of-two N: 16s plus one remainder radix b in {2,4,8} (or none).
// MODE 0: remainder last; 1: remainder first; 2 (FFT_TAIL): a radix-2 remainder merged with the
// last radix-16 stage into one radix-32 stage on lane pairs (stage_r32_pair_last) -- one LDS
// exchange and its barriers fewer; other remainders as MODE 0.  (The register hand-off between
// a MODE-0 forward and a MODE-1 inverse, as in the CZT kernels, needs MODE 0 / 1.)
// Measured on cfg2 (8192 points): the column pass (complex image, 4 waves/SIMD) runs 2.69 -> 2.32
// ms per 32 planes with the pair tail (MODE 2).  The 64-VGPR split-image row passes do not gain
// from either lane-pair form: the tail spills at 64 VGPRs (K3 2.19 -> 2.62 ms); the head (MODE 3,
// one LDS exchange fewer, no input twiddles) leaves a full radix-16 last stage whose twiddles and
// cropped stores spill at 64 VGPRs (3.31 ms) and run 2.32 ms at 7 waves/SIMD without spills --
// so the row passes are not LDS-exchange-bound and keep MODE 0 (FFT_ROWS).  fft_rows_kernel
// (diagnostics) runs MODE 2 forward and MODE 3 inverse so both split-image forms stay tested.
// The column pass's inverse uses MODE 2; the row passes MODE 0 (measured above).
constexpr int FFT_TAIL = 2;
constexpr int FFT_ROWS = 0;
template <int N>
struct Pow2Sched {
  static constexpr int log2n() {
    int l = 0;
    while ((1 << l) < N) ++l;
    return l;
  }
  static constexpr int LOG = log2n();
  static constexpr int V = pow2_v(N);
  static constexpr int LV = pow2_log(V);
  static constexpr int NS16 = LOG / LV;  // full-radix (V) stages
  static constexpr int REM = 1 << (LOG % LV);
  static constexpr int NST = NS16 + (REM > 1 ? 1 : 0);
  static constexpr bool PAIR = REM == 2 && V == 16 && NS16 >= 2;
  static constexpr int nst(int mode) { return mode >= 2 && PAIR ? NS16 : NST; }
  static constexpr int radix(int s, int mode) {
    if (REM == 1) return V;
    if (mode == 1) return s == 0 ? REM : V;
    if (mode == 2 && PAIR) return s == NS16 - 1 ? 32 : V;
    if (mode == 3 && PAIR) return s == 0 ? 32 : V;
    return s == NST - 1 ? REM : V;
  }
};

// ---------------------------------------------------------------------------------------------
// Radix-32 last stage on lane pairs (MODE 2; L = N/32 butterflies, k = i, L R = N).  Butterfly i
// runs on lanes l and l + 32 of one wave (i = 32 wave + l mod 32, e = l / 32); lane e holds the
// inputs x_{2s+e}, s < 16, and forms A_e = w^{e i} DFT16_s(x_{2s+e} w^{2 s i}).  Then
// X_q = A_0[q] + w32^q A_1[q] and X_{q+16} = A_0[q] - w32^q A_1[q]: one v_permlane32_swap per
// dword pairs (A_0[q], A_1[q]) for even q in the low half-wave and for odd q in the high half,
// and each lane finishes 8 radix-2 butterflies -- no LDS exchange and no barrier for the
// radix-2 step.  Reads of this stage (x[i + (2s+e) L]) are conflict-free on the L = N/512
// exchange images: every 32-lane group shares e and covers 32 consecutive i.
// ---------------------------------------------------------------------------------------------
__host__ __device__ constexpr int pair_i(int tid) { return ((tid >> 6) << 5) | (tid & 31); }

__device__ __forceinline__ void swap_halves(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(b), false, false);
  a = __int_as_float(r[0]);
  b = __int_as_float(r[1]);
}

template <bool INV, int N, class Tw, class Sv>
__device__ __forceinline__ void stage_r32_pair_last(const Tw& tw, int tid, float2 (&x)[16], Sv& sv) {
  constexpr int L = N / 32;
  // exp(-2 pi i q / 32) = (C32C[q], -C32S[q]), q < 16
  constexpr float C32C[16] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                              0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                              0.19509032201612826785f, 0.0f, -0.19509032201612826785f, -0.38268343236508977173f,
                              -0.55557023301960222474f, -0.70710678118654752440f, -0.83146961230254523708f,
                              -0.92387953251128675613f, -0.98078528040323044913f};
  constexpr float C32S[16] = {0.0f, 0.19509032201612826785f, 0.38268343236508977173f, 0.55557023301960222474f,
                              0.70710678118654752440f, 0.83146961230254523708f, 0.92387953251128675613f,
                              0.98078528040323044913f, 1.0f, 0.98078528040323044913f, 0.92387953251128675613f,
                              0.83146961230254523708f, 0.70710678118654752440f, 0.55557023301960222474f,
                              0.38268343236508977173f, 0.19509032201612826785f};
  const int e = (tid >> 5) & 1, i = pair_i(tid);
  {
    // w^{2 i s}: the powers 1, 2, 4, 8 from the table, the rest by the products of
    // twiddle_powers, each formed next to its use (short live ranges: the row kernels run at 64
    // VGPRs)
    const float2 w1 = twat(tw, 2 * i), w2 = twat(tw, 4 * i), w4 = twat(tw, 8 * i), w8 = twat(tw, 16 * i);
    const float2 w3 = cmul(w1, w2), w5 = cmul(w1, w4), w6 = cmul(w2, w4), w7 = cmul(w3, w4);
    x[1] = cmul_tw<INV>(x[1], w1);
    x[2] = cmul_tw<INV>(x[2], w2);
    x[3] = cmul_tw<INV>(x[3], w3);
    x[4] = cmul_tw<INV>(x[4], w4);
    x[5] = cmul_tw<INV>(x[5], w5);
    x[6] = cmul_tw<INV>(x[6], w6);
    x[7] = cmul_tw<INV>(x[7], w7);
    x[8] = cmul_tw<INV>(x[8], w8);
    x[9] = cmul_tw<INV>(x[9], cmul(w1, w8));
    x[10] = cmul_tw<INV>(x[10], cmul(w2, w8));
    x[11] = cmul_tw<INV>(x[11], cmul(w3, w8));
    x[12] = cmul_tw<INV>(x[12], cmul(w4, w8));
    x[13] = cmul_tw<INV>(x[13], cmul(w5, w8));
    x[14] = cmul_tw<INV>(x[14], cmul(w6, w8));
    x[15] = cmul_tw<INV>(x[15], cmul(w7, w8));
  }
  dftR<16, INV>(x);
  // The odd lane's common input factor w^{i} is left out above and applied after the swap
  // (linearity).  The swap pairs registers (2p, 2p + 1): the low half-wave then holds
  // (A_0[q], A_1[q]) for q = 2p and the high half for q = 2p + 1, so a lane's outputs
  // q + 16 e' (e' = 0, 1) sit at the same place relative to a centred crop in both halves and
  // every store of a cropped row is all-lanes or none.
  const float2 wi = twat(tw, i);
  const float2 f = e ? cmul(wi, make_float2(C32C[1], -C32S[1])) : wi;  // w^i w32^e
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    float2 a = x[2 * p], b = x[2 * p + 1];
    swap_halves(a.x, b.x);
    swap_halves(a.y, b.y);
    // now (a, w^i b) = (A_0[q], A_1[q]), q = 2p + e;  w32^q = w32^{2p} w32^e
    const float2 t = cmul_tw<INV>(b, p == 0 ? f : cmul(f, make_float2(C32C[2 * p], -C32S[2 * p])));
    const int q = 2 * p + e;
    sv(0, 2 * p, i + q * L, cadd(a, t));
    sv(0, 2 * p + 16, i + (q + 16) * L, csub(a, t));
    // keep each p's swap / multiply next to its (predicated) stores: hoisting them all above
    // the first store region spills the 64-VGPR row kernels
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Radix-32 FIRST stage on lane pairs (MODE 3; L = 1), decimation in frequency.  Lane e of
// butterfly i loads x_r, r = 16 e + r' (r' < 16), from x[i + r N/32].  One v_permlane32_swap per
// dword pairs (x_r, x_{r+16}) for even r in the low half-wave and odd r in the high half; each
// lane forms y_r = x_r + x_{r+16} and z_r = (x_r - x_{r+16}) w32^r; a second swap gathers every
// y in the low half and every z in the high half, and one DFT16 per lane gives
// v[k] = X_{2k+e} (X_{2k} = DFT16(y)_k, X_{2k+1} = DFT16(z)_k).  No input twiddles (L = 1).
template <bool INV, int N, class In>
__device__ __forceinline__ void stage_r32_pair_first(int tid, In& in, float2 (&v)[16]) {
  constexpr int LP = N / 32;
  // w32^{2p} = exp(-2 pi i p / 16), p < 8
  constexpr float C16C[8] = {1.0f, 0.92387953251128675613f, 0.70710678118654752440f, 0.38268343236508977173f,
                             0.0f, -0.38268343236508977173f, -0.70710678118654752440f, -0.92387953251128675613f};
  constexpr float C16S[8] = {0.0f, 0.38268343236508977173f, 0.70710678118654752440f, 0.92387953251128675613f,
                             1.0f, 0.92387953251128675613f, 0.70710678118654752440f, 0.38268343236508977173f};
  const int e = (tid >> 5) & 1, i = pair_i(tid);
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = in(0, r, i + (16 * e + r) * LP);
  // w32^e
  const float2 f1 = e ? make_float2(0.98078528040323044913f, -0.19509032201612826785f) : make_float2(1.f, 0.f);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    float2 a = v[2 * p], b = v[2 * p + 1];
    swap_halves(a.x, b.x);
    swap_halves(a.y, b.y);
    // (a, b) = (x_r, x_{r+16}), r = 2p + e;  w32^r = w32^{2p} w32^e
    const float2 y = cadd(a, b);
    const float2 z = cmul_tw<INV>(csub(a, b), p == 0 ? f1 : cmul(f1, make_float2(C16C[p], -C16S[p])));
    float2 lo = y, hi = z;
    swap_halves(lo.x, hi.x);
    swap_halves(lo.y, hi.y);
    v[2 * p] = lo;      // low half: y_{2p}, high half: z_{2p}
    v[2 * p + 1] = hi;  // low half: y_{2p+1}, high half: z_{2p+1}
  }
  dftR<16, INV>(v);
}

// The pair stage reads x[i + (2s+e) L] at base lay(i + e L) plus lay(2 s L) - lay(0): true for
// the layouts used when the per-lane part of the index never carries into the padded bits.
template <class F>
__host__ __device__ constexpr bool pair_offsets_ok(F lay, int N) {
  const int L = N / 32;
  for (int e = 0; e < 2; ++e)
    for (int i = 0; i < L; i += L - 1)
      for (int s = 0; s < 16; ++s)
        if (lay(i + e * L + 2 * s * L) - lay(i + e * L) != lay(2 * s * L) - lay(0)) return false;
  return true;
}

struct NoIO {
  __device__ float2 operator()(int, int, int) const { return make_float2(0.f, 0.f); }
  __device__ void operator()(int, int, int, float2) const {}
};

// Stages S .. NST-1 of a power-of-two transform.  Stage 0 reads through ld unless
// FIRST_LDS; the final stage writes through sv unless LAST_LDS.
template <bool INV, int N, int T, int MODE, bool FIRST_LDS, bool LAST_LDS, int S = 0, int L = 1, class Tw, class Ld,
          class Sv>
__device__ __forceinline__ void fft_pow2_io(float2* lds, const Tw& tw, int tid, Ld& ld, Sv& sv) {
  using P = Pow2Sched<N>;
  constexpr int NS = P::nst(MODE);
  if constexpr (S < NS) {
    constexpr int R = P::radix(S, MODE);
    constexpr bool IN_LDS = S > 0 || FIRST_LDS;
    constexpr bool OUT_LDS = S < NS - 1 || LAST_LDS;
    // image layouts: the previous stage's (L / its radix); natural-order padx at the two ends
    constexpr int LIN = S == 0 ? 1 : L / P::radix(S - 1, MODE);
    constexpr int LOUT = S == NS - 1 ? 1 : L;
    if constexpr (R == 32) {
      static_assert(S > 0 && S == NS - 1 && !LAST_LDS && T == N / 16, "pair stage: last, reading LDS");
      static_assert(pair_offsets_ok([](int j) { return c64_lay<LIN>(j); }, N), "pair-stage offsets");
      constexpr int LP = N / 32;
      const int e = (tid >> 5) & 1;
      const float2* src = lds + c64_lay<LIN>(pair_i(tid) + e * LP);
      float2 x[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) x[s] = src[c64_lay<LIN>(2 * s * LP) - c64_lay<LIN>(0)];
      stage_r32_pair_last<INV, N>(tw, tid, x, sv);
    } else {
      stage_x<R, INV, N, L, T, IN_LDS, OUT_LDS, LIN, LOUT>(lds, tw, tid, ld, sv);
      fft_pow2_io<INV, N, T, MODE, FIRST_LDS, LAST_LDS, S + 1, L * R>(lds, tw, tid, ld, sv);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Split-exchange form of the power-of-two transform.  The LDS image holds ONE float per
// element; each Stockham exchange moves the real parts, then the imaginary parts (four
// barriers instead of two).  The data image is half the size (N floats + padding), so twice as
// many workgroups fit on a CU -- for a latency-bound row pass that is the larger effect.
// Stage 0 reads through ld(m, r, idx), the last stage writes through sv(m, r, idx, v); every
// stage keeps its butterflies' operands in registers (the exchange lands them there directly).
__host__ __device__ constexpr int lds_split_f2(int n) { return (lds_floats2(n) + 1) / 2; }

template <int R, bool INV, int N, int L, int T, class Tw, class In>
__device__ __forceinline__ void stage_core(const Tw& tw, int tid, In& in, float2 (&v)[N / R / T][R]) {
  constexpr int NB = N / R;
  constexpr int MB = NB / T;
  static_assert(MB * T == NB, "pow2 plan must tile exactly");
  constexpr int TWS = N / (L * R);
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int i = tid + m * T;
#pragma unroll
    for (int r = 0; r < R; ++r) v[m][r] = in(m, r, i + r * NB);
    if constexpr (L > 1) {
      float2 w[R];
      if constexpr (L * R == 256 && std::is_same<Tw, TwLds>::value) {
        static_assert(L == 16, "the L R = 256 stage of a radix-16 schedule");
        const int k = i & (L - 1);
#pragma unroll
        for (int r = 1; r < R; ++r) w[r] = tw.t256[16 * r + k];
      } else {
        twiddle_powers<R>(tw, (i & (L - 1)) * TWS, w);
      }
#pragma unroll
      for (int r = 1; r < R; ++r) v[m][r] = cmul_tw<INV>(v[m][r], w[r]);
    }
    dftR<R, INV>(v[m]);
  }
}

// LDS layout of one split exchange: element j lives at float j + C (j >> SH).  Chosen per
// exchange (by the writing stage's L) so that its write pattern (j = (i - k) R + k + r L) and the
// next stage's read pattern (i + r N/R2) are both free of bank conflicts under the ds_read_b32 /
// ds_write_b32 banking (two 32-lane groups, bank = dword mod 32; MI355X_MICROARCH.md §LDS), and
// the r-offsets stay compile-time constants.  Found by search (scripts/lds_bank_sim.py layouts)
// for every power-of-two size and both schedules; all fit in N + N/16 floats.  The fixed
// j + (j >> 4) it replaces costs 67 % extra LDS cycles on the 8192-point schedule.
__host__ __device__ constexpr int split_sh(int L) { return L == 1 ? 5 : (L <= 16 ? 4 + pow2_log(L) : 11); }
__host__ __device__ constexpr int split_c(int L) { return L == 1 ? 1 : (L <= 16 ? L : 1); }
template <int L>
__host__ __device__ constexpr int split_lay(int j) { return j + split_c(L) * (j >> split_sh(L)); }

struct NoHook {
  __device__ void operator()() const {}
};
template <bool INV, int N, int T, int MODE, int S = 0, int L = 1, class Tw, class In, class Sv, class Hook = NoHook>
__device__ __forceinline__ void fft_pow2_split_io(float* lds, const Tw& tw, int tid, In& in, Sv& sv,
                                                  Hook hook = Hook{}) {
  using P = Pow2Sched<N>;
  constexpr int R = P::radix(S, MODE);
  if constexpr (R == 32 && S == 0) {
    // lane-pair radix-32 first stage (MODE 3), then the exchange into the L = 32 stage: lane
    // (i, e) holds X_{2k+e}, Stockham output j = 32 i + 2k + e (conflict-free on split_lay<1>:
    // 32 consecutive i per lane group)
    static_assert(T == N / 16 && P::radix(1, MODE) == 16 && P::nst(MODE) >= 2, "pair-first layout");
    constexpr int NB2 = N / 16;
    constexpr int MB2 = NB2 / T;
    float2 v1[16];
    stage_r32_pair_first<INV, N>(tid, in, v1);
    hook();
    float2 nx[MB2][16];
    float* dst = lds + split_lay<1>(32 * pair_i(tid) + ((tid >> 5) & 1));
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k) dst[split_lay<1>(2 * k) - split_lay<1>(0)] = part ? v1[k].y : v1[k].x;
      __syncthreads();
#pragma unroll
      for (int m = 0; m < MB2; ++m) {
        const float* src = lds + split_lay<1>(tid + m * T);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float x = src[split_lay<1>(m * T + r * NB2) - split_lay<1>(m * T)];
          if (part) nx[m][r].y = x;
          else nx[m][r].x = x;
        }
      }
    }
    auto in2 = [&](int m, int r, int) { return nx[m][r]; };
    fft_pow2_split_io<INV, N, T, MODE, 1, 32>(lds, tw, tid, in2, sv);
  } else {
  constexpr int MB = N / R / T;
  float2 v[MB][R];
  stage_core<R, INV, N, L, T>(tw, tid, in, v);
  if constexpr (S == 0) hook();  // e.g. the twiddle tables' LDS writes, after the first stage's loads
  if constexpr (S == P::nst(MODE) - 1) {
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int i = tid + m * T;
#pragma unroll
      for (int r = 0; r < R; ++r) sv(m, r, i + r * L, v[m][r]);  // last stage: L R = N, k = i
    }
  } else {
    constexpr int R2 = P::radix(S + 1, MODE);
    constexpr bool PAIR = R2 == 32;  // next: the radix-32 lane-pair last stage
    constexpr int NB2 = N / R2;
    constexpr int MB2 = PAIR ? 1 : NB2 / T;
    constexpr int RR2 = PAIR ? 16 : R2;
    static_assert(split_lay<L>(N - 1) < 2 * lds_split_f2(N), "split layout exceeds the LDS image");
    static_assert(!PAIR || (T == N / 16 && S + 2 == P::nst(MODE)), "pair stage layout");
    static_assert(!PAIR || pair_offsets_ok([](int j) { return split_lay<L>(j); }, N), "pair-stage offsets");
    float2 nx[MB2][RR2];
    // output element j = (i - k) R + k + r L of this stage -> input i2 + r2 NB2 of the next; the
    // per-r address offsets are those of thread 0 (constant over threads for these layouts)
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      __syncthreads();  // previous readers of the image are done
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        const int i = tid + m * T;
        const int k = i & (L - 1);
        const int i0 = m * T, k0 = i0 & (L - 1), j0 = (i0 - k0) * R + k0;  // folds after unrolling
        float* dst = lds + split_lay<L>((i - k) * R + k);
#pragma unroll
        for (int r = 0; r < R; ++r)
          dst[split_lay<L>(j0 + r * L) - split_lay<L>(j0)] = part ? v[m][r].y : v[m][r].x;
      }
      __syncthreads();
      if constexpr (PAIR) {
        constexpr int LP = N / 32;
        const float* src = lds + split_lay<L>(pair_i(tid) + ((tid >> 5) & 1) * LP);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const float x = src[split_lay<L>(2 * s * LP) - split_lay<L>(0)];
          if (part) nx[0][s].y = x;
          else nx[0][s].x = x;
        }
      } else {
#pragma unroll
        for (int m = 0; m < MB2; ++m) {
          const float* src = lds + split_lay<L>(tid + m * T);
#pragma unroll
          for (int r = 0; r < R2; ++r) {
            const float x = src[split_lay<L>(m * T + r * NB2) - split_lay<L>(m * T)];
            if (part) nx[m][r].y = x;
            else nx[m][r].x = x;
          }
        }
      }
    }
    if constexpr (PAIR) {
      stage_r32_pair_last<INV, N>(tw, tid, nx[0], sv);
    } else {
      auto in2 = [&](int m, int r, int) { return nx[m][r]; };
      fft_pow2_split_io<INV, N, T, MODE, S + 1, L * R>(lds, tw, tid, in2, sv);
    }
  }
  }
}

// The row / column kernels' transform runs the split exchanges; tw_slot is where that kernel's
// twiddle tables start in LDS.
template <int N>
__device__ __forceinline__ float2* tw_slot(float2* lds) {
  return lds + lds_split_f2(N);
}
template <bool INV, int N, int T, int MODE, class Tw, class Ld, class Sv, class Hook = NoHook>
__device__ __forceinline__ void fft_pow2_run(float2* lds, const Tw& tw, int tid, Ld& ld, Sv& sv, Hook hook = Hook{}) {
  fft_pow2_split_io<INV, N, T, MODE>(reinterpret_cast<float*>(lds), tw, tid, ld, sv, hook);
}

// Whole transform with the data in LDS (natural order in and out).
template <bool INV, int N, int T, class Tw>
__device__ __forceinline__ void fft_pow2(float2* lds, const Tw& tw, int tid) {
  NoIO io;
  fft_pow2_io<INV, N, T, false, true, true>(lds, tw, tid, io, io);
}

// ---------------------------------------------------------------------------------------------
// Compile-time mixed-radix plans (non-power-of-two sizes with a fixed radix list, e.g.
// 300 = 5·3·4·5): the runtime plan's Stockham stages with N, L, R and the thread count known to
// the compiler (constant-divisor index math, exact butterfly trip counts, inlined), and the
// same fused I/O contract as fft_pow2_io: the first stage reads operand i + r N/R0 through
// ld(m, r, idx), the last stage hands result i + r N/Rlast to sv(m, r, j) from registers, with
// butterfly i = tid + m T.  A transform whose first radix equals the previous one's last radix
// therefore reads exactly the elements the previous transform left in this thread's registers.
// Twiddles exp(-+2 pi i k t / N) come from the plan's global table (L2-resident, N float2).
// ---------------------------------------------------------------------------------------------
template <bool INV, int N, int T, int L, int R, bool FIRST, bool LAST, int MW, class Ld, class Sv>
__device__ __forceinline__ void mx_stage(float2* lds, const float2 (&w1)[MW], const float2* __restrict__ tw, int tid,
                                         Ld& ld, Sv& sv) {
  constexpr int NB = N / R;
  constexpr int MB = (NB + T - 1) / T;
  static_assert(MB <= MW, "mixed plan: twiddle registers");
  float2 v[MB][R];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int i = tid + m * T;
    if (NB % T == 0 || i < NB) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (FIRST) v[m][r] = ld(m, r, i + r * NB);
        else v[m][r] = lds[i + r * NB];
      }
      if constexpr (L > 1) {
        const float2 w = w1[m];
        float2 wr = w;
#pragma unroll
        for (int r = 1; r < R; ++r) {
          v[m][r] = cmul_tw<INV>(v[m][r], wr);
          if (r + 1 < R) wr = cmul(wr, w);
        }
      }
      dftR<R, INV>(v[m]);
    }
  }
  if constexpr (LAST) {
    static_assert(L * R == N, "mixed plan: radices must multiply to N");
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int i = tid + m * T;
      if (NB % T == 0 || i < NB) {
#pragma unroll
        for (int r = 0; r < R; ++r) sv(m, r, i + r * NB, v[m][r]);
      }
    }
  } else {
    __syncthreads();  // every read of this stage (or the previous transform's) is done
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int i = tid + m * T;
      if (NB % T == 0 || i < NB) {
        const int k = i % L;
        const int j = (i - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[j + r * L] = v[m][r];
      }
    }
    __syncthreads();
  }
}

template <bool INV, int N, int T, int L, int S, bool FIRST, int NS, int MW, class Ld, class Sv, int R, int... Rest>
__device__ __forceinline__ void mx_stages(float2* lds, const float2 (&w1)[NS][MW], const float2* __restrict__ tw, int tid,
                                          Ld& ld, Sv& sv) {
  mx_stage<INV, N, T, L, R, FIRST, sizeof...(Rest) == 0>(lds, w1[S], tw, tid, ld, sv);
  if constexpr (sizeof...(Rest) > 0)
    mx_stages<INV, N, T, L * R, S + 1, false, NS, MW, Ld, Sv, Rest...>(lds, w1, tw, tid, ld, sv);
}

// The per-thread stage twiddles exp(-2 pi i k / (L R)), k = i mod L, of every stage, loaded once
// from the plan's table (tw[k N / (L R)]) and kept in registers across transforms.
template <int N, int T, int... Rs>
struct MxTw {
  static constexpr int NS = sizeof...(Rs);
  static constexpr int MW = (N / 2 + T - 1) / T;  // butterflies per thread of the smallest radix
  float2 w[NS][MW];
  const float2* tw;
  template <int L, int S, int R, int... Rest>
  __device__ __forceinline__ void fill(const float2* __restrict__ tw, int tid) {
    constexpr int NB = N / R, MB = (NB + T - 1) / T;
#pragma unroll
    for (int m = 0; m < MW; ++m) {
      const int i = tid + m * T;
      w[S][m] = (L > 1 && m < MB && i < NB) ? tw[(i % L) * (N / (L * R))] : make_float2(1.f, 0.f);
    }
    if constexpr (sizeof...(Rest) > 0) fill<L * R, S + 1, Rest...>(tw, tid);
  }
};

template <int... Rs>
struct MxPlan {
  static constexpr int N = (Rs * ...);
  static constexpr int RADIX[] = {Rs...};
  static constexpr int R0 = RADIX[0];
  static constexpr int RL = RADIX[sizeof...(Rs) - 1];
  template <int T>
  using Tw = MxTw<N, T, Rs...>;
  template <int T>
  __device__ __forceinline__ static Tw<T> twiddles(const float2* __restrict__ tw, int tid) {
    Tw<T> t;
    t.tw = tw;
    t.template fill<1, 0, Rs...>(tw, tid);
    return t;
  }
  template <bool INV, int T, class Ld, class Sv>
  __device__ __forceinline__ static void run(float2* lds, const Tw<T>& t, int tid, Ld& ld, Sv& sv) {
    mx_stages<INV, N, T, 1, 0, true, Tw<T>::NS, Tw<T>::MW, Ld, Sv, Rs...>(lds, t.w, t.tw, tid, ld, sv);
  }
};
// 300 = 5 3 4 5: first and last radix 5 (60 butterflies: one per lane of a 64-thread workgroup),
// so the forward's spectrum is 5 values per lane and the inverse starts from it directly
// (5 4 3 5 and 5 12 5 measured within noise / slower)
using Mx300 = MxPlan<5, 3, 4, 5>;
// 500 = 5 4 5 5 (the extended-DOF grid: 100 x 100 with padding scale 4): first and last radix 5
// (100 butterflies: two per lane of the 64-thread workgroup, the second on 36 lanes)
using Mx500 = MxPlan<5, 4, 5, 5>;
// the compile-time plan of a mixed-radix size
template <int N>
struct MxOf;
template <>
struct MxOf<300> {
  using type = Mx300;
};
template <>
struct MxOf<500> {
  using type = Mx500;
};

// Full transform of one row held in LDS (natural order in and out).  Unnormalised.
template <bool INV>
__device__ void fft_lds(float2* lds, const FftPlan& p, int tid, int nthr) {
  int L = 1;
  for (int s = 0; s < p.nst; ++s) {
    const int R = p.radix[s];
    switch (R) {
      case 16: stage_reg<16, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 8: stage_reg<8, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 4: stage_reg<4, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 2: stage_reg<2, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 3: stage_reg<3, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 5: stage_reg<5, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      case 7: stage_reg<7, INV>(lds, p.n, L, p.tw, tid, nthr); break;
      default: stage_generic<INV>(lds, p.n, L, R, p.tw, tid, nthr); break;
    }
    L *= R;
  }
}

}  // namespace thz
