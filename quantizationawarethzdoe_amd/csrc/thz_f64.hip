// Double-precision (complex128) propagators for gfx950: ASM, CZT and RSC / VRS as the reference
// computes them when a field is complex128 or its wavelengths are float64
// (DataType/ElectricField.py:85-90: tensor wavelengths keep their dtype and the products promote;
// the reference's only script, test_czt.py:12, runs RSC + CZT that way).
//
// Same decompositions as the fp32 kernels -- ASM and RSC as three LDS passes (row FFT of the
// windowed input, per-column FFT x transfer function x inverse with the row window kept, row
// inverse with the column window kept), CZT as two Bluestein passes -- on a runtime mixed-radix
// Stockham transform in double2 (radix 4, 2, 3, 5, 7 in registers, any other prime by a
// table DFT), every physics scalar in double.  No band pruning and no fused I/O: fp64 is the
// accuracy path, the fp32 kernels are the throughput path.  LDS holds one line of n double2
// (n <= 8192: 139 KiB with padding; 16 values per thread, 512 threads).
#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "thz_common.hpp"
#include "thz_dev.hpp"

namespace thz {
namespace f64 {

constexpr int MAXV = 16;           // values per thread per stage (512 threads at n = 8192)
constexpr int MAXT = 512;          // threads per line (up to 256 VGPRs: the 16 double2 a column keeps)
constexpr int MAX_N = 8192;        // longest transform (LDS: n + n/16 + 1 double2)
constexpr double TWO_PI = 6.283185307179586476925;

struct DPlan {
  int n, nst;
  int radix[FFT_MAX_STAGES];
  const double2* tw;  // exp(-2 pi i t / n), t < n
};

__device__ __forceinline__ int pad(int a) { return a + (a >> 4); }
inline size_t lds_bytes(int n) { return (size_t)(n + (n >> 4) + 1) * sizeof(double2); }
inline int threads(int n) {
  int t = (n + MAXV - 1) / MAXV;
  t = (t + 63) / 64 * 64;
  return std::max(64, std::min(MAXT, t));
}

__device__ __forceinline__ double2 dc(double x, double y) { return make_double2(x, y); }
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return dc(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return dc(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) { return dc(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ double2 conjd(double2 a) { return dc(a.x, -a.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) { return dc(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cis(double ph) {
  double s, c;
  sincos(ph, &s, &c);
  return dc(c, s);
}
// torch.linspace(start, end, n)[i] in fp64 (the two-sided form of ATen's kernel)
__device__ __forceinline__ double lin(double start, double end, int n, int i) {
  if (n == 1) return start;
  const double step = (end - start) / (double)(n - 1);
  return i < n / 2 ? start + step * (double)i : end - step * (double)(n - 1 - i);
}
// exp(i k r) z / (2 pi r^2) (1/r - i k), r = sqrt(x^2 + y^2 + z^2) (Props/CZT_Prop.py:44-57,
// Props/RSC_Prop.py:129-167)
__device__ __forceinline__ double2 rs_kernel(double x, double y, double z, double k) {
  const double r = sqrt(x * x + y * y + z * z);
  const double f = (1.0 / TWO_PI) * z / (r * r);
  return cmul(cis(k * r), dc(f * (1.0 / r), -f * k));
}

// ---------------------------------------------------------------------------------------------
// The transform: Stockham stages in place in LDS (read every operand, barrier, write)
// ---------------------------------------------------------------------------------------------
template <bool INV>
__device__ __forceinline__ double2 tw_at(const double2* __restrict__ tw, int t) {
  const double2 w = tw[t];
  return INV ? conjd(w) : w;
}

// in-register DFT of R values; roots w_R^q = tw[q n / R] of the length-n table
template <int R, bool INV>
__device__ __forceinline__ void dft(double2* v, const double2* __restrict__ tw, int n) {
  if constexpr (R == 2) {
    const double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    const double2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const double2 b0 = cadd(v[1], v[3]), b1 = csub(v[1], v[3]);
    // -i (forward) / +i (inverse) times b1
    const double2 jb1 = INV ? dc(-b1.y, b1.x) : dc(b1.y, -b1.x);
    v[0] = cadd(a0, b0);
    v[2] = csub(a0, b0);
    v[1] = cadd(a1, jb1);
    v[3] = csub(a1, jb1);
  } else {
    double2 w[R];
#pragma unroll
    for (int q = 0; q < R; ++q) w[q] = tw_at<INV>(tw, q * (n / R));
    double2 o[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      double2 acc = v[0];
#pragma unroll
      for (int r = 1; r < R; ++r) acc = cadd(acc, cmul(v[r], w[(r * q) % R]));
      o[q] = acc;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = o[q];
  }
}

template <int R, bool INV>
__device__ __forceinline__ void stage(double2* lds, int n, int L, const double2* __restrict__ tw, int tid, int nt) {
  constexpr int MB = (MAXV + R - 1) / R;
  const int nb = n / R;
  const int step = n / (L * R);
  double2 v[MB][R];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int i = tid + m * nt;
    if (i < nb) {
      const int k = i % L;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double2 x = lds[pad(i + r * nb)];
        v[m][r] = r == 0 ? x : cmul(x, tw_at<INV>(tw, k * r * step));
      }
      dft<R, INV>(v[m], tw, n);
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int i = tid + m * nt;
    if (i < nb) {
      const int k = i % L;
      const int j = (i - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) lds[pad(j + r * L)] = v[m][r];
    }
  }
  __syncthreads();
}

// any radix: each thread forms MAXV outputs straight from the table
template <bool INV>
__device__ __forceinline__ void stage_generic(double2* lds, int n, int L, int R, const double2* __restrict__ tw, int tid,
                                           int nt) {
  const int nb = n / R, LR = L * R, step = n / LR;
  double2 out[MAXV];
#pragma unroll
  for (int m = 0; m < MAXV; ++m) {
    const int o = tid + m * nt;
    out[m] = dc(0.0, 0.0);
    if (o < n) {
      const int k = o % L, q = (o / L) % R, b = o / LR;
      const int i = b * L + k, e = k + q * L;
      double2 acc = dc(0.0, 0.0);
      int t = 0;
      for (int r = 0; r < R; ++r) {
        acc = cadd(acc, cmul(lds[pad(i + r * nb)], tw_at<INV>(tw, t * step)));
        t += e;
        if (t >= LR) t -= LR;
      }
      out[m] = acc;
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MAXV; ++m) {
    const int o = tid + m * nt;
    if (o < n) lds[pad(o)] = out[m];
  }
  __syncthreads();
}

// unnormalised transform of the line in LDS (natural order in and out); callers barrier before
template <bool INV>
__device__ __noinline__ void fft(double2* lds, const DPlan& p, int tid, int nt) {
  int L = 1;
  for (int s = 0; s < p.nst; ++s) {
    const int R = p.radix[s];
    switch (R) {
      case 4: stage<4, INV>(lds, p.n, L, p.tw, tid, nt); break;
      case 2: stage<2, INV>(lds, p.n, L, p.tw, tid, nt); break;
      case 3: stage<3, INV>(lds, p.n, L, p.tw, tid, nt); break;
      case 5: stage<5, INV>(lds, p.n, L, p.tw, tid, nt); break;
      case 7: stage<7, INV>(lds, p.n, L, p.tw, tid, nt); break;
      default: stage_generic<INV>(lds, p.n, L, R, p.tw, tid, nt); break;
    }
    L *= R;
  }
}

// rows transforms: row r at in/out + r * stride (in place allowed), or with cstride > 1 the
// columns of a [rows x n] plane (element j of transform r at r + j * cstride)
__global__ void __launch_bounds__(MAXT) fft_lines(const double2* __restrict__ in, double2* __restrict__ out, DPlan p,
                                                 int inverse, size_t stride, int cstride) {
  extern __shared__ double2 dlds[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t base = cstride > 1 ? (size_t)blockIdx.x : (size_t)blockIdx.x * stride;
  const size_t es = cstride > 1 ? (size_t)cstride : 1;
  for (int j = tid; j < p.n; j += nt) dlds[pad(j)] = in[base + j * es];
  __syncthreads();
  if (inverse) fft<true>(dlds, p, tid, nt);
  else fft<false>(dlds, p, tid, nt);
  for (int j = tid; j < p.n; j += nt) out[base + j * es] = dlds[pad(j)];
}

// ---------------------------------------------------------------------------------------------
// ASM / RSC: three passes
// ---------------------------------------------------------------------------------------------
struct ConvArgs {
  int BC, C, Ph, Pw;
  int in_r0, in_c0, Hin, Win;      // input window inside the padded plane
  int out_r0, out_c0, Hout, Wout;  // output window
  int nz, zoff;
  int bl, adjoint;
  double dx, dy, scale;
  const double2* tft;  // RSC: transfer-function table [C][Pw][Ph] (column-major), else analytic ASM
  int vec;             // VRS: plane b == 2 is Ez = Ex x / r + Ey y / r on the unpadded grid
  double zr;
  double lam[THZ_MAX_WAVELENGTHS];
  double zv[THZ_MAX_Z];
};

// H(kx, ky) = exp(i z sqrt(k^2 - K^2)), evanescent and band-limit masks (Props/ASM_Prop.py:212-311)
__device__ __forceinline__ double2 tf_value(const ConvArgs& a, double lam, double z, int mx, int my) {
  const double kx = (double)mx / (double)a.Ph, ky = (double)my / (double)a.Pw;
  const double Kx = TWO_PI * kx / a.dx, Ky = TWO_PI * ky / a.dy;
  const double K2 = Kx * Kx + Ky * Ky;
  const double k = TWO_PI / lam;
  const double k2 = k * k;
  if (k2 - K2 < 0.0) return dc(0.0, 0.0);
  if (a.bl == THZ_BANDLIMIT_EXACT) {
    const double du = ((TWO_PI / a.dx) / (2.0 * a.Ph)) / TWO_PI;
    const double dv = ((TWO_PI / a.dy) / (2.0 * a.Ph)) / TWO_PI;  // Ph for v too (:290-291)
    const double ul = 1.0 / sqrt((2.0 * du * z) * (2.0 * du * z) + 1.0) / lam;
    const double vl = 1.0 / sqrt((2.0 * dv * z) * (2.0 * dv * z) + 1.0) / lam;
    const double au = TWO_PI * ul, av = TWO_PI * vl;
    const bool c1 = (Kx * Kx) / (au * au) + (Ky * Ky) / k2 <= 1.0;
    const bool c2 = (Kx * Kx) / k2 + (Ky * Ky) / (av * av) <= 1.0;
    if (!(c1 && c2)) return dc(0.0, 0.0);
  } else if (a.bl == THZ_BANDLIMIT_APPROX) {
    const double Lx = a.Ph * a.dx, Ly = a.Ph * a.dy;  // length_y uses Ph (:275)
    const double kxm = TWO_PI / sqrt((2.0 * (1.0 / Lx) * z) * (2.0 * (1.0 / Lx) * z) + 1.0) / lam;
    const double kym = TWO_PI / sqrt((2.0 * (1.0 / Ly) * z) * (2.0 * (1.0 / Ly) * z) + 1.0) / lam;
    if (fabs(Kx) > kxm || fabs(Ky) > kym) return dc(0.0, 0.0);
  }
  const double2 h = cis(z * sqrt(k2 - K2));
  return a.adjoint ? conjd(h) : h;
}

// K1: per input row (plane zz of the chunk only for a multi-plane adjoint is not used: Z == 1),
// FFT(Pw) of the windowed row -> T[bc][j][h] (column-major)
__global__ void __launch_bounds__(MAXT) conv_rows_fwd(const double2* __restrict__ in, double2* __restrict__ T, DPlan pw,
                                                     ConvArgs a) {
  extern __shared__ double2 dlds[];
  const int row = blockIdx.x;
  const int bc = row / a.Hin, h = row - bc * a.Hin;
  const int tid = threadIdx.x, nt = blockDim.x;
  const double2* src = in + ((size_t)bc * a.Hin + h) * a.Win;
  const bool ez = a.vec && bc / a.C == 2;
  const double2* sx = in + ((size_t)(bc % a.C) * a.Hin + h) * a.Win;
  const double2* sy = in + ((size_t)(a.C + bc % a.C) * a.Hin + h) * a.Win;
  const double xh = ez ? lin(-(double)a.Hin * a.dx / 2.0, (double)a.Hin * a.dx / 2.0, a.Hin, h) : 0.0;
  for (int j = tid; j < a.Pw; j += nt) {
    const int s = j - a.in_c0;
    double2 v = dc(0.0, 0.0);
    if (s >= 0 && s < a.Win) {
      if (!ez) {
        v = src[s];
      } else {  // Props/RSC_Prop.py:294-303 (dx on both axes, :83-84)
        const double y = lin(-(double)a.Win * a.dx / 2.0, (double)a.Win * a.dx / 2.0, a.Win, s);
        const double r = sqrt(xh * xh + y * y + a.zr * a.zr);
        v = cadd(cscale(sx[s], xh / r), cscale(sy[s], y / r));
      }
    }
    dlds[pad(j)] = v;
  }
  __syncthreads();
  fft<false>(dlds, pw, tid, nt);
  double2* dst = T + (size_t)bc * a.Pw * a.Hin + h;
  for (int j = tid; j < a.Pw; j += nt) dst[(size_t)j * a.Hin] = dlds[pad(j)];
}

// K2: per (bc, column j): FFT(Ph) of the windowed column once, kept in the workspace S (a line of
// 16 double2 per thread does not fit beside the transform's registers), then per z: S x H_z (or
// the RSC table), inverse, keep the output rows -> U[z][bc][j][r]
__global__ void __launch_bounds__(MAXT) conv_cols(const double2* __restrict__ T, double2* __restrict__ S,
                                                 double2* __restrict__ U, DPlan ph, ConvArgs a) {
  extern __shared__ double2 dlds[];
  const int id = blockIdx.x;
  const int bc = id / a.Pw, j = id - bc * a.Pw;
  const int tid = threadIdx.x, nt = blockDim.x;
  const double2* col = T + ((size_t)bc * a.Pw + j) * a.Hin;
  double2* spec = S + ((size_t)bc * a.Pw + j) * a.Ph;
  for (int i = tid; i < a.Ph; i += nt) {
    const int s = i - a.in_r0;
    dlds[pad(i)] = (s >= 0 && s < a.Hin) ? col[s] : dc(0.0, 0.0);
  }
  __syncthreads();
  fft<false>(dlds, ph, tid, nt);
  if (a.zoff == 0)
    for (int i = tid; i < a.Ph; i += nt) spec[i] = dlds[pad(i)];
  const double lam = a.lam[bc % a.C];
  const int my = freq_index(j, a.Pw);
  const double2* tcol = a.tft ? a.tft + ((size_t)(bc % a.C) * a.Pw + j) * a.Ph : nullptr;
  for (int zz = 0; zz < a.nz; ++zz) {
    const double z = a.zv[a.zoff + zz];
    __syncthreads();  // the previous plane's readers are done with the line (and spec is written)
    for (int i = tid; i < a.Ph; i += nt) {
      const double2 h = tcol ? (a.adjoint ? conjd(tcol[i]) : tcol[i]) : tf_value(a, lam, z, freq_index(i, a.Ph), my);
      dlds[pad(i)] = cmul(spec[i], h);
    }
    __syncthreads();
    fft<true>(dlds, ph, tid, nt);
    double2* dst = U + (((size_t)zz * a.BC + bc) * a.Pw + j) * a.Hout;
    for (int r = tid; r < a.Hout; r += nt) dst[r] = cscale(dlds[pad(a.out_r0 + r)], a.scale);
  }
}

// K3: per output row of each plane: IFFT(Pw) of U's row, keep the output columns
__global__ void __launch_bounds__(MAXT) conv_rows_inv(const double2* __restrict__ U, double2* __restrict__ out, DPlan pw,
                                                     ConvArgs a) {
  extern __shared__ double2 dlds[];
  const int row = blockIdx.x;  // (zz BC + bc) Hout + r
  const int plane = row / a.Hout, r = row - plane * a.Hout;
  const int tid = threadIdx.x, nt = blockDim.x;
  const double2* src = U + (size_t)plane * a.Pw * a.Hout + r;
  for (int j = tid; j < a.Pw; j += nt) dlds[pad(j)] = src[(size_t)j * a.Hout];
  __syncthreads();
  fft<true>(dlds, pw, tid, nt);
  double2* dst = out + ((size_t)(a.zoff * a.BC + plane) * a.Hout + r) * a.Wout;
  for (int w = tid; w < a.Wout; w += nt) dst[w] = dlds[pad(a.out_c0 + w)];
}

// RSC spatial kernel on the P grid: K[c][i][j] = RS(x_i, y_j), x = linspace(-Ph dx/2, Ph dx/2, Ph),
// y = linspace(-Pw dx/2, Pw dx/2, Pw) (dx on both axes, Props/RSC_Prop.py:79-87, 129-167)
__global__ void rsc_spatial(double2* __restrict__ K, int Ph, int Pw, double dx, double z, ConvArgs a) {
  const int c = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)Ph * Pw) return;
  const int i = (int)(e / Pw), j = (int)(e - (size_t)i * Pw);
  const double x = lin(-(double)Ph * dx / 2.0, (double)Ph * dx / 2.0, Ph, i);
  const double y = lin(-(double)Pw * dx / 2.0, (double)Pw * dx / 2.0, Pw, j);
  K[(size_t)c * Ph * Pw + e] = rs_kernel(x, y, z, TWO_PI / a.lam[c]);
}

// [C][Ph][Pw] row-major -> [C][Pw][Ph] (the column pass reads a column contiguously)
__global__ void transpose_planes(const double2* __restrict__ in, double2* __restrict__ out, int Ph, int Pw) {
  const int c = blockIdx.y;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)Ph * Pw) return;
  const int j = (int)(e / Ph), i = (int)(e - (size_t)j * Ph);
  out[(size_t)c * Ph * Pw + e] = in[(size_t)c * Ph * Pw + (size_t)i * Pw + j];
}

// ---------------------------------------------------------------------------------------------
// CZT: two Bluestein passes (Props/CZT_Prop.py:132-250); see thz_czt.hip for the decomposition
// ---------------------------------------------------------------------------------------------
struct Pass {
  int m, M, np2, ntab;
  double f1, f2;
};
struct CztArgs {
  int BC, C, H, W, outH, outW;
  double dx, dy, odx, ody, z;
  Pass pa, pb;  // pass A: W axis (fx, outH); pass B: H axis (fy, outW)
  size_t preA, postA, ftA, preB, postB, ftB, tabStride;  // double2 offsets per wavelength
  double lam[THZ_MAX_WAVELENGTHS];
};

struct Blue {
  double Dm, D1, D2, thA, thW;
};
__device__ __forceinline__ Blue blue(const Pass& p, double lam, double z, double dx) {
  Blue b;
  b.Dm = lam * z / dx;
  const double f1 = p.f1 + b.Dm / 2, f2 = p.f2 + b.Dm / 2, M = p.M;
  b.D1 = f1 + (M * b.Dm + f2 - f1) / (2 * M);
  b.D2 = f2 + (M * b.Dm + f2 - f1) / (2 * M);
  b.thA = TWO_PI * b.D1 / b.Dm;
  b.thW = -TWO_PI * (b.D1 - b.D2) / (M * b.Dm);
  return b;
}

// pre[j] = A^-j W^(j^2/2), post[l] = W^(l^2/2) M_shift[l] / np2, g[t] = 1/h[t] (FFT'd afterwards)
__global__ void czt_tables(CztArgs a, double2* __restrict__ ws, int pass) {
  const int c = blockIdx.y;
  const Pass& p = pass == 0 ? a.pa : a.pb;
  const Blue b = blue(p, a.lam[c], a.z, a.dx);
  double2* pre = ws + (pass == 0 ? a.preA : a.preB) + (size_t)c * a.tabStride;
  double2* post = ws + (pass == 0 ? a.postA : a.postB) + (size_t)c * a.tabStride;
  double2* g = ws + (pass == 0 ? a.ftA : a.ftB) + (size_t)c * a.tabStride;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < p.m) pre[n] = cis(-b.thA * n + b.thW * (double)n * n / 2);
  if (n < p.M) {
    const double l = n;
    const double ell = l / p.M * (b.D2 - b.D1) + b.D1;
    const double shift = -TWO_PI * ell * (-p.m / 2.0 + 0.5) / b.Dm;
    post[n] = cscale(cis(b.thW * l * l / 2 + shift), 1.0 / p.np2);
  }
  if (n < p.np2) {
    const double jj = n - p.m + 1;
    g[n] = n < p.ntab ? cis(-b.thW * jj * jj / 2) : dc(0.0, 0.0);
  }
}

// one Bluestein line: LDS <- ld(j) (j < np2), FFT, x filter (conj for the adjoint), IFFT -> st(j, v)
template <class Ld, class St>
__device__ __forceinline__ void blue_line(double2* lds, const DPlan& p, const double2* __restrict__ ft, bool adj,
                                          Ld& ld, St& st) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int j = tid; j < p.n; j += nt) lds[pad(j)] = ld(j);
  __syncthreads();
  fft<false>(lds, p, tid, nt);
  for (int j = tid; j < p.n; j += nt) lds[pad(j)] = cmul(lds[pad(j)], adj ? conjd(ft[j]) : ft[j]);
  __syncthreads();
  fft<true>(lds, p, tid, nt);
  for (int j = tid; j < p.n; j += nt) st(j, lds[pad(j)]);
}

// pass A (rows, W axis): in [BC][H][W] -> V [BC][q][h], q < outH
__global__ void __launch_bounds__(MAXT) czt_rows(const double2* __restrict__ in, double2* __restrict__ V,
                                                const double2* __restrict__ ws, DPlan pl, CztArgs a) {
  extern __shared__ double2 dlds[];
  const int row = blockIdx.x;
  const int bc = row / a.H, h = row - bc * a.H, c = bc % a.C;
  const double lam = a.lam[c], k = TWO_PI / lam;
  const double xh = lin(-(double)a.H * a.dx / 2.0, (double)a.H * a.dx / 2.0, a.H, h);
  const double ylo = -(double)a.W * a.dy / 2.0, yhi = (double)a.W * a.dy / 2.0;
  const double2* src = in + ((size_t)bc * a.H + h) * a.W;
  const double2* pre = ws + a.preA + (size_t)c * a.tabStride;
  const double2* post = ws + a.postA + (size_t)c * a.tabStride;
  const double2* ft = ws + a.ftA + (size_t)c * a.tabStride;
  double2* dst = V + (size_t)bc * a.outH * a.H + h;
  const int m = a.W, M = a.outH;
  auto ld = [&](int w) {
    if (w >= m) return dc(0.0, 0.0);
    return cmul(cmul(src[w], rs_kernel(xh, lin(ylo, yhi, a.W, w), a.z, k)), pre[w]);
  };
  auto st = [&](int j, double2 v) {
    const int q = j - m;
    if (q >= 0 && q < M) dst[(size_t)q * a.H] = cmul(v, post[q]);
  };
  blue_line(dlds, pl, ft, false, ld, st);
}

// pass B (columns, H axis) of V -> out [BC][outW][outH]: out[p][q] = F0 U z dxo dyo lambda
__global__ void __launch_bounds__(MAXT) czt_cols(const double2* __restrict__ V, double2* __restrict__ out,
                                                const double2* __restrict__ ws, DPlan pl, CztArgs a) {
  extern __shared__ double2 dlds[];
  const int id = blockIdx.x;
  const int bc = id / a.outH, q = id - bc * a.outH, c = bc % a.C;
  const double lam = a.lam[c], k = TWO_PI / lam;
  const double2* col = V + ((size_t)bc * a.outH + q) * a.H;
  const double2* pre = ws + a.preB + (size_t)c * a.tabStride;
  const double2* post = ws + a.postB + (size_t)c * a.tabStride;
  const double2* ft = ws + a.ftB + (size_t)c * a.tabStride;
  double2* dst = out + (size_t)bc * a.outW * a.outH + q;
  const int m = a.H, M = a.outW;
  const double yq = lin(-(double)a.outW * a.ody / 2.0, (double)a.outW * a.ody / 2.0, a.outW, q);
  const double xlo = -(double)a.outH * a.odx / 2.0, xhi = (double)a.outH * a.odx / 2.0;
  const double cst = a.z * a.odx * a.ody * lam;
  auto ld = [&](int h) { return h < m ? cmul(col[h], pre[h]) : dc(0.0, 0.0); };
  auto st = [&](int j, double2 v) {
    const int p = j - m;
    if (p >= 0 && p < M)
      dst[(size_t)p * a.outH] = cscale(cmul(rs_kernel(lin(xlo, xhi, a.outH, p), yq, a.z, k), cmul(v, post[p])), cst);
  };
  blue_line(dlds, pl, ft, false, ld, st);
}

// adjoint of pass B: G [BC][outW][outH] (column q) -> V^ [BC][q][h]
__global__ void __launch_bounds__(MAXT) czt_cols_adj(const double2* __restrict__ G, double2* __restrict__ V,
                                                    const double2* __restrict__ ws, DPlan pl, CztArgs a) {
  extern __shared__ double2 dlds[];
  const int id = blockIdx.x;
  const int bc = id / a.outH, q = id - bc * a.outH, c = bc % a.C;
  const double lam = a.lam[c], k = TWO_PI / lam;
  const double2* pre = ws + a.preB + (size_t)c * a.tabStride;
  const double2* post = ws + a.postB + (size_t)c * a.tabStride;
  const double2* ft = ws + a.ftB + (size_t)c * a.tabStride;
  const double2* src = G + (size_t)bc * a.outW * a.outH + q;
  double2* dst = V + ((size_t)bc * a.outH + q) * a.H;
  const int m = a.H, M = a.outW, N = pl.n;
  const double yq = lin(-(double)a.outW * a.ody / 2.0, (double)a.outW * a.ody / 2.0, a.outW, q);
  const double xlo = -(double)a.outH * a.odx / 2.0, xhi = (double)a.outH * a.odx / 2.0;
  const double cst = a.z * a.odx * a.ody * lam;
  auto ld = [&](int j) {
    int p = j - m;
    if (p < 0) p += N;
    if (p >= M) return dc(0.0, 0.0);
    const double2 F0 = rs_kernel(lin(xlo, xhi, a.outH, p), yq, a.z, k);
    return cmul(conjd(post[p]), cscale(cmul(conjd(F0), src[(size_t)p * a.outH]), cst));
  };
  auto st = [&](int j, double2 v) {
    if (j < m) dst[j] = cmul(conjd(pre[j]), v);
  };
  blue_line(dlds, pl, ft, true, ld, st);
}

// adjoint of pass A: V^ row h -> grad_in [BC][H][W]
__global__ void __launch_bounds__(MAXT) czt_rows_adj(const double2* __restrict__ V, double2* __restrict__ gin,
                                                    const double2* __restrict__ ws, DPlan pl, CztArgs a) {
  extern __shared__ double2 dlds[];
  const int row = blockIdx.x;
  const int bc = row / a.H, h = row - bc * a.H, c = bc % a.C;
  const double lam = a.lam[c], k = TWO_PI / lam;
  const double xh = lin(-(double)a.H * a.dx / 2.0, (double)a.H * a.dx / 2.0, a.H, h);
  const double ylo = -(double)a.W * a.dy / 2.0, yhi = (double)a.W * a.dy / 2.0;
  const double2* pre = ws + a.preA + (size_t)c * a.tabStride;
  const double2* post = ws + a.postA + (size_t)c * a.tabStride;
  const double2* ft = ws + a.ftA + (size_t)c * a.tabStride;
  const double2* src = V + (size_t)bc * a.outH * a.H + h;
  double2* dst = gin + ((size_t)bc * a.H + h) * a.W;
  const int m = a.W, M = a.outH, N = pl.n;
  auto ld = [&](int j) {
    int qq = j - m;
    if (qq < 0) qq += N;
    if (qq >= M) return dc(0.0, 0.0);
    return cmul(conjd(post[qq]), src[(size_t)qq * a.H]);
  };
  auto st = [&](int j, double2 v) {
    if (j < m) dst[j] = cmul(conjd(rs_kernel(xh, lin(ylo, yhi, a.W, j), a.z, k)), cmul(conjd(pre[j]), v));
  };
  blue_line(dlds, pl, ft, true, ld, st);
}

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
static std::vector<int> factorise(int n) {
  std::vector<int> r;
  while (n % 4 == 0) { r.push_back(4); n /= 4; }
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

static std::mutex g_mu;
static std::map<std::pair<int, int>, double2*> g_tw;  // (device, n) -> table

static int get_plan(int n, DPlan* out) {
  if (n < 1 || n > MAX_N) return fail(THZ_E_UNSUPPORTED, "fp64 FFT length %d outside [1, %d]", n, MAX_N);
  std::vector<int> f = factorise(n);
  if ((int)f.size() > FFT_MAX_STAGES) return fail(THZ_E_UNSUPPORTED, "fp64 FFT length %d: too many stages", n);
  int dev = 0;
  THZ_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_pair(dev, n);
  auto it = g_tw.find(key);
  if (it == g_tw.end()) {
    std::vector<double2> h(n);
    for (int t = 0; t < n; ++t) {
      // exp(-2 pi i t / n) from the reduced angle (t / n in [0, 1) revolutions, long double)
      const long double a = -2.0L * 3.141592653589793238462643383279502884L * (long double)t / (long double)n;
      h[t] = make_double2((double)cosl(a), (double)sinl(a));
    }
    double2* d = nullptr;
    THZ_HIP_CHECK(hipMalloc(&d, sizeof(double2) * n));
    THZ_HIP_CHECK(hipMemcpy(d, h.data(), sizeof(double2) * n, hipMemcpyHostToDevice));
    it = g_tw.emplace(key, d).first;
  }
  out->n = n;
  out->nst = (int)f.size();
  for (int s = 0; s < FFT_MAX_STAGES; ++s) out->radix[s] = s < (int)f.size() ? f[s] : 1;
  out->tw = it->second;
  return THZ_OK;
}

static int lds_attr() {
  static std::once_flag once;
  static hipError_t err = hipSuccess;
  std::call_once(once, [] {
    const int mx = (int)lds_bytes(MAX_N);
    const void* ks[] = {(const void*)fft_lines,    (const void*)conv_rows_fwd, (const void*)conv_cols,
                        (const void*)conv_rows_inv, (const void*)czt_rows,     (const void*)czt_cols,
                        (const void*)czt_rows_adj,  (const void*)czt_cols_adj};
    for (const void* k : ks) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      if (e != hipSuccess) err = e;
    }
  });
  if (err != hipSuccess) return fail(THZ_E_HIP, "hipFuncSetAttribute(fp64): %s", hipGetErrorString(err));
  return THZ_OK;
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

static int lines(const double2* in, double2* out, int count, const DPlan& p, int inverse, size_t stride, int cstride,
                 hipStream_t s) {
  hipLaunchKernelGGL(fft_lines, dim3(count), dim3(threads(p.n)), lds_bytes(p.n), s, in, out, p, inverse, stride,
                     cstride);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}

// --- ASM / RSC pipeline ----------------------------------------------------------------------
struct ConvGeom {
  int zc;
  size_t t, s, u;  // workspace bytes: row spectra T, column spectra S, column-pass output U
  size_t total() const { return t + s + u; }
};

static ConvGeom conv_geom(const ConvArgs& a, int Z) {
  ConvGeom g;
  const double per_z = (double)a.BC * a.Pw * a.Hout * sizeof(double2);
  g.zc = (int)std::max(1.0, std::min((double)Z, std::floor((8192.0 * 1024 * 1024) / per_z)));
  g.t = a256((size_t)a.BC * a.Pw * a.Hin * sizeof(double2));
  g.s = a256((size_t)a.BC * a.Pw * a.Ph * sizeof(double2));
  g.u = a256((size_t)g.zc * a.BC * a.Pw * a.Hout * sizeof(double2));
  return g;
}

static int run_conv(ConvArgs a, int Z, const double2* in, double2* out, char* ws, hipStream_t s) {
  int e;
  if ((e = lds_attr())) return e;
  DPlan pw, ph;
  if ((e = get_plan(a.Pw, &pw))) return e;
  if ((e = get_plan(a.Ph, &ph))) return e;
  const ConvGeom g = conv_geom(a, Z);
  double2* T = (double2*)ws;
  double2* S = (double2*)(ws + g.t);
  double2* U = (double2*)(ws + g.t + g.s);
  {
    KernelTimer kt("asm64_rows_fwd", s);
    hipLaunchKernelGGL(conv_rows_fwd, dim3(a.BC * a.Hin), dim3(threads(a.Pw)), lds_bytes(a.Pw), s, in, T, pw, a);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  for (int z0 = 0; z0 < Z; z0 += g.zc) {
    a.zoff = z0;
    a.nz = std::min(g.zc, Z - z0);
    KernelTimer kt("asm64_cols_rows", s);
    hipLaunchKernelGGL(conv_cols, dim3(a.BC * a.Pw), dim3(threads(a.Ph)), lds_bytes(a.Ph), s, (const double2*)T, S,
                       U, ph, a);
    THZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(conv_rows_inv, dim3(a.nz * a.BC * a.Hout), dim3(threads(a.Pw)), lds_bytes(a.Pw), s,
                       (const double2*)U, out, pw, a);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  return THZ_OK;
}

static int asm_args(const thz_asm_desc64* d, ConvArgs* a) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || d->pad_h < 0 || d->pad_w < 0)
    return fail(THZ_E_ARG, "bad shape B=%d C=%d H=%d W=%d pad=(%d,%d)", d->B, d->C, d->H, d->W, d->pad_h, d->pad_w);
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d wavelengths", d->C, THZ_MAX_WAVELENGTHS);
  if (d->Z < 1 || d->Z > THZ_MAX_Z) return fail(THZ_E_UNSUPPORTED, "Z=%d outside [1, %d]", d->Z, THZ_MAX_Z);
  if (d->adjoint && d->Z != 1) return fail(THZ_E_ARG, "the fp64 adjoint takes one z-plane (got %d)", d->Z);
  if (d->bandlimit < 0 || d->bandlimit > 2) return fail(THZ_E_ARG, "bad bandlimit %d", d->bandlimit);
  if (!d->wavelengths || !d->z) return fail(THZ_E_ARG, "null wavelengths / z");
  if (!(d->dx > 0.0) || !(d->dy > 0.0)) return fail(THZ_E_ARG, "spacing must be > 0");
  *a = ConvArgs{};
  a->BC = d->B * d->C;
  a->C = d->C;
  a->Ph = d->H + 2 * d->pad_h;
  a->Pw = d->W + 2 * d->pad_w;
  if (a->Ph > MAX_N || a->Pw > MAX_N)
    return fail(THZ_E_UNSUPPORTED, "fp64 padded size %dx%d exceeds %d", a->Ph, a->Pw, MAX_N);
  const int Ho = d->unpad ? d->H : a->Ph, Wo = d->unpad ? d->W : a->Pw;
  const int o_r0 = d->unpad ? d->pad_h : 0, o_c0 = d->unpad ? d->pad_w : 0;
  if (!d->adjoint) {
    a->in_r0 = d->pad_h; a->in_c0 = d->pad_w; a->Hin = d->H; a->Win = d->W;
    a->out_r0 = o_r0; a->out_c0 = o_c0; a->Hout = Ho; a->Wout = Wo;
  } else {
    a->in_r0 = o_r0; a->in_c0 = o_c0; a->Hin = Ho; a->Win = Wo;
    a->out_r0 = d->pad_h; a->out_c0 = d->pad_w; a->Hout = d->H; a->Wout = d->W;
  }
  a->bl = d->bandlimit;
  a->adjoint = d->adjoint;
  a->dx = d->dx;
  a->dy = d->dy;
  a->scale = 1.0 / ((double)a->Ph * (double)a->Pw);
  for (int c = 0; c < d->C; ++c) {
    if (!(d->wavelengths[c] > 0.0)) return fail(THZ_E_ARG, "wavelength[%d] must be > 0", c);
    a->lam[c] = d->wavelengths[c];
  }
  for (int zi = 0; zi < d->Z; ++zi) a->zv[zi] = d->z[zi];
  return THZ_OK;
}

// --- RSC -------------------------------------------------------------------------------------
struct RscPlan64 {
  ConvArgs a;
  size_t kt, kf;  // spatial kernel / its spectrum (transposed), bytes
};

static int rsc_args(const thz_rsc_desc64* d, RscPlan64* p) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1) return fail(THZ_E_ARG, "bad RSC shape");
  if (d->vectorial && d->B < 2) return fail(THZ_E_ARG, "vectorial RSC needs Ex, Ey planes (B >= 2)");
  if (d->adjoint && d->vectorial) return fail(THZ_E_ARG, "RSC adjoint is per plane: vectorial must be 0");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  if (!d->wavelengths) return fail(THZ_E_ARG, "null wavelengths");
  ConvArgs& a = p->a;
  a = ConvArgs{};
  a.Ph = d->H + 2 * (d->H / 2);
  a.Pw = d->W + 2 * (d->W / 2);
  if (a.Ph > MAX_N || a.Pw > MAX_N) return fail(THZ_E_UNSUPPORTED, "fp64 RSC grid %dx%d too large", a.Ph, a.Pw);
  a.BC = (d->vectorial ? 3 : d->B) * d->C;
  a.C = d->C;
  if (!d->adjoint) {  // U[..., :H, :W] = field (:198-200); ifft2(...)[..., H:, W:] (:207)
    a.in_r0 = 0; a.in_c0 = 0; a.Hin = d->H; a.Win = d->W;
    a.out_r0 = d->H; a.out_c0 = d->W; a.Hout = a.Ph - d->H; a.Wout = a.Pw - d->W;
  } else {
    a.in_r0 = d->H; a.in_c0 = d->W; a.Hin = a.Ph - d->H; a.Win = a.Pw - d->W;
    a.out_r0 = 0; a.out_c0 = 0; a.Hout = d->H; a.Wout = d->W;
    a.adjoint = 1;
  }
  a.bl = THZ_BANDLIMIT_NONE;
  a.dx = d->dx;
  a.dy = d->dy;
  a.scale = d->dx * d->dy / ((double)a.Ph * (double)a.Pw);
  a.vec = d->vectorial;
  a.zr = d->z;
  a.nz = 1;
  a.zv[0] = d->z;
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  p->kt = a256((size_t)d->C * a.Ph * a.Pw * sizeof(double2));
  p->kf = p->kt;
  return THZ_OK;
}

// --- CZT -------------------------------------------------------------------------------------
static int np2_of(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

static int czt_args(const thz_czt_desc64* d, CztArgs* a, size_t* total) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || d->outH < 1 || d->outW < 1)
    return fail(THZ_E_ARG, "bad CZT shape");
  if (d->outH != d->outW)
    return fail(THZ_E_ARG, "CZT output must be square: the reference multiplies F0 [outH,outW] with the "
                           "transposed [outW,outH] transform (Props/CZT_Prop.py:248); got %dx%d", d->outH, d->outW);
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  if (!d->wavelengths) return fail(THZ_E_ARG, "null wavelengths");
  *a = CztArgs{};
  a->BC = d->B * d->C;
  a->C = d->C;
  a->H = d->H;
  a->W = d->W;
  a->outH = d->outH;
  a->outW = d->outW;
  a->dx = d->dx;
  a->dy = d->dy;
  a->odx = d->odx;
  a->ody = d->ody;
  a->z = d->z;
  auto make = [](Pass* p, int m, int M, double lo, double hi) {
    p->m = m;
    p->M = M;
    const int mp = m + M - 1;
    p->np2 = np2_of(mp);
    p->ntab = std::min(mp + 1, m + std::max(M - 1, m - 1));
    p->f1 = lo;
    p->f2 = hi;
  };
  // x_out = linspace(-outH dxo/2, outH dxo/2, outH), y_out likewise (Props/CZT_Prop.py:101-102)
  const double xo = d->outH * d->odx / 2.0, yo = d->outW * d->ody / 2.0;
  make(&a->pa, d->W, d->outH, -xo, xo);  // the reference's second Bluestein (:246): fx, outH
  make(&a->pb, d->H, d->outW, -yo, yo);  // its first (:243): fy, outW
  // mp a power of two: the reference raises there (see thz_czt.hip czt_validate)
  if (a->pa.np2 == a->pa.m + a->pa.M - 1 || a->pb.np2 == a->pb.m + a->pb.M - 1)
    return fail(THZ_E_ARG, "CZT Bluestein length m + M - 1 is a power of two: the reference's slice "
                           "b[m:mp+1] keeps M - 1 rows there and its product with h[m-1:mp] raises "
                           "(Props/CZT_Prop.py:206,211)");
  if (a->pa.np2 > MAX_N || a->pb.np2 > MAX_N)
    return fail(THZ_E_UNSUPPORTED, "fp64 Bluestein length %d/%d exceeds %d", a->pa.np2, a->pb.np2, MAX_N);
  size_t off = 0;
  auto take = [&](size_t n) {
    const size_t o = off;
    off += (n + 15) & ~(size_t)15;
    return o;
  };
  a->preA = take(a->pa.m);
  a->postA = take(a->pa.M);
  a->ftA = take(a->pa.np2);
  a->preB = take(a->pb.m);
  a->postB = take(a->pb.M);
  a->ftB = take(a->pb.np2);
  a->tabStride = off;
  for (int c = 0; c < d->C; ++c) {
    if (!(d->wavelengths[c] > 0.0)) return fail(THZ_E_ARG, "wavelength[%d] must be > 0", c);
    a->lam[c] = d->wavelengths[c];
  }
  *total = a256(off * d->C * sizeof(double2)) + a256((size_t)a->BC * d->outH * d->H * sizeof(double2));
  return THZ_OK;
}

}  // namespace f64
}  // namespace thz

using namespace thz;

extern "C" int thz_fft64_rows(const void* in, void* out, int rows, int n, int inverse, thz_stream_t stream) {
  if (!in || !out || rows < 1) return fail(THZ_E_ARG, "bad fft64_rows arguments");
  int e;
  f64::DPlan p;
  if ((e = f64::get_plan(n, &p))) return e;
  if ((e = f64::lds_attr())) return e;
  return f64::lines((const double2*)in, (double2*)out, rows, p, inverse, (size_t)n, 1, (hipStream_t)stream);
}

extern "C" int thz_asm64_workspace_size(const thz_asm_desc64* d, size_t* bytes) {
  f64::ConvArgs a;
  int e = f64::asm_args(d, &a);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  const f64::ConvGeom g = f64::conv_geom(a, d->Z);
  *bytes = g.total();
  return THZ_OK;
}

extern "C" int thz_asm64_forward(const thz_asm_desc64* d, const void* in, void* out, void* workspace,
                                 size_t workspace_bytes, thz_stream_t stream) {
  f64::ConvArgs a;
  int e = f64::asm_args(d, &a);
  if (e) return e;
  if (!in || !out) return fail(THZ_E_ARG, "null data pointer");
  const f64::ConvGeom g = f64::conv_geom(a, d->Z);
  if (!workspace || workspace_bytes < g.total())
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, g.total());
  return f64::run_conv(a, d->Z, (const double2*)in, (double2*)out, (char*)workspace, (hipStream_t)stream);
}

extern "C" int thz_rsc64_workspace_size(const thz_rsc_desc64* d, size_t* bytes) {
  f64::RscPlan64 p;
  int e = f64::rsc_args(d, &p);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  const f64::ConvGeom g = f64::conv_geom(p.a, 1);
  *bytes = p.kt + p.kf + g.total();
  return THZ_OK;
}

extern "C" int thz_rsc64_forward(const thz_rsc_desc64* d, const void* in, void* out, void* workspace,
                                 size_t workspace_bytes, thz_stream_t stream) {
  f64::RscPlan64 p;
  int e = f64::rsc_args(d, &p);
  if (e) return e;
  if (!in || !out) return fail(THZ_E_ARG, "null data pointer");
  const f64::ConvGeom g = f64::conv_geom(p.a, 1);
  if (!workspace || workspace_bytes < p.kt + p.kf + g.total())
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, p.kt + p.kf + g.total());
  if ((e = f64::lds_attr())) return e;
  hipStream_t s = (hipStream_t)stream;
  const int Ph = p.a.Ph, Pw = p.a.Pw;
  f64::DPlan pw, ph;
  if ((e = f64::get_plan(Pw, &pw))) return e;
  if ((e = f64::get_plan(Ph, &ph))) return e;
  char* w = (char*)workspace;
  double2* K = (double2*)w;
  double2* KF = (double2*)(w + p.kt);
  {
    KernelTimer kt("rsc64_kernel_fft", s);
    const size_t n = (size_t)Ph * Pw;
    hipLaunchKernelGGL(f64::rsc_spatial, dim3((unsigned)((n + 255) / 256), d->C), dim3(256), 0, s, K, Ph, Pw, d->dx,
                       d->z, p.a);
    THZ_LAUNCH_CHECK();
    // FFT2(K): rows in place, then columns in place (stride Pw), then [Ph][Pw] -> [Pw][Ph]
    if ((e = f64::lines(K, K, d->C * Ph, pw, 0, (size_t)Pw, 1, s))) return e;
    for (int c = 0; c < d->C; ++c)
      if ((e = f64::lines(K + (size_t)c * n, K + (size_t)c * n, Pw, ph, 0, 0, Pw, s))) return e;
    hipLaunchKernelGGL(f64::transpose_planes, dim3((unsigned)((n + 255) / 256), d->C), dim3(256), 0, s,
                       (const double2*)K, KF, Ph, Pw);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  f64::ConvArgs a = p.a;
  a.tft = KF;
  return f64::run_conv(a, 1, (const double2*)in, (double2*)out, w + p.kt + p.kf, s);
}

extern "C" int thz_czt64_workspace_size(const thz_czt_desc64* d, size_t* bytes) {
  f64::CztArgs a;
  size_t total = 0;
  int e = f64::czt_args(d, &a, &total);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  *bytes = total;
  return THZ_OK;
}

extern "C" int thz_czt64_forward(const thz_czt_desc64* d, const void* in, void* out, void* workspace,
                                 size_t workspace_bytes, thz_stream_t stream) {
  f64::CztArgs a;
  size_t need = 0;
  int e = f64::czt_args(d, &a, &need);
  if (e) return e;
  if (!in || !out) return fail(THZ_E_ARG, "null data pointer");
  if (!workspace || workspace_bytes < need)
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  if ((e = f64::lds_attr())) return e;
  f64::DPlan pA, pB;
  if ((e = f64::get_plan(a.pa.np2, &pA))) return e;
  if ((e = f64::get_plan(a.pb.np2, &pB))) return e;
  hipStream_t s = (hipStream_t)stream;
  double2* ws = (double2*)workspace;
  double2* V = (double2*)((char*)workspace + f64::a256(a.tabStride * d->C * sizeof(double2)));
  {
    KernelTimer kt("czt64_tables", s);
    const int nA = std::max({a.pa.m, a.pa.M, a.pa.np2}), nB = std::max({a.pb.m, a.pb.M, a.pb.np2});
    hipLaunchKernelGGL(f64::czt_tables, dim3((nA + 255) / 256, d->C), dim3(256), 0, s, a, ws, 0);
    THZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(f64::czt_tables, dim3((nB + 255) / 256, d->C), dim3(256), 0, s, a, ws, 1);
    THZ_LAUNCH_CHECK();
    if ((e = f64::lines(ws + a.ftA, ws + a.ftA, d->C, pA, 0, a.tabStride, 1, s))) return e;
    if ((e = f64::lines(ws + a.ftB, ws + a.ftB, d->C, pB, 0, a.tabStride, 1, s))) return e;
    kt.stop();
  }
  KernelTimer kt("czt64", s);
  if (d->adjoint) {  // G [B, C, outW, outH] -> grad_in [B, C, H, W]: column pass first
    hipLaunchKernelGGL(f64::czt_cols_adj, dim3(a.BC * d->outH), dim3(f64::threads(pB.n)), f64::lds_bytes(pB.n), s,
                       (const double2*)in, V, (const double2*)ws, pB, a);
    THZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(f64::czt_rows_adj, dim3(a.BC * d->H), dim3(f64::threads(pA.n)), f64::lds_bytes(pA.n), s,
                       (const double2*)V, (double2*)out, (const double2*)ws, pA, a);
    THZ_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(f64::czt_rows, dim3(a.BC * d->H), dim3(f64::threads(pA.n)), f64::lds_bytes(pA.n), s,
                       (const double2*)in, V, (const double2*)ws, pA, a);
    THZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(f64::czt_cols, dim3(a.BC * d->outH), dim3(f64::threads(pB.n)), f64::lds_bytes(pB.n), s,
                       (const double2*)V, (double2*)out, (const double2*)ws, pB, a);
    THZ_LAUNCH_CHECK();
  }
  kt.stop();
  return THZ_OK;
}
