// Chirp-z (Bluestein) Rayleigh-Sommerfeld propagation with output zoom, CZT_prop
// (Props/CZT_Prop.py:11-314), for gfx950.
//
// Reference sequence (per wavelength c, Dm = lambda z / dx_in):
//   U0 = E * F(x_in, y_in)                                   RS kernel, :44-57, :238
//   U1 = Bluestein(U0, axis H, fy1, fy2, M = outW)           :243  (output transposed)
//   U2 = Bluestein(U1, axis W, fx1, fx2, M = outH)           :246
//   out = F0(x_out, y_out) * U2 * z * dxo * dyo * lambda     :248
// Bluestein (:132-225): x * A^-j * h[m-1+j] -> FFT_np2 -> * FFT_np2(1/h[0:mp+1]) -> IFFT ->
// rows [m, m+M) -> * h[m-1+l] * M_shift[l], h[t] = W^((t-m+1)^2/2), np2 = 2^ceil(log2(m+M-1)).
//
// The two 1-D transforms act on different axes, so they commute; this build runs the W
// axis first over contiguous rows (pass A, params fx / outH) and the H axis second over the
// blocked-column intermediate (pass B, params fy / outW), producing the reference's
// [B, C, outW, outH] result.  Each pass is one kernel: fused-I/O forward FFT (input chirp and
// RS kernel applied in the first-stage loader), spectrum kept in registers, filter multiply
// in the inverse's first-stage loader, output chirp / M_shift (and F0 for pass B) applied in
// the last-stage storer.  The chirp tables are generated on the device in DOUBLE precision
// (the reference's fp32 complex pow is its dominant error), the filter
// spectra by the same LDS FFT.
//
// Forward passes whose output fits half a 1024-point block (M <= 512) and whose input is long
// (cfg3: m = 2048) run the overlap-add form instead (czt_rows_blk / czt_cols_blk, below): the input
// split into 512-point blocks, each block's 1024-point spectrum accumulated against a precomputed
// block filter spectrum, one inverse per line -- 5 transforms of 1024 points per line where the
// np2 form runs 2 of 4096, on one wavefront per line without workgroup barriers (thz_wfft.hpp).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "thz_common.hpp"
#include "thz_dev.hpp"
#include "thz_wfft.hpp"


namespace thz {

struct BluePass {
  int m, M, np2;
  int ntab;        // length of the 1/h sequence actually used: min(mp + 1, Lh)
  int nb;          // > 0: overlap-add form, nb blocks of CZB_BS inputs (else one np2 transform pair)
  int nrm;         // inverse-transform length whose 1/n the post table carries (np2 or wf::N)
  double f1, f2;   // frequency range
};

struct CztArgs {
  int BC, C, H, W, outH, outW;
  float dx, dy, odx, ody, z;
  BluePass pa, pb;   // pass A: W axis (fx, outH); pass B: H axis (fy, outW)
  int ncbA;          // blocks of CB columns covering the intermediate V's outH columns (allocation)
  // table offsets (in float2) inside the workspace, per wavelength stride; ft* holds the np2 filter
  // spectrum, or for an overlap-add pass the nb block spectra (nb x wf::N)
  size_t preA, postA, ftA, preB, postB, ftB, tabStride;
  const float2* tw1024;  // the 1024-point plan's twiddle table (overlap-add wavefront transforms)
  float lam[THZ_MAX_WAVELENGTHS];
};

// --------------------------------------------------------------------------------------------
// Bluestein parameters in double from the fp32-rounded inputs (Props/CZT_Prop.py:109-116,
// 179-225).
// --------------------------------------------------------------------------------------------
struct BlueD {
  double Dm, D1, D2, thA, thW;
};

__device__ __forceinline__ BlueD blue_params(const BluePass& p, double lam, double z, double dx) {
  BlueD b;
  b.Dm = lam * z / dx;
  const double f1 = p.f1 + b.Dm / 2, f2 = p.f2 + b.Dm / 2;
  const double M = p.M;
  b.D1 = f1 + (M * b.Dm + f2 - f1) / (2 * M);
  b.D2 = f2 + (M * b.Dm + f2 - f1) / (2 * M);
  const double twopi = 6.283185307179586476925;
  b.thA = twopi * b.D1 / b.Dm;
  b.thW = -twopi * (b.D1 - b.D2) / (M * b.Dm);
  return b;
}

// Tables for one pass and one wavelength: pre[j] = A^-j W^(j^2/2), post[l] = W^(l^2/2) *
// M_shift[l] / np2 (the unnormalised inverse FFT's 1/np2 folded in), g[t] = 1/h[t] (FFT'd
// in place afterwards into the filter spectrum).
__global__ void czt_tables(CztArgs a, float2* __restrict__ ws, int pass) {
  const int c = blockIdx.y;
  const BluePass& p = pass == 0 ? a.pa : a.pb;
  const BlueD b = blue_params(p, (double)a.lam[c], (double)a.z, (double)a.dx);
  float2* pre = ws + (pass == 0 ? a.preA : a.preB) + (size_t)c * a.tabStride;
  float2* post = ws + (pass == 0 ? a.postA : a.postB) + (size_t)c * a.tabStride;
  float2* g = ws + (pass == 0 ? a.ftA : a.ftB) + (size_t)c * a.tabStride;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < p.m) {
    const double j = n;
    pre[n] = cis_d(-b.thA * j + b.thW * j * j / 2);
  }
  if (n < p.M) {
    const double l = n;
    const double ell = l / p.M * (b.D2 - b.D1) + b.D1;
    const double shift = -6.283185307179586476925 * ell * (-p.m / 2.0 + 0.5) / b.Dm;
    const float2 v = cis_d(b.thW * l * l / 2 + shift);
    const float s = 1.0f / (float)p.nrm;
    post[n] = make_float2(v.x * s, v.y * s);
  }
  if (n < p.np2 && !p.nb) {
    if (n < p.ntab) {
      const double jj = n - p.m + 1;
      g[n] = cis_d(-b.thW * jj * jj / 2);
    } else {
      g[n] = make_float2(0.f, 0.f);
    }
  }
}

// The intermediate V between the passes: blocked column-major per plane, element (q, h) at
// ((q / CB) * H + h) * CB + q % CB (q < outH, h < H).  The rows pass stores a row's outputs as whole
// 128-B lines; the columns pass's 16 waves of a workgroup read one 16-column block, so each line
// they touch serves all 16.  (Measured against a plain column-major V with the rows pass's outputs
// transposed through LDS into 32-B column sectors: columns 0.24 -> 0.20 ms, rows 0.55 -> 0.62 ms at
// cfg3, so the blocked form stays.)
__device__ __forceinline__ size_t vcol(int q, int h, int H) { return blk(q, h, H); }
constexpr int VHS = CB;  // stride of consecutive h in a column of V

template <int PN>
struct CztGeo {
  static constexpr int T = PN > 0 ? PN / pow2_v(PN) : 0;
};

// ---------------------------------------------------------------------------------------------
// Pass A: rows (W axis).  in [BC][H][W] -> V [BC][q][h], q in [0, outH)
// ---------------------------------------------------------------------------------------------
template <int PN>
__global__ void __launch_bounds__(1024) czt_rows(const float2* __restrict__ in, float2* __restrict__ V,
                                                const float2* __restrict__ ws, FftPlan pl, CztArgs a) {
  extern __shared__ float2 lds[];
  const int row = blockIdx.x;
  const int bc = row / a.H, h = row - bc * a.H;
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float xh = lin(-(float)a.H * a.dx / 2.0f, (float)a.H * a.dx / 2.0f, a.H, h);
  const float2* src = in + ((size_t)bc * a.H + h) * a.W;
  const float2* pre = ws + a.preA + (size_t)c * a.tabStride;
  const float2* post = ws + a.postA + (size_t)c * a.tabStride;
  const float2* ft = ws + a.ftA + (size_t)c * a.tabStride;
  float2* dst = V + (size_t)bc * a.ncbA * CB * a.H;
  const int m = a.W, M = a.outH;
  const float ylo = -(float)a.W * a.dy / 2.0f, yhi = (float)a.W * a.dy / 2.0f;
  auto load_x = [&](int w) {
    if (w >= m) return make_float2(0.f, 0.f);
    const float2 F = rs_kernel(xh, lin(ylo, yhi, a.W, w), a.z, k, rph);
    return cmul(cmul(src[w], F), pre[w]);
  };
  auto store_y = [&](int j, float2 v) {
    const int q = j - m;
    if (q >= 0 && q < M) dst[vcol(q, h, a.H)] = cmul(v, post[q]);
  };
  int tid = threadIdx.x;
  if constexpr (PN > 0) {
    using S = Pow2Sched<PN>;
    constexpr int TT = CztGeo<PN>::T;
    constexpr int RL = S::radix(S::NST - 1, false);
    constexpr int MBL = PN / RL / TT;
    float2 sp[MBL][RL];
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), pl.tw, tid, blockDim.x);
    auto ld0 = [&](int, int, int idx) { return load_x(idx); };
    auto sv0 = [&](int mm, int r, int, float2 v) { sp[mm][r] = v; };
    fft_pow2_run<false, PN, TT, false>(lds, twl, tid, ld0, sv0);
    asm volatile("" : "+v"(tid));
    auto ld1 = [&](int mm, int r, int idx) { return cmul(sp[mm][r], ft[idx]); };
    auto sv1 = [&](int, int, int j, float2 v) { store_y(j, v); };
    fft_pow2_run<true, PN, TT, true>(lds, twl, tid, ld1, sv1);
  } else {
    const int n = pl.n, nt = blockDim.x;
    for (int j = tid; j < n; j += nt) lds[padx(j)] = load_x(j);
    __syncthreads();
    fft_lds<false>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) lds[padx(j)] = cmul(lds[padx(j)], ft[j]);
    __syncthreads();
    fft_lds<true>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) store_y(j, lds[padx(j)]);
  }
}

// ---------------------------------------------------------------------------------------------
// Pass B: columns (H axis) of V.  -> out [BC][outW][outH]: out[p][q] = F0 * U * z dxo dyo lambda
// ---------------------------------------------------------------------------------------------
template <int PN>
__global__ void __launch_bounds__(1024) czt_cols(const float2* __restrict__ V, float2* __restrict__ out,
                                                const float2* __restrict__ ws, FftPlan pl, CztArgs a) {
  extern __shared__ float2 lds[];
  const int id = xcd_chunk(blockIdx.x, gridDim.x);
  const int bc = id / a.outH, q = id - bc * a.outH;
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float2* col = V + (size_t)bc * a.ncbA * CB * a.H + vcol(q, 0, a.H);
  const float2* pre = ws + a.preB + (size_t)c * a.tabStride;
  const float2* post = ws + a.postB + (size_t)c * a.tabStride;
  const float2* ft = ws + a.ftB + (size_t)c * a.tabStride;
  float2* dst = out + (size_t)bc * a.outW * a.outH + q;
  const int m = a.H, M = a.outW;
  // F0 on the output mesh: Outmeshx[p][q] = x_out[p] (outH, dxo), Outmeshy = y_out[q] (outW, dyo)
  const float yq = lin(-(float)a.outW * a.ody / 2.0f, (float)a.outW * a.ody / 2.0f, a.outW, q);
  const float xlo = -(float)a.outH * a.odx / 2.0f, xhi = (float)a.outH * a.odx / 2.0f;
  const float cst = ((a.z * a.odx) * a.ody) * lam;
  auto load_x = [&](int h) { return h < m ? cmul(col[(size_t)h * VHS], pre[h]) : make_float2(0.f, 0.f); };
  auto store_y = [&](int j, float2 v) {
    const int p = j - m;
    if (p >= 0 && p < M) {
      const float2 F0 = rs_kernel(lin(xlo, xhi, a.outH, p), yq, a.z, k, rph);
      dst[(size_t)p * a.outH] = cscale(cmul(F0, cmul(v, post[p])), cst);
    }
  };
  int tid = threadIdx.x;
  if constexpr (PN > 0) {
    using S = Pow2Sched<PN>;
    constexpr int TT = CztGeo<PN>::T;
    constexpr int RL = S::radix(S::NST - 1, false);
    constexpr int MBL = PN / RL / TT;
    float2 sp[MBL][RL];
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), pl.tw, tid, blockDim.x);
    auto ld0 = [&](int, int, int idx) { return load_x(idx); };
    auto sv0 = [&](int mm, int r, int, float2 v) { sp[mm][r] = v; };
    fft_pow2_run<false, PN, TT, false>(lds, twl, tid, ld0, sv0);
    asm volatile("" : "+v"(tid));
    auto ld1 = [&](int mm, int r, int idx) { return cmul(sp[mm][r], ft[idx]); };
    auto sv1 = [&](int, int, int j, float2 v) { store_y(j, v); };
    fft_pow2_run<true, PN, TT, true>(lds, twl, tid, ld1, sv1);
  } else {
    const int n = pl.n, nt = blockDim.x;
    for (int j = tid; j < n; j += nt) lds[padx(j)] = load_x(j);
    __syncthreads();
    fft_lds<false>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) lds[padx(j)] = cmul(lds[padx(j)], ft[j]);
    __syncthreads();
    fft_lds<true>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) store_y(j, lds[padx(j)]);
  }
}

// ---------------------------------------------------------------------------------------------
// Overlap-add Bluestein (forward passes with M <= CZB_BS).  Per line the kept outputs are
//   y[q] = post[q] sum_{w < m} x'[w] g[q + m - w],   q < M,  x' = x pre,  g = 1/h   (:179-225)
// (a linear correlation: the reference's np2 >= m + M - 1 circular convolution never wraps for the
// kept rows [m, m + M)).  Split the input into nb blocks of CZB_BS = 512: with
// g_b[t] = g[t + m - 512 (b + 1)] (zero outside [0, ntab)),
//   y[q] = post[q] sum_b (x_b (*) g_b)[q + 512],  x_b[u] = x'[512 b + u], u < 512,
// and since 1 <= q + 512 - u <= 1023 the 1024-point circular convolution equals the linear one:
//   y[q] = post[q] / 1024 * IFFT_1024( sum_b FFT_1024(x_b) FFT_1024(g_b) )[q + 512].
// One wavefront per line: nb half-zero forward transforms accumulated in registers against the
// precomputed block spectra G_b (per wavelength, L2-resident), one inverse keeping its upper half.
// For cfg3 (m = 2048, M = 512) that is 5 transforms of 1024 points per line instead of 2 of 4096.
// ---------------------------------------------------------------------------------------------
constexpr int CZB_BS = wf::N / 2;

constexpr int CZB_W = 8;   // rows pass: lines (waves) per workgroup (8: the twiddle tables are gathered once per 8 lines; 4 -> 8 measured 0.59 -> 0.565 ms at cfg3, profiles/r03_czt_probe.txt)
#ifndef CZB_WPE
#define CZB_WPE 4
#endif
constexpr size_t czb_lds_bytes(int waves) { return wf::TAB * sizeof(float2) + waves * wf::IMG * sizeof(float); }

// g_b[t] for every block b and wavelength (then FFT'd in place by fft_rows_strided)
__global__ void czt_blk_tables(CztArgs a, float2* __restrict__ ws, int pass) {
  const int c = blockIdx.z, b = blockIdx.y;
  const BluePass& p = pass == 0 ? a.pa : a.pb;
  const BlueD bd = blue_params(p, (double)a.lam[c], (double)a.z, (double)a.dx);
  float2* g = ws + (pass == 0 ? a.ftA : a.ftB) + ((size_t)c * p.nb + b) * wf::N;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= wf::N) return;
  const int gi = t + p.m - CZB_BS * (b + 1);
  if (gi >= 0 && gi < p.ntab) {
    const double jj = gi - p.m + 1;
    g[t] = cis_d(-bd.thW * jj * jj / 2);
  } else {
    g[t] = make_float2(0.f, 0.f);
  }
}

// one overlap-add line on this wave: ld(w0, u) = x'[w0 + u] for block start w0 and u = lane + 64 r
// (r < 8); st(i, o, v) for output o = lane + 64 i (i < 8; o may exceed M)
template <class Ld, class St>
__device__ __forceinline__ void czb_line(float* img, const wf::Tabs& tw, int lane, int nb,
                                         const float2* __restrict__ G, Ld& ld, St& st) {
  float2 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = make_float2(0.f, 0.f);
  for (int b = 0; b < nb; ++b) {
    // an opaque copy of the lane id per block: otherwise every twiddle / image address of the
    // transform is hoisted out of the block loop and held live across it (register spills)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const float2* Gb = G + (size_t)b * wf::N + ln;
    auto mac = [&](int i, float2 x) { acc[i] = cadd(acc[i], cmul(x, Gb[64 * (i >> 2) + 256 * (i & 3)])); };
    const int w0 = CZB_BS * b;
    auto ldb = [&](int u) { return ld(w0, u); };
    wf::forward<true>(img, tw, ln, ldb, mac);
  }
  auto sv = [&](int q, int j, float2 v) { st(q - 8, j - CZB_BS, v); };
  wf::inverse<8>(img, tw, lane, acc, sv);
}

// pass A (rows, W axis): in [BC][H][W] -> V [BC][q][h], q < outH
// PARTIAL: m is not a multiple of CZB_BS (the last block's loads are bounds-tested)
template <bool PARTIAL>
__global__ void __launch_bounds__(64 * CZB_W) __attribute__((amdgpu_waves_per_eu(CZB_WPE))) czt_rows_blk(const float2* __restrict__ in, float2* __restrict__ V,
                                                           const float2* __restrict__ ws, CztArgs a) {
  extern __shared__ float2 lds[];
  const wf::Tabs tw = wf::fill_tables<64 * CZB_W>(lds, a.tw1024, threadIdx.x);
  float* img = wf::wave_image(lds, threadIdx.x >> 6);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * CZB_W + (threadIdx.x >> 6);
  if (row >= a.BC * a.H) return;
  const int bc = row / a.H, h = row - bc * a.H;
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float xh = lin(-(float)a.H * a.dx / 2.0f, (float)a.H * a.dx / 2.0f, a.H, h);
  const float2* src = in + ((size_t)bc * a.H + h) * a.W;
  const float2* pre = ws + a.preA + (size_t)c * a.tabStride;
  const float2* post = ws + a.postA + (size_t)c * a.tabStride;
  const float2* G = ws + a.ftA + (size_t)c * a.pa.nb * wf::N;
  float2* dst = V + (size_t)bc * a.ncbA * CB * a.H;
  const int m = a.W, M = a.outH;
  const float ylo = -(float)a.W * a.dy / 2.0f, yhi = (float)a.W * a.dy / 2.0f;
  // block-relative pointers: the 8 loads of a block are one address plus immediate offsets
  auto ld = [&](int w0, int u) {
    const int w = w0 + u;
    const float2 F = rs_kernel_fast(xh, lin(ylo, yhi, a.W, w), a.z, k, rph);
    float2 x = make_float2(0.f, 0.f), pw = make_float2(0.f, 0.f);
    if (!PARTIAL || w < m) {
      {  // the input rows are read once: streaming loads keep the L2 for the block spectra and tables
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 t = __builtin_nontemporal_load(reinterpret_cast<const f32x2*>(src + w0) + u);
        x = make_float2(t.x, t.y);
      }
      pw = (pre + w0)[u];
    }
    return cmul(cmul(x, F), pw);
  };
  auto st = [&](int, int q, float2 v) {
    if (q < M) dst[vcol(q, h, a.H)] = cmul(v, post[q]);
  };
  czb_line(img, tw, lane, a.pa.nb, G, ld, st);
}

// pass B (columns, H axis) of V -> out [BC][outW][outH]: out[p][q] = F0 * U * z dxo dyo lambda.
// One workgroup per half of a 16-column block of V (8 columns, one wave per column).  A block's
// CZB_BS rows of the 8 columns are 512 rows x 64 B of V: the workgroup loads them coalesced (16 B
// per lane) and writes each value straight into the image of the wave that transforms its column
// (real parts at [0, 512), imaginary parts at [544, 1056): the first stage reads lane + 64 r, then
// the transform's own exchanges reuse the image), so there is no separate transpose tile.  The
// 53 KB of LDS per workgroup leave room for two workgroups per CU (VGPR-bound at 4 waves / SIMD):
// one workgroup's block loads overlap the other's transforms.  (The round-3 form staged a whole
// 16-column block through a 64 KB tile: one 16-wave workgroup per CU, every block load exposed.)
// The sibling half-blocks of a V block run on one XCD (blockIdx b and b ^ 8), so the L2 merges
// their half-line reads.
constexpr int CZB_WC = CB / 2;  // columns pass: 8 columns (waves) per workgroup
constexpr int CZB_IMS = wf::IMG + 4;  // wave image stride: +4 floats skews the images' banks for the block writes
constexpr int CZB_IMM = 544;          // imaginary parts of the staged column, float offset in the image
// + the block's filter spectrum G_b, shared by the workgroup's 8 columns (one wavelength), staged
// in LDS with the block: its MACs read LDS instead of issuing 16 dependent L2 loads per lane
// (czt_cols 0.176-0.180 -> 0.166-0.168 ms at cfg3, profiles/r06_experiments.txt 8)
constexpr size_t czb_cols_lds_bytes() {
  return wf::TAB * sizeof(float2) + CZB_WC * CZB_IMS * sizeof(float) + wf::N * sizeof(float2);
}

template <bool PARTIAL>
__global__ void __launch_bounds__(64 * CZB_WC) __attribute__((amdgpu_waves_per_eu(CZB_WPE))) czt_cols_blk(const float2* __restrict__ V, float2* __restrict__ out,
                                                           const float2* __restrict__ ws, CztArgs a) {
  static_assert(2 * CZB_WC == CB, "two workgroups per V column block");
  static_assert(CZB_IMM + CZB_BS <= wf::IMG && CZB_IMM % 32 == 0, "staged column inside the wave image");
  extern __shared__ float2 lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* const img0 = reinterpret_cast<float*>(lds + wf::TAB);
  float* img = img0 + wave * CZB_IMS;
  float2* const gl = reinterpret_cast<float2*>(img0 + CZB_WC * CZB_IMS);  // G_b of the current block
  {
    int off = 0;
    asm volatile("" : "+v"(off));  // keep the image base in the address register (wf::wave_image)
    img += off;
  }
  // blockIdx -> (block, half): halves h = 0, 1 of block id at blockIdx (id & 7) | ((id >> 3) << 4) | (h << 3)
  const int bid = (int)blockIdx.x, hb = (bid >> 3) & 1, blkid = (bid & 7) | ((bid >> 4) << 3);
  if (blkid >= a.BC * a.ncbA) return;  // the rounded-up grid's tail (whole workgroup)
  const wf::Tabs tw = wf::fill_tables<64 * CZB_WC>(lds, a.tw1024, threadIdx.x);
  const int bc = blkid / a.ncbA, qb = blkid - bc * a.ncbA;
  const int q = qb * CB + hb * CZB_WC + wave;
  const bool live = q < a.outH;  // every wave takes part in the block loads and barriers
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float4* vblk = reinterpret_cast<const float4*>(V + ((size_t)bc * a.ncbA + qb) * CB * a.H) + hb * (CZB_WC / 2);
  const float2* pre = ws + a.preB + (size_t)c * a.tabStride;
  const float2* post = ws + a.postB + (size_t)c * a.tabStride;
  const float2* G = ws + a.ftB + (size_t)c * a.pb.nb * wf::N;
  float2* dst = out + (size_t)bc * a.outW * a.outH + q;
  const int m = a.H, M = a.outW;
  const float yq = lin(-(float)a.outW * a.ody / 2.0f, (float)a.outW * a.ody / 2.0f, a.outW, q);
  const float xlo = -(float)a.outH * a.odx / 2.0f, xhi = (float)a.outH * a.odx / 2.0f;
  const float cst = ((a.z * a.odx) * a.ody) * lam;
  float2 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = make_float2(0.f, 0.f);
  for (int b = 0; b < a.pb.nb; ++b) {
    const int h0 = CZB_BS * b;
    // the half block's [CZB_BS rows][8 columns]: 4 x 16 B per thread (row e / 4, columns 2 (e % 4) + {0, 1})
    float4 t4[4];
    static_assert(2 * 64 * CZB_WC == wf::N, "two spectrum values per thread");
    const float2* Gs = G + (size_t)b * wf::N + 2 * threadIdx.x;
    const float2 g0 = Gs[0], g1 = Gs[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = (int)threadIdx.x + 64 * CZB_WC * i;
      if (!PARTIAL || h0 + (e >> 2) < m) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const f32x4 t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(vblk) + (size_t)(h0 + (e >> 2)) * (CB / 2) + (e & 3));
        t4[i] = make_float4(t.x, t.y, t.z, t.w);
      } else {
        t4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();  // every wave is done with its image (the previous block's transform)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = (int)threadIdx.x + 64 * CZB_WC * i, row = e >> 2, col = 2 * (e & 3);
      float* d0 = img0 + col * CZB_IMS + row;
      float* d1 = d0 + CZB_IMS;
      d0[0] = t4[i].x;
      d0[CZB_IMM] = t4[i].y;
      d1[0] = t4[i].z;
      d1[CZB_IMM] = t4[i].w;
    }
    gl[2 * threadIdx.x] = g0;
    gl[2 * threadIdx.x + 1] = g1;
    __syncthreads();
    if (live) {
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const float2* Gb = gl + ln;
      auto mac = [&](int i, float2 x) { acc[i] = cadd(acc[i], cmul(x, Gb[64 * (i >> 2) + 256 * (i & 3)])); };
      auto ldb = [&](int u) {
        if (PARTIAL && h0 + u >= m) return make_float2(0.f, 0.f);
        return cmul(make_float2(img[u], img[CZB_IMM + u]), (pre + h0)[u]);
      };
      wf::forward<true>(img, tw, ln, ldb, mac);
    }
  }
  if (!live) return;
  auto st = [&](int, int p, float2 v) {
    if (p < M) {
      const float2 F0 = rs_kernel_fast(lin(xlo, xhi, a.outH, p), yq, a.z, k, rph);
      dst[(size_t)p * a.outH] = cscale(cmul(F0, cmul(v, post[p])), cst);
    }
  };
  auto sv = [&](int qq, int j, float2 v) { st(qq - 8, j - CZB_BS, v); };
  wf::inverse<8>(img, tw, lane, acc, sv);
}

// ---------------------------------------------------------------------------------------------
// Adjoint (autograd backward).  Per pass the forward is y[q] = post[q] sum_w x[w] pre[w]
// g[(q + m - w) mod N] (N = np2, post holding the unnormalised IFFT's 1/N), so
//   x^[w] = conj(pre[w]) IFFT_N( FFT_N(Z) conj(FFT_N(g)) )[w],  Z[(q + m) mod N] = conj(post[q]) y^[q]
// i.e. the same kernel shape with the conj filter spectrum and the windows exchanged; the
// passes run in reverse order (columns first), F0 / the RS input kernel conjugated at the ends.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float2 conjf2(float2 v) { return make_float2(v.x, -v.y); }

// one Bluestein transform of the adjoint in an LDS workgroup: loader / storer on N points
template <int PN, class LdX, class StY>
__device__ __forceinline__ void czt_adj_line(float2* lds, const FftPlan& pl, const float2* __restrict__ ft,
                                             LdX& load_x, StY& store_y) {
  int tid = threadIdx.x;
  if constexpr (PN > 0) {
    using S = Pow2Sched<PN>;
    constexpr int TT = CztGeo<PN>::T;
    constexpr int RL = S::radix(S::NST - 1, false);
    constexpr int MBL = PN / RL / TT;
    float2 sp[MBL][RL];
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), pl.tw, tid, blockDim.x);
    auto ld0 = [&](int, int, int idx) { return load_x(idx); };
    auto sv0 = [&](int mm, int r, int, float2 v) { sp[mm][r] = v; };
    fft_pow2_run<false, PN, TT, false>(lds, twl, tid, ld0, sv0);
    asm volatile("" : "+v"(tid));
    auto ld1 = [&](int mm, int r, int idx) { return cmul(sp[mm][r], conjf2(ft[idx])); };
    auto sv1 = [&](int, int, int j, float2 v) { store_y(j, v); };
    fft_pow2_run<true, PN, TT, true>(lds, twl, tid, ld1, sv1);
  } else {
    const int n = pl.n, nt = blockDim.x;
    for (int j = tid; j < n; j += nt) lds[padx(j)] = load_x(j);
    __syncthreads();
    fft_lds<false>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) lds[padx(j)] = cmul(lds[padx(j)], conjf2(ft[j]));
    __syncthreads();
    fft_lds<true>(lds, pl, tid, nt);
    for (int j = tid; j < n; j += nt) store_y(j, lds[padx(j)]);
  }
}

// adjoint of pass B: G [BC][outW][outH] (column q) -> V^ [BC][q][h]
template <int PN>
__global__ void __launch_bounds__(1024) czt_cols_adj(const float2* __restrict__ G, float2* __restrict__ V,
                                                    const float2* __restrict__ ws, FftPlan pl, CztArgs a) {
  extern __shared__ float2 lds[];
  const int id = xcd_chunk(blockIdx.x, gridDim.x);
  const int bc = id / a.outH, q = id - bc * a.outH;
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float2* pre = ws + a.preB + (size_t)c * a.tabStride;
  const float2* post = ws + a.postB + (size_t)c * a.tabStride;
  const float2* ft = ws + a.ftB + (size_t)c * a.tabStride;
  const float2* src = G + (size_t)bc * a.outW * a.outH + q;
  float2* dst = V + (size_t)bc * a.ncbA * CB * a.H + vcol(q, 0, a.H);
  const int m = a.H, M = a.outW, N = pl.n;
  const float yq = lin(-(float)a.outW * a.ody / 2.0f, (float)a.outW * a.ody / 2.0f, a.outW, q);
  const float xlo = -(float)a.outH * a.odx / 2.0f, xhi = (float)a.outH * a.odx / 2.0f;
  const float cst = ((a.z * a.odx) * a.ody) * lam;
  auto load_x = [&](int j) {
    int p = j - m;
    if (p < 0) p += N;
    if (p >= M) return make_float2(0.f, 0.f);
    const float2 F0 = rs_kernel(lin(xlo, xhi, a.outH, p), yq, a.z, k, rph);
    return cmul(conjf2(post[p]), cscale(cmul(conjf2(F0), src[(size_t)p * a.outH]), cst));
  };
  auto store_y = [&](int j, float2 v) {
    if (j < m) dst[(size_t)j * VHS] = cmul(conjf2(pre[j]), v);
  };
  czt_adj_line<PN>(lds, pl, ft, load_x, store_y);
}

// adjoint of pass A: V^ row h -> grad_in [BC][H][W]
template <int PN>
__global__ void __launch_bounds__(1024) czt_rows_adj(const float2* __restrict__ V, float2* __restrict__ gin,
                                                    const float2* __restrict__ ws, FftPlan pl, CztArgs a) {
  extern __shared__ float2 lds[];
  const int row = blockIdx.x;
  const int bc = row / a.H, h = row - bc * a.H;
  const int c = bc % a.C;
  const float lam = a.lam[c];
  const float k = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, a.z);
  const float xh = lin(-(float)a.H * a.dx / 2.0f, (float)a.H * a.dx / 2.0f, a.H, h);
  const float2* pre = ws + a.preA + (size_t)c * a.tabStride;
  const float2* post = ws + a.postA + (size_t)c * a.tabStride;
  const float2* ft = ws + a.ftA + (size_t)c * a.tabStride;
  const float2* src = V + (size_t)bc * a.ncbA * CB * a.H;
  float2* dst = gin + ((size_t)bc * a.H + h) * a.W;
  const int m = a.W, M = a.outH, N = pl.n;
  const float ylo = -(float)a.W * a.dy / 2.0f, yhi = (float)a.W * a.dy / 2.0f;
  auto load_x = [&](int j) {
    int qq = j - m;
    if (qq < 0) qq += N;
    if (qq >= M) return make_float2(0.f, 0.f);
    return cmul(conjf2(post[qq]), src[vcol(qq, h, a.H)]);
  };
  auto store_y = [&](int j, float2 v) {
    if (j < m) {
      const float2 F = rs_kernel(xh, lin(ylo, yhi, a.W, j), a.z, k, rph);
      dst[j] = cmul(conjf2(F), cmul(conjf2(pre[j]), v));
    }
  };
  czt_adj_line<PN>(lds, pl, ft, load_x, store_y);
}

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
static int np2_of(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Forward passes take the overlap-add form when M fits its half block and it needs fewer
// 1024-point transforms (nb + 1) than the np2 pair costs in 1024-point equivalents (the adjoint
// always runs the np2 form).
static void make_pass(BluePass* p, int m, int M, double lo, double hi, bool allow_blk) {
  p->m = m;
  p->M = M;
  const int mp = m + M - 1;
  p->np2 = np2_of(mp);
  const int Lh = m + std::max(M - 1, m - 1);  // arange(-m+1, max(M-1, m-1)+1)
  p->ntab = std::min(mp + 1, Lh);
  p->f1 = lo;
  p->f2 = hi;
  const int nb = (m + CZB_BS - 1) / CZB_BS;
  const double cost_blk = (nb + 1) * (double)wf::N * 10.0;
  const double cost_np2 = 2.0 * p->np2 * std::log2((double)p->np2);
  p->nb = (allow_blk && M <= CZB_BS && cost_blk < cost_np2) ? nb : 0;
  p->nrm = p->nb ? wf::N : p->np2;
}

static int czt_validate(const thz_czt_desc* d) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || d->outH < 1 || d->outW < 1)
    return fail(THZ_E_ARG, "bad CZT shape");
  if (d->outH != d->outW)
    return fail(THZ_E_ARG, "CZT output must be square: the reference multiplies F0 [outH,outW] with the "
                           "transposed [outW,outH] transform (Props/CZT_Prop.py:248); got %dx%d",
                d->outH, d->outW);
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  if (!d->wavelengths) return fail(THZ_E_ARG, "null wavelengths");
  const int nA = np2_of(d->W + d->outH - 1), nB = np2_of(d->H + d->outW - 1);
  // mp = m + M - 1 a power of two: the reference's np2 = 2^ceil(log2 mp) equals mp, its slice
  // b[m:mp+1] of the np2 inverse then has M - 1 rows and the product with the M-entry chirp
  // h[m-1:mp] raises (Props/CZT_Prop.py:206,211).  Refused here instead of leaving row M - 1 unset.
  if (nA == d->W + d->outH - 1 || nB == d->H + d->outW - 1)
    return fail(THZ_E_ARG, "CZT Bluestein length m + M - 1 = %d is a power of two: the reference's slice "
                           "b[m:mp+1] keeps M - 1 rows there and its product with h[m-1:mp] raises "
                           "(Props/CZT_Prop.py:206,211)",
                nA == d->W + d->outH - 1 ? nA : nB);
  if (nA > FFT_MAX_N || nB > FFT_MAX_N)
    return fail(THZ_E_UNSUPPORTED, "Bluestein length %d/%d exceeds %d", nA, nB, FFT_MAX_N);
  return THZ_OK;
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

static void czt_layout(const thz_czt_desc* d, CztArgs* a, size_t* total) {
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
  // x_out = linspace(-outH dxo/2, outH dxo/2, outH), y_out likewise (Props/CZT_Prop.py:101-102)
  const double xo = (double)(float)((float)d->outH * d->odx / 2.0f);
  const double yo = (double)(float)((float)d->outW * d->ody / 2.0f);
  make_pass(&a->pa, d->W, d->outH, -xo, xo, !d->adjoint);  // second reference Bluestein (:246): fx, outH
  make_pass(&a->pb, d->H, d->outW, -yo, yo, !d->adjoint);  // first reference Bluestein (:243): fy, outW
  a->ncbA = (d->outH + CB - 1) / CB;
  size_t off = 0;
  auto take = [&](size_t n) {
    size_t o = off;
    off += (n + 31) & ~(size_t)31;
    return o;
  };
  a->preA = take(a->pa.m);
  a->postA = take(a->pa.M);
  a->ftA = a->pa.nb ? 0 : take(a->pa.np2);
  a->preB = take(a->pb.m);
  a->postB = take(a->pb.M);
  a->ftB = a->pb.nb ? 0 : take(a->pb.np2);
  a->tabStride = off;
  // overlap-add block spectra: [C][nb][wf::N] after the per-wavelength tables (one FFT launch)
  size_t gend = (size_t)a->tabStride * d->C;
  if (a->pa.nb) {
    a->ftA = gend;
    gend += (size_t)d->C * a->pa.nb * wf::N;
  }
  if (a->pb.nb) {
    a->ftB = gend;
    gend += (size_t)d->C * a->pb.nb * wf::N;
  }
  for (int c = 0; c < d->C; ++c) a->lam[c] = d->wavelengths[c];
  const size_t tab = a256(gend * sizeof(float2));
  const size_t vbytes = a256((size_t)a->BC * a->ncbA * CB * d->H * sizeof(float2));
  *total = tab + vbytes;
}

static int czt_pow2(int n) {
  switch (n) {
    case 1024: case 2048: case 4096: case 8192: case 16384: return n;
    default: return 0;
  }
}

#define THZ_CZT_SWITCH(n, KER, ...)                                                     \
  switch (czt_pow2(n)) {                                                                 \
    case 1024: hipLaunchKernelGGL(KER<1024>, __VA_ARGS__); break;                        \
    case 2048: hipLaunchKernelGGL(KER<2048>, __VA_ARGS__); break;                        \
    case 4096: hipLaunchKernelGGL(KER<4096>, __VA_ARGS__); break;                        \
    case 8192: hipLaunchKernelGGL(KER<8192>, __VA_ARGS__); break;                        \
    case 16384: hipLaunchKernelGGL(KER<16384>, __VA_ARGS__); break;                      \
    default: hipLaunchKernelGGL(KER<0>, __VA_ARGS__); break;                             \
  }

static int czt_lds_attr() {
  static std::once_flag once;
  static hipError_t err = hipSuccess;
  std::call_once(once, [] {
    const int mx = (int)std::max(fft_lds_bytes(FFT_MAX_N), czb_cols_lds_bytes());
    const void* ks[] = {
        (const void*)czt_rows_blk<false>, (const void*)czt_rows_blk<true>,
        (const void*)czt_cols_blk<false>, (const void*)czt_cols_blk<true>,
        (const void*)czt_rows<0>,     (const void*)czt_rows<1024>, (const void*)czt_rows<2048>,
        (const void*)czt_rows<4096>,  (const void*)czt_rows<8192>, (const void*)czt_rows<16384>,
        (const void*)czt_cols<0>,     (const void*)czt_cols<1024>, (const void*)czt_cols<2048>,
        (const void*)czt_cols<4096>,  (const void*)czt_cols<8192>, (const void*)czt_cols<16384>,
        (const void*)czt_rows_adj<0>,  (const void*)czt_rows_adj<1024>, (const void*)czt_rows_adj<2048>,
        (const void*)czt_rows_adj<4096>, (const void*)czt_rows_adj<8192>, (const void*)czt_rows_adj<16384>,
        (const void*)czt_cols_adj<0>,  (const void*)czt_cols_adj<1024>, (const void*)czt_cols_adj<2048>,
        (const void*)czt_cols_adj<4096>, (const void*)czt_cols_adj<8192>, (const void*)czt_cols_adj<16384>};
    for (const void* k : ks) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      if (e != hipSuccess) err = e;
    }
  });
  if (err != hipSuccess) return fail(THZ_E_HIP, "hipFuncSetAttribute: %s", hipGetErrorString(err));
  return THZ_OK;
}

static int threads_pow2_or(int n) { return czt_pow2(n) ? n / pow2_v(n) : fft_threads(n); }

// Per-device cache of a call's tables -- pre / post chirps and the filter spectra of both passes,
// the workspace's leading table region -- keyed by everything they depend on (geometry, spacings,
// z, wavelengths, direction): SURVEY §8(b)'s immutable per-device caches.  A repeated call with
// the same key skips the six table launches (≈ 35 µs of a 0.85 ms cfg3 call).  Entries live for
// the process; past CZT_TAB_MAX entries or bytes a call builds its tables in its workspace as
// before, and so does a call made while its stream is being captured into a graph.
struct CztTabKey {
  int dev, adjoint, H, W, outH, outW, C;
  float dx, dy, odx, ody, z;
  std::vector<float> lam;
  bool operator<(const CztTabKey& o) const {
    return std::tie(dev, adjoint, H, W, outH, outW, C, dx, dy, odx, ody, z, lam) <
           std::tie(o.dev, o.adjoint, o.H, o.W, o.outH, o.outW, o.C, o.dx, o.dy, o.odx, o.ody, o.z, o.lam);
  }
};
struct CztTabEntry {
  float2* buf;
  hipEvent_t ready;  // recorded after the tables are built (another stream's call waits on it)
};
constexpr int CZT_TAB_MAX = 64;
constexpr size_t CZT_TAB_MAX_BYTES = (size_t)512 << 20;
static std::mutex g_tab_mu;
static std::map<CztTabKey, CztTabEntry> g_tabs;
static size_t g_tab_bytes = 0;

static size_t czt_tab_bytes(const CztArgs& a, int C) {
  size_t gend = (size_t)a.tabStride * C;
  if (a.pa.nb) gend += (size_t)C * a.pa.nb * wf::N;
  if (a.pb.nb) gend += (size_t)C * a.pb.nb * wf::N;
  return a256(gend * sizeof(float2));
}

// Build the tables of one call into tab (its workspace, or a cache buffer).
static int czt_build_tables(const CztArgs& a, const thz_czt_desc* d, float2* tab, hipStream_t s) {
  int e;
  {
    KernelTimer kt("czt_tables", s);
    const int nA = std::max({a.pa.m, a.pa.M, a.pa.np2}), nB = std::max({a.pb.m, a.pb.M, a.pb.np2});
    hipLaunchKernelGGL(czt_tables, dim3((nA + 255) / 256, d->C), dim3(256), 0, s, a, tab, 0);
    THZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(czt_tables, dim3((nB + 255) / 256, d->C), dim3(256), 0, s, a, tab, 1);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  // filter spectra in place, one launch per axis: FFT_np2(1/h) (one row per wavelength) or, for an
  // overlap-add pass, FFT_1024 of each block's g_b (nb rows per wavelength)
  const BluePass* ps[2] = {&a.pa, &a.pb};
  const size_t fts[2] = {a.ftA, a.ftB};
  for (int ax = 0; ax < 2; ++ax) {
    const BluePass& p = *ps[ax];
    if (p.nb) {
      hipLaunchKernelGGL(czt_blk_tables, dim3(wf::N / 256, p.nb, d->C), dim3(256), 0, s, a, tab, ax);
      THZ_LAUNCH_CHECK();
      if ((e = fft_rows_strided(tab + fts[ax], tab + fts[ax], d->C * p.nb, wf::N, (size_t)wf::N, 0, s))) return e;
    } else if ((e = fft_rows_strided(tab + fts[ax], tab + fts[ax], d->C, p.np2, (size_t)a.tabStride, 0, s))) {
      return e;
    }
  }
  return THZ_OK;
}

// The tables for this call: a cached buffer (built on first use), or its own workspace.
static int czt_tables_for(const CztArgs& a, const thz_czt_desc* d, float2* ws, hipStream_t s, const float2** tab) {
  *tab = ws;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  THZ_HIP_CHECK(hipStreamIsCapturing(s, &cs));
  int dev = 0;
  THZ_HIP_CHECK(hipGetDevice(&dev));
  if (cs != hipStreamCaptureStatusNone) return czt_build_tables(a, d, ws, s);
  CztTabKey k{dev, d->adjoint, d->H, d->W, d->outH, d->outW, d->C, d->dx, d->dy, d->odx, d->ody, d->z,
              std::vector<float>(d->wavelengths, d->wavelengths + d->C)};
  const size_t bytes = czt_tab_bytes(a, d->C);
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto it = g_tabs.find(k);
  if (it != g_tabs.end()) {
    THZ_HIP_CHECK(hipStreamWaitEvent(s, it->second.ready, 0));
    *tab = it->second.buf;
    return THZ_OK;
  }
  if ((int)g_tabs.size() >= CZT_TAB_MAX || g_tab_bytes + bytes > CZT_TAB_MAX_BYTES)
    return czt_build_tables(a, d, ws, s);
  CztTabEntry en{};
  // A cache entry needs a hipMalloc and an event; both are refused while another thread has a
  // stream in a global-mode capture (or when memory is short).  Then this call builds its tables in
  // its own workspace, as an uncached call does, instead of failing.
  if (hipEventCreateWithFlags(&en.ready, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return czt_build_tables(a, d, ws, s);
  }
  if (hipMalloc(&en.buf, bytes) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipEventDestroy(en.ready);
    return czt_build_tables(a, d, ws, s);
  }
  int e = czt_build_tables(a, d, en.buf, s);
  if (e == THZ_OK) e = hipEventRecord(en.ready, s) == hipSuccess ? THZ_OK : THZ_E_HIP;
  if (e != THZ_OK) {
    // the buffer may still be in use by launched work: keep it (leaked) rather than free it early
    return e == THZ_E_HIP ? fail(THZ_E_HIP, "CZT table cache event") : e;
  }
  g_tabs.emplace(std::move(k), en);
  g_tab_bytes += bytes;
  *tab = en.buf;
  return THZ_OK;
}

}  // namespace thz

using namespace thz;

extern "C" int thz_czt_workspace_size(const thz_czt_desc* d, size_t* bytes) {
  int e = czt_validate(d);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  CztArgs a;
  czt_layout(d, &a, bytes);
  return THZ_OK;
}

extern "C" int thz_czt_forward(const thz_czt_desc* d, const void* in, void* out, void* workspace,
                               size_t workspace_bytes, thz_stream_t stream) {
  int e = czt_validate(d);
  if (e) return e;
  if (!in || !out) return fail(THZ_E_ARG, "null data pointer");
  CztArgs a{};
  size_t need = 0;
  czt_layout(d, &a, &need);
  if (!workspace || workspace_bytes < need)
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  if ((e = czt_lds_attr())) return e;
  FftPlan plA, plB, pl1024;
  if ((e = get_plan(1024, &pl1024))) return e;
  a.tw1024 = pl1024.tw;
  if ((e = get_plan(a.pa.np2, &plA))) return e;
  if ((e = get_plan(a.pb.np2, &plB))) return e;
  hipStream_t s = (hipStream_t)stream;
  float2* V = (float2*)((char*)workspace + need - a256((size_t)a.BC * a.ncbA * CB * d->H * sizeof(float2)));
  const float2* ws = nullptr;  // the tables: cached, or built in the workspace's leading region
  if ((e = czt_tables_for(a, d, (float2*)workspace, s, &ws))) return e;
  if (d->adjoint) {  // G [B, C, outW, outH] -> grad_in [B, C, H, W]: column pass first
    KernelTimer kt("czt_adjoint", s);
    THZ_CZT_SWITCH(a.pb.np2, czt_cols_adj, dim3(a.BC * d->outH), dim3(threads_pow2_or(a.pb.np2)),
                   fft_lds_bytes_io(a.pb.np2), s, (const float2*)in, V, ws, plB, a);
    THZ_LAUNCH_CHECK();
    THZ_CZT_SWITCH(a.pa.np2, czt_rows_adj, dim3(a.BC * d->H), dim3(threads_pow2_or(a.pa.np2)),
                   fft_lds_bytes_io(a.pa.np2), s, (const float2*)V, (float2*)out, ws, plA, a);
    THZ_LAUNCH_CHECK();
    kt.stop();
    return THZ_OK;
  }
  {
    KernelTimer kt("czt_rows", s);
    if (a.pa.nb) {
      hipLaunchKernelGGL(d->W % CZB_BS ? czt_rows_blk<true> : czt_rows_blk<false>, dim3((a.BC * d->H + CZB_W - 1) / CZB_W), dim3(64 * CZB_W), czb_lds_bytes(CZB_W), s,
                         (const float2*)in, V, ws, a);
    } else {
      THZ_CZT_SWITCH(a.pa.np2, czt_rows, dim3(a.BC * d->H), dim3(threads_pow2_or(a.pa.np2)),
                     fft_lds_bytes_io(a.pa.np2), s, (const float2*)in, V, ws, plA, a);
    }
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  {
    KernelTimer kt("czt_cols", s);
    if (a.pb.nb) {
      // two half-block workgroups per V block; the grid rounded up to whole runs of 16 ids (sibling
      // halves b and b ^ 8), the ids past the last block exit at once
      hipLaunchKernelGGL(d->H % CZB_BS ? czt_cols_blk<true> : czt_cols_blk<false>, dim3((a.BC * a.ncbA + 7) / 8 * 16), dim3(64 * CZB_WC), czb_cols_lds_bytes(),
                         s, (const float2*)V, (float2*)out, ws, a);
    } else {
      THZ_CZT_SWITCH(a.pb.np2, czt_cols, dim3(a.BC * d->outH), dim3(threads_pow2_or(a.pb.np2)),
                     fft_lds_bytes_io(a.pb.np2), s, (const float2*)V, (float2*)out, ws, plB, a);
    }
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  return THZ_OK;
}
