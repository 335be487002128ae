// Band-limited angular-spectrum propagation (Props/ASM_Prop.py:17-378) for gfx950.
//
// The reference computes crop(ift2(ft2(pad x) * H_centred)).  The four fftshifts cancel
// against the centred grid, so this is crop(IFFT2(FFT2(pad x) * H_nat))
// with H evaluated on the natural (fftfreq) index order.  It runs as three LDS passes
// with NO materialised padding, transfer function or shifts:
//
//   K1 rows_fwd  : per input row, length-Pw FFT of the zero-padded row; keep only the
//                  spectral column band |m_y| <= J that can be non-zero (evanescent and
//                  band-limit cut-offs, computed on the host), store column-major
//                  T[bc][c][h] so the column pass reads contiguous memory.
//   K2 cols      : per (bc, band column c): length-Ph FFT of the zero-padded column,
//                  then for each z of the chunk: x H_z(kx, ky) evaluated on the fly
//                  (fp32, same operation order as the reference, contraction off),
//                  inverse FFT, keep the Ho cropped rows, scale 1/(Ph Pw).  The spectrum
//                  is kept in registers across the z loop (forward FFT once per column).
//   K3 rows_inv  : per output row, gather the band (zero elsewhere), length-Pw inverse
//                  FFT, keep the Wo cropped columns, write out[z][b][c][h][w].
//
// The adjoint (autograd backward) is the same pipeline with conj(H) and the input and
// output windows exchanged.
#include <algorithm>
#include <map>
#include <mutex>
#include <cmath>
#include <cstdlib>
#include <tuple>
#include <vector>

#include "thz_common.hpp"
#include "thz_dev.hpp"
#include "thz_wfft.hpp"


namespace thz {

// non-temporal (streaming) 8-byte store
__device__ __forceinline__ void st_stream(float2* p, float2 v) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(f32x2{v.x, v.y}, reinterpret_cast<f32x2*>(p));
}

constexpr float TWO_PI_F = 6.283185307179586f;  // (float)(2*pi), as torch casts the python scalar

struct AsmArgs {
  int BC, C;
  int Ph, Pw;
  int in_r0, in_c0, Hin, Win;     // input window inside the padded plane
  int out_r0, out_c0, Hout, Wout; // output window
  int ncols, J;                   // kept spectral columns, m_y = c - J
  int ncb;                        // column blocks of CB columns (blocked T layout)
  int ncbu;                       // column blocks of CBU columns (blocked U layout)
  int nz, zoff;                   // z-planes in this chunk, offset into zv
  int kfull, kparts;              // K2 tasks: kfull whole columns, then the rest split in kparts z-ranges
  int bl, adjoint;
  // adjoint over Z planes in one pipeline (autograd backward of a multi-plane forward): K1 runs
  // over the chunk's nz input planes (T holds nz planes), K2 sums FFT(T_z) conj(H_z) over them
  // into one spectrum per column and inverts once (zacc: add into U, for the chunks after the
  // first), K3 runs once on the single summed plane
  int zsum, zacc;
  // 1: the power-of-two column pass may take the plane recurrence where its planes allow it
  // (asm_cols_body decides per column; 0 = THZ_K2_RECURRENCE=0, the per-plane sincos everywhere)
  int zrec;
  float dx, dy, scale;
  const float2* tft;  // RSC: column-major transfer-function table [C][ncols][Ph] (nullptr: analytic ASM)
  int vec;            // VRS: plane b == 2 is Ez = (Ex x + Ey y) / r computed in the row pass
  float zr;           // VRS: z of the Ez grid
  float* sqt;         // mixed-radix K2: sqrt(k^2 - Kx^2 - Ky^2) per [C][ncols][Ph] (asm_tf_tables)
  int* mzt;           // mixed-radix K2: kept-row bound M_z per [C][ncols][nz] of the current z-chunk
  // fused DOE modulation in the row pass (thz_asm_forward_modulated): the input row is field * t_c(h)
  const float* mod_h;   // height map [mod_hs][mod_ws] (nullptr: no modulation)
  const float* mod_u;   // U[0,1) height-noise draw, same shape (nullptr: no noise)
  float* mod_hfull;     // optional: the noisy, upsampled height map [Hin][Win]
  int mod_hs, mod_ws;
  float mod_tol, mod_eps, mod_tand;
  const unsigned* mod_rng;  // device generator state for the height noise when mod_u is null
  unsigned mod_rng_stream;
  // fused |E|^2 -> normalize -> MSE in K3's storer (thz_asm_forward_loss, Z == 1): ls.stats
  // non-null; K1 zeroes its accumulators
  LossSink ls;
  // adjoint of the fused loss (thz_asm_adjoint_loss): the row pass's input is the loss gradient
  // dL/dE at the forward output lg_field (thz_intensity_mse_backward's formula), plus the out
  // cotangent `in` when that is given
  const float2* lg_field;
  const float* lg_gloss;
  const float* lg_target;
  const float* lg_stats;
  int lg_tB, lg_tC;
  float lg_two_inv_n;
  // mixed-radix K2 tables of the first z-chunk computed by tab_blocks extra K1 workgroups
  int tab_blocks;
  // thz_asm_desc.window_mask: 1 = multiply the K3 stores by the mask (forward), 2 = the K1 loads
  // (adjoint input); apm is the mask on that grid
  int ap_side;
  ApertureArgs apm;
  const float* zdev;  // thz_asm_desc.z_dev: the plane distances in device memory (nullptr: zv)
  float lam[THZ_MAX_WAVELENGTHS];
  float zv[THZ_MAX_Z];
};

// plane distance i of the call: from device memory when the caller gave z_dev (graph-replayable)
__device__ __forceinline__ float zval(const AsmArgs& a, int i) { return a.zdev ? a.zdev[i] : a.zv[i]; }


// Per-(wavelength, z) scalars of the transfer function, fp32 with the reference's
// operation order (Props/ASM_Prop.py:253, 290-294, 303-304).
struct TfScalars {
  float z, kl2, A, Bv, kxm, kym;
};

#pragma clang fp contract(off)
__device__ __forceinline__ TfScalars tf_scalars(const AsmArgs& a, float lam, float z) {
  TfScalars s;
  s.z = z;
  const float kl = TWO_PI_F / lam;
  s.kl2 = kl * kl;
  const float du = ((TWO_PI_F / a.dx) / (float)(2 * a.Ph)) / TWO_PI_F;
  const float dv = ((TWO_PI_F / a.dy) / (float)(2 * a.Ph)) / TWO_PI_F;  // Ph for v too (:291)
  const float tu = (2.0f * du) * z;
  const float tv = (2.0f * dv) * z;
  const float ul = (1.0f / sqrtf(tu * tu + 1.0f)) / lam;
  const float vl = (1.0f / sqrtf(tv * tv + 1.0f)) / lam;
  const float au = TWO_PI_F * ul, av = TWO_PI_F * vl;
  s.A = au * au;
  s.Bv = av * av;
  const float lx = (float)a.Ph * a.dx, ly = (float)a.Ph * a.dy;  // length_y uses Ph (:275)
  const float ax = (2.0f * (1.0f / lx)) * z, ay = (2.0f * (1.0f / ly)) * z;
  s.kxm = (TWO_PI_F / sqrtf(ax * ax + 1.0f)) / lam;
  s.kym = (TWO_PI_F / sqrtf(ay * ay + 1.0f)) / lam;
  return s;
}

__device__ __forceinline__ float kfreq(int m, int P, float d) { return (TWO_PI_F * ((float)m / (float)P)) / d; }
// single IEEE operations that must not be fused with neighbours (contraction is off here)
__device__ __forceinline__ float tf_mul(float x, float y) { return x * y; }
__device__ __forceinline__ float tf_add(float x, float y) { return x + y; }
__device__ __forceinline__ float tf_sub(float x, float y) { return x - y; }
__device__ __forceinline__ float tf_div(float x, float y) { return x / y; }



// Mask of H at spectral row m (Kx = kfreq(m)) for the column Ky: exactly the tests of
// tf_value below, in the same fp32 operation order.
__device__ __forceinline__ bool tf_pass(int bl, int Ph, float dx, const TfScalars& s, float Ky, int m) {
  const float Kx = kfreq(m, Ph, dx);
  const float Kx2 = Kx * Kx, Ky2 = Ky * Ky;
  const float d = s.kl2 - (Kx2 + Ky2);
  if (d < 0.0f) return false;
  if (bl == THZ_BANDLIMIT_EXACT) {
    const bool c1 = (Kx2 / s.A + Ky2 / s.kl2) <= 1.0f;
    const bool c2 = (Kx2 / s.kl2 + Ky2 / s.Bv) <= 1.0f;
    return c1 && c2;
  }
  if (bl == THZ_BANDLIMIT_APPROX) return !(fabsf(Kx) > s.kxm || fabsf(Ky) > s.kym);
  return true;
}

// H(kx, ky) = exp(i z sqrt(k^2 - K^2)) with the evanescent and band-limit masks
// (Props/ASM_Prop.py:245-306).  conj for the adjoint.
__device__ __forceinline__ float2 tf_value(const AsmArgs& a, const TfScalars& s, float Kx, float Ky) {
  const float Kx2 = Kx * Kx, Ky2 = Ky * Ky;
  const float K2 = Kx2 + Ky2;
  const float d = s.kl2 - K2;
  if (d < 0.0f) return make_float2(0.f, 0.f);
  if (a.bl == THZ_BANDLIMIT_EXACT) {
    const bool c1 = (Kx2 / s.A + Ky2 / s.kl2) <= 1.0f;
    const bool c2 = (Kx2 / s.kl2 + Ky2 / s.Bv) <= 1.0f;
    if (!(c1 && c2)) return make_float2(0.f, 0.f);
  } else if (a.bl == THZ_BANDLIMIT_APPROX) {
    if (fabsf(Kx) > s.kxm || fabsf(Ky) > s.kym) return make_float2(0.f, 0.f);
  }
  const float ang = s.z * sqrtf(d);
  float sn, cs;
  sincos_rad(ang, &sn, &cs);
  return make_float2(cs, a.adjoint ? -sn : sn);
}
#pragma clang fp contract(on)

// PN > 0: compile-time power-of-two transform with fused global I/O (blockDim == PN / FFT_MAXV):
// the first Stockham stage reads its operands straight from global memory and the last
// stage writes its results straight to global memory (coalesced in both cases), so a
// transform costs NST-1 LDS round trips instead of NST+1.  PN == 0: runtime mixed-radix
// plan, data staged through LDS.
template <int PN>
struct Geo {
  static constexpr int T = PN > 0 ? PN / pow2_v(PN) : 0;
};

// Compile-time mixed-radix sizes (MxPlan, one 64-thread workgroup per transform): the P = 300
// grid of the cfg4 / cfg5 layers.  Other non-power-of-two sizes run the runtime plan.
constexpr int MX_T = 64;
// threads of a compile-time mixed-radix transform: one wave for 300 (the radix-5 stages' 60
// butterflies on one lane each), two waves for 500 (its radix-5 stages' 100 and radix-4 stage's 125
// butterflies one per lane: on one wave, two per lane, the row and column passes spilled)
__host__ __device__ constexpr int mx_threads(int n) { return n == 500 ? 128 : MX_T; }
// waves per SIMD of the mixed-radix column pass: 6 lets it keep its 70 VGPRs (8 spilled 5 of them
// to scratch): cfg5 chained batch 256 0.986 -> 0.952 ms, dual-plane 0.080 -> 0.077 ms per step,
// batch 32 0.290 -> 0.296 (profiles/r05_experiments.txt 4)
constexpr int MX_WPE = 6;
__host__ __device__ constexpr bool is_mx(int n) { return n == Mx300::N || n == Mx500::N; }

__device__ __forceinline__ int band_col(int j, int P, int J, int ncols) {
  const int c = freq_index(j, P) + J;
  return (c >= 0 && c < ncols) ? c : -1;
}

// ---------------------------------------------------------------------------------------------
// K1: row FFT of the zero-padded input rows -> band columns, column-major T[bc][c][h]
// ---------------------------------------------------------------------------------------------
#pragma clang fp contract(off)
__device__ __forceinline__ float2 vrs_ez(float2 ex, float2 ey, float x, float y, float z) {
  const float r = sqrtf(x * x + y * y + z * z);
  return make_float2((ex.x * x) / r + (ey.x * y) / r, (ex.y * x) / r + (ey.y * y) / r);
}
#pragma clang fp contract(on)

template <int PN>
__device__ __forceinline__ void tf_tables_body(const AsmArgs& a, int blk, int with_sq);
// The K1 input element s of row h of plane `plane` (s < Win): the field, or what the fused
// loaders make of it -- the loss gradient of the adjoint of the fused loss, the DOE modulation
// t_c(h + noise) (writing the noisy height map once), or the VRS Ez plane.
// AP: apply the window mask of the adjoint's input (only the 300-point row pass carries it: the
// runtime test costs the 64-VGPR power-of-two row kernels registers)
template <bool AP>
struct RowSrc {
  const AsmArgs& a;
  const float2* in;
  const float2* src;
  int h, bc;
  bool ez;
  const float2 *sx, *sy;
  float xh;
  int hsrc;
  float lam_c;
  const float2* lg_row = nullptr;
  const float* lg_t = nullptr;
  float lg_m = 0.f, lg_S = 0.f, lg_g = 0.f;
  int lg_am = -1;
  __device__ __forceinline__ RowSrc(const AsmArgs& a_, const float2* in_, int plane, int h_) : a(a_), in(in_), h(h_) {
    bc = plane % a.BC;
    src = in + ((size_t)((a.zsum ? a.zoff * a.BC : 0) + plane) * a.Hin + h) * a.Win;
    // VRS (Props/RSC_Prop.py:294-303): plane b = 2 is Ez = Ex x / r + Ey y / r on the unpadded
    // grid linspace(-N dx/2, N dx/2, N) (dx on both axes, :83-84)
    ez = a.vec && bc / a.C == 2;
    sx = in + ((size_t)(bc % a.C) * a.Hin + h) * a.Win;
    sy = in + ((size_t)(a.C + bc % a.C) * a.Hin + h) * a.Win;
    xh = ez ? lin(-(float)a.Hin * a.dx / 2.0f, (float)a.Hin * a.dx / 2.0f, a.Hin, h) : 0.f;
    hsrc = a.mod_h ? doe_nearest_src(h, a.mod_hs, a.Hin) * a.mod_ws : 0;
    lam_c = a.lam[bc % a.C];
    // loss gradient rows: field E, target T and the statistics of loss item b (the forward's plane
    // z and batch item: b = z B + batch, the Z-summing adjoint's planes included)
    if (a.lg_field) {
      const int gp = (a.zsum ? a.zoff * a.BC : 0) + plane;
      const int b = gp / a.C, c = gp - b * a.C;
      lg_row = a.lg_field + ((size_t)gp * a.Hin + h) * a.Win;
      const int tb = a.lg_tB == 1 ? 0 : b, tc = a.lg_tC == 1 ? 0 : c;
      lg_t = a.lg_target + (((size_t)tb * a.lg_tC + tc) * a.Hin + h) * a.Win;
      lg_m = a.lg_stats[3 * b];
      lg_S = a.lg_stats[3 * b + 2];
      // the argmax relative to this row's first element (c H + h) W
      lg_am = __float_as_int(a.lg_stats[3 * b + 1]) - (c * a.Hin + h) * a.Win;
      lg_g = a.lg_gloss[0] * a.lg_two_inv_n;
    }
  }
  __device__ __forceinline__ float2 operator()(int s) const {
    const float2 v = value(s);
    // the adjoint of (window mask) * ASM: the mask on the adjoint's input (NaN / inf propagate)
    if constexpr (AP) return a.ap_side == 2 && !aperture_open(a.apm, h, s) ? cscale(v, 0.f) : v;
    else return v;
  }
  __device__ __forceinline__ float2 value(int s) const {
    if (a.lg_field) {  // dL/dE = 2 E dL/dI, dL/dI = g (r / m - [argmax] S / m^2) (mse_backward_kernel)
      const float2 e = lg_row[s];
      const float I = loss_intensity(e);
      const float r = I / lg_m - lg_t[s];
      float dI = lg_g * r / lg_m;
      if (s == lg_am) dI -= lg_g * lg_S / (lg_m * lg_m);
      const float2 gl = make_float2(2.f * dI * e.x, 2.f * dI * e.y);
      return in ? cadd(src[s], gl) : gl;
    }
    if (a.mod_h) {  // DOELayer.modulate fused into the loader (Components/QuantizedDOE.py:92-126)
      const float hv = doe_noisy_h(a.mod_h, a.mod_u, hsrc + doe_nearest_src(s, a.mod_ws, a.Win), a.mod_tol,
                                   a.mod_rng, a.mod_rng_stream);
      if (a.mod_hfull && bc == 0) a.mod_hfull[(size_t)h * a.Win + s] = hv;
      return cmul(src[s], doe_transmission(hv, lam_c, a.mod_eps, a.mod_tand, nullptr));
    }
    if (!ez) return src[s];
    return vrs_ez(sx[s], sy[s], xh, lin(-(float)a.Win * a.dx / 2.0f, (float)a.Win * a.dx / 2.0f, a.Win, s), a.zr);
  }
};


// MID (PN = 300 only): the input window [N/3, 2N/3) of the layers' geometry as constants
template <int PN, bool MID = false>
__global__ void __launch_bounds__(1024) THZ_ROW_ATTR asm_rows_fwd(const float2* __restrict__ in, float2* __restrict__ T,
                                                    FftPlan pw, AsmArgs a) {
  static_assert(!MID || is_mx(PN), "window constants: the 300-point pass");
  extern __shared__ float2 lds[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int nrows = gridDim.x - a.tab_blocks;
  if constexpr (PN == Mx300::N) {
    // the extra workgroups past the rows: the mixed-radix column pass's tables of the first
    // z-chunk (asm_tf_tables, one launch fewer; K2 runs after this kernel on the stream).  The
    // 300-point pass only: in asm_rows_fwd<500> the tables' code made the compiler copy the whole
    // argument block to scratch (1.6 KB per lane); P = 500 launches asm_tf_tables<500> instead
    if ((int)blockIdx.x >= nrows) {
      tf_tables_body<PN>(a, blockIdx.x - nrows, 1);
      return;
    }
  }
  const int row = xcd_rows(blockIdx.x, nrows);
  // plane = zz * BC + bc: one plane (zz = 0) except in the Z-summing adjoint, whose chunk's input
  // planes start at plane zoff * BC of `in`
  const int plane = row / a.Hin, h = row - plane * a.Hin;
  float2* dst = T + (size_t)plane * a.ncb * CB * a.Hin;
  const RowSrc<is_mx(PN)> fetch(a, in, plane, h);  // the 300-point pass carries the adjoint's window mask
  if constexpr (PN > 0 && !is_mx(PN)) {
    // twiddle-table loads first, their LDS writes after the row loads (as in K3)
    constexpr int TT = Geo<PN>::T;
    const auto twf = tw_fetch<PN, TT>(pw.tw, tid);
    const TwLds twl = tw_lds_at<PN>(tw_slot<PN>(lds));
    auto tw_hook = [&]() { tw_store<PN, TT>(tw_slot<PN>(lds), twf, tid); };
    auto ld = [&](int, int, int idx) {
      const int s = idx - a.in_c0;
      return (s >= 0 && s < a.Win) ? fetch(s) : make_float2(0.f, 0.f);
    };
    auto sv = [&](int, int, int j, float2 v) {
      const int c = band_col(j, PN, a.J, a.ncols);
      if (c >= 0) dst[blk(c, h, a.Hin)] = v;
    };
    fft_pow2_run<false, PN, TT, FFT_ROWS>(lds, twl, tid, ld, sv, tw_hook);
  } else if constexpr (is_mx(PN)) {
    constexpr int MT = mx_threads(PN);
    if constexpr (MID) __builtin_assume(tid >= 0 && tid < MT);
    using MP = typename MxOf<PN>::type;
    const auto twr = MP::template twiddles<MT>(pw.tw, tid);
    auto ld = [&](int, int, int idx) {
      const int s = idx - (MID ? PN / 3 : a.in_c0);
      return (s >= 0 && s < (MID ? PN / 3 : a.Win)) ? fetch(s) : make_float2(0.f, 0.f);
    };
    auto sv = [&](int, int, int j, float2 v) {
      const int c = band_col(j, PN, a.J, a.ncols);
      if (c >= 0) dst[blk(c, h, a.Hin)] = v;
    };
    MP::template run<false, MT>(lds, twr, tid, ld, sv);
  } else {
    for (int j = tid; j < a.Pw; j += nt) {
      const int s = j - a.in_c0;
      lds[padx(j)] = (s >= 0 && s < a.Win) ? fetch(s) : make_float2(0.f, 0.f);
    }
    __syncthreads();
    fft_lds<false>(lds, pw, tid, nt);
    for (int c = tid; c < a.ncols; c += nt) {
      int j = c - a.J;
      if (j < 0) j += a.Pw;
      dst[blk(c, h, a.Hin)] = lds[padx(j)];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K2: per band column: FFT(Ph) once, then per z: x H_z, IFFT(Ph), crop, scale -> U[z][bc][c][r]
// ---------------------------------------------------------------------------------------------
// Plane zz of the column task's range [z_lo, z_hi) may be reached from its predecessor in the order
// the planes are run (ascending, or descending from the range's last plane) by the plane recurrence
// of asm_cols_body: with dz the range's first step in that order, the step to zz and eps = step - dz
// are both EXACT fp32 differences (so the recurrence's phase sums to (z_zz - z_first) sq exactly)
// and |eps| k <= 1e-4 rad (so 1 + i eps sq stands for exp(i eps sq) to 5e-9).  Evaluated on the
// device, so a device-resident plane list (thz_asm_desc.z_dev) decides exactly as the host list does.
// register slot of the step factor D of kept spectrum value r (r < 4 or r >= 12): the slots
// [4, 12) of sp, whose values are zero whenever the recurrence runs
__host__ __device__ constexpr int rec_dslot(int r) { return r < 4 ? r + 4 : r - 4; }

// the step from plane zp to plane zc against the range's first step z0 -> z1 (either direction)
__device__ __forceinline__ bool recurrence_step_ok(float z0, float z1, float zp, float zc, float kl) {
  const float dz = z1 - z0, step = zc - zp, eps = step - dz;
  return dz != 0.0f && (double)dz == (double)z1 - (double)z0 && (double)step == (double)zc - (double)zp &&
         (double)eps == (double)step - (double)dz && fabs((double)eps) * (double)kl <= 1e-4;
}

// ZSUM: the Z-summing adjoint's column pass (a separate instantiation, so the forward's register
// allocation is untouched by it).
template <int PN, bool ZSUM>
__device__ __forceinline__ void asm_cols_body(const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph,
                                              AsmArgs a) {
  extern __shared__ float2 lds[];
  // Tasks: the first kfull blocks are whole columns (all nz planes; full dispatch rounds of the
  // resident-workgroup count), the last partial round's columns are split into kparts z-ranges
  // so that round is short instead of a whole column pass on a few CUs.
  int id, z_lo = 0, z_hi = a.nz;
  if ((int)blockIdx.x < a.kfull) {
    id = xcd_chunk(blockIdx.x, a.kfull);
  } else {
    const int t = blockIdx.x - a.kfull, part = t % a.kparts;
    id = a.kfull + t / a.kparts;
    z_lo = part * a.nz / a.kparts;
    z_hi = (part + 1) * a.nz / a.kparts;
  }
  const int bc = id / a.ncols, c = id - bc * a.ncols;
  const int nt = blockDim.x;
  const int Ph = a.Ph;
  const float2* col = T + (size_t)bc * a.ncb * CB * a.Hin + blk(c, 0, a.Hin);
  const float lam = a.lam[bc % a.C];
  const float Ky = kfreq(c - a.J, a.Pw, a.dy);
  // Each phase works from its own opaque copy of threadIdx.x: otherwise the compiler CSEs /
  // hoists the forward and inverse transforms' LDS addresses and twiddle loads across the
  // whole kernel and spills (the two transforms share every twiddle address).
  int tid = threadIdx.x;
  if constexpr (PN > 0) {
    using S = Pow2Sched<PN>;
    constexpr int TT = Geo<PN>::T;
    // forward = small radix first (its twiddle-free first stage is the cheap one, run once per
    // column); inverse = radix-16 first (twiddle-free, run per z) reading exactly the elements the
    // forward's last radix-16 stage left in this thread's registers
    constexpr int RL = S::radix(S::NST - 1, true);   // radix of the forward's last stage
    constexpr int MBL = PN / RL / TT;                // its butterflies per thread
    float2 sp[MBL][RL];                              // spectrum, element i + r*PN/RL
    const TwLds twl = load_tw_lds<PN>(lds + lds_floats2(PN), ph.tw, threadIdx.x, blockDim.x);
    auto ld0 = [&](int, int, int idx) {
      const int s = idx - a.in_r0;
      return (s >= 0 && s < a.Hin) ? col[(size_t)s * CB] : make_float2(0.f, 0.f);
    };
    auto sv0 = [&](int m, int r, int, float2 v) { sp[m][r] = v; };
    if constexpr (!ZSUM) fft_pow2_io<false, PN, TT, true, false, false>(lds, twl, tid, ld0, sv0);
    if (!ZSUM && !a.tft) {
      // 1 / (Ph Pw) is a power of two: scaling the spectrum once per column instead of every
      // output plane is exact
#pragma unroll
      for (int m = 0; m < MBL; ++m)
#pragma unroll
        for (int r = 0; r < RL; ++r) sp[m][r] = cscale(sp[m][r], a.scale);
    }
    if (!ZSUM && a.tft) {  // RSC: tabulated transfer function FFT2(K), one z
      const float2* tcol = a.tft + ((size_t)(bc % a.C) * a.ncols + c) * PN;
      int tz = threadIdx.x;
      asm volatile("" : "+v"(tz));
      auto ld1 = [&](int m, int r, int idx) {
        const float2 t = tcol[idx];
        return cmul(sp[m][r], a.adjoint ? make_float2(t.x, -t.y) : t);
      };
      float2* dst = U + (size_t)bc * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
      auto sv1 = [&](int, int, int j, float2 v) {
        const int r = j - a.out_r0;
        if (r >= 0 && r < a.Hout) dst[u_roff(r)] = cscale(v, a.scale);
      };
      fft_pow2_io<true, PN, TT, FFT_TAIL, false, false>(lds, twl, tz, ld1, sv1);
      return;
    }
    // The evanescent and band-limit masks are monotone in |m_x| (every fp32 operation of
    // Props/ASM_Prop.py:245-306 is monotone), so for each z the kept rows of this column are
    // exactly |m_x| <= M_z.  One lane per z finds M_z by bisection with the exact
    // reference-order tests; the per-element work is then sqrt once per column and one
    // sincos per z.
    int* mz = reinterpret_cast<int*>(lds + lds_floats2(PN) + tw_lds_count(PN));
    const float kl = TWO_PI_F / lam;
    const float kl2 = tf_mul(kl, kl);
    const float Ky2 = tf_mul(Ky, Ky);
    // strided over the chunk: a z_chunk may exceed the workgroup (64 threads at P = 1024)
    int* zok = mz + THZ_MAX_Z;  // plane recurrence allowed at this plane (below)
    // the chunk's z values, staged next to mz for the z-loop of the forward (an LDS read per
    // plane instead of a dependent global load at the top of every plane)
    float* zl = reinterpret_cast<float*>(zok + THZ_MAX_Z);
    for (int zz = tid; zz < z_hi - z_lo; zz += nt) {
      const float zq = zval(a, a.zoff + z_lo + zz);
      if constexpr (!ZSUM) zl[zz] = zq;
      const TfScalars s = tf_scalars(a, lam, zq);
      int lo = -1, hi = PN / 2 + 1;
      const int bl = a.bl, P = a.Ph;
      const float dx = a.dx;
      if (tf_pass(bl, P, dx, s, Ky, 0)) {
        lo = 0;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (tf_pass(bl, P, dx, s, Ky, mid)) lo = mid;
          else hi = mid;
        }
      }
      mz[zz] = lo;
      if constexpr (!ZSUM) {
        // bit 0: plane zz is reached from zz - 1 in ascending order; bit 1: from zz + 1 in
        // descending order (the range's last plane first)
        const int nzr = z_hi - z_lo;
        auto zv = [&](int q) { return zval(a, a.zoff + z_lo + q); };
        const bool fwd = zz == 0 || (nzr >= 2 && recurrence_step_ok(zv(0), zv(1), zv(zz - 1), zv(zz), kl));
        const bool bwd = zz == nzr - 1 ||
                         (nzr >= 2 && recurrence_step_ok(zv(nzr - 1), zv(nzr - 2), zv(zz + 1), zv(zz), kl));
        // bit 2 (on plane 0): |z| falls along the range (a sweep towards the aperture)
        const bool inward = zz == 0 && fabsf(zv(nzr - 1)) < fabsf(zv(0));
        zok[zz] = (fwd ? 1 : 0) | (bwd ? 2 : 0) | (inward ? 4 : 0);
      }
    }
    // sqrt(k^2 - Kx^2 - Ky^2) of the elements this thread holds: z-independent, computed once
    // per column (the per-z work is then one product and one sincos per element)
    float sq[MBL][RL];
#pragma unroll
    for (int m = 0; m < MBL; ++m)
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        const float Kx = kfreq(freq_index(tid + m * TT + r * (PN / RL), PN), PN, a.dx);
        sq[m][r] = sqrtf(fmaxf(tf_sub(kl2, tf_add(tf_mul(Kx, Kx), Ky2)), 0.0f));
      }
    __syncthreads();  // mz visible
    // the plane recurrence (below) for this column?
    bool rec = false, rev = false;
    if constexpr (!ZSUM && RL == 16 && MBL == 1) {
      if (a.zrec && z_hi - z_lo >= 3) {
        // one plane per lane, every wave voting on its own copy (no loop over the planes per
        // thread, no extra barrier); the votes are wave-uniform
        bool okf = true, okr = true, wide = false;
        const int lane = threadIdx.x & 63;
        for (int q0 = 0; q0 < z_hi - z_lo; q0 += 64) {
          const int q = q0 + lane;
          bool pf = true, pr = true, pw = false;
          if (q < z_hi - z_lo) {
            // the band may only narrow in the order the planes are run (an element that leaves
            // it is zeroed in the recurrence for good, below): ascending order for a band that
            // narrows with the plane index (cfg2's increasing z), descending order for one that
            // widens (a decreasing z-sweep)
            const int m = mz[q], mp = q > 0 ? mz[q - 1] : m, zk = zok[q];
            pf = (zk & 1) && m <= mp;
            pr = (zk & 2) && m >= mp;
            pw = m >= PN / 4;
          }
          okf = okf && __ballot(!pf) == 0;
          okr = okr && __ballot(!pr) == 0;
          wide = wide || __ballot(pw) != 0;
        }
        rec = (okf || okr) && !wide;
        // a band constant over the range allows both orders: run the range from its plane nearest
        // the aperture, as every column with a changing band of the same sweep does
        // (read wave-uniform: the plane order, and with it every plane index and z of the loop
        // below, stays in scalar registers)
        const int zk0 = __builtin_amdgcn_readfirstlane(zok[0]);
        rev = rec && okr && (!okf || (zk0 & 4));
      }
    }
    if constexpr (ZSUM) {
      // adjoint over the chunk's planes: sp = sum_z FFT(T_z column) conj(H_z), then one inverse
#pragma unroll
      for (int m = 0; m < MBL; ++m)
#pragma unroll
        for (int r = 0; r < RL; ++r) sp[m][r] = make_float2(0.f, 0.f);
      for (int zz = z_lo; zz < z_hi; ++zz) {
        const float z = zval(a, a.zoff + zz);
        const int M = mz[zz - z_lo];
        const float2* colz = T + ((size_t)zz * a.BC + bc) * a.ncb * CB * a.Hin + blk(c, 0, a.Hin);
        int tz = threadIdx.x;
        asm volatile("" : "+v"(tz));
        auto ldz = [&](int, int, int idx) {
          const int s = idx - a.in_r0;
          return (s >= 0 && s < a.Hin) ? colz[(size_t)s * CB] : make_float2(0.f, 0.f);
        };
        auto acc = [&](int m, int r, int j, float2 v) {
          const int mx = freq_index(j, PN);
          if (mx > M || -mx > M) return;
          float sn, cs;
          sincos_hw(tf_mul(z, sq[m][r]), &sn, &cs);
          sp[m][r] = cadd(sp[m][r], cmul(v, make_float2(cs, -sn)));
        };
        fft_pow2_io<false, PN, TT, true, false, false>(lds, twl, tz, ldz, acc);
      }
#pragma unroll
      for (int m = 0; m < MBL; ++m)
#pragma unroll
        for (int r = 0; r < RL; ++r) sp[m][r] = cscale(sp[m][r], a.scale);
      int tz = threadIdx.x;
      asm volatile("" : "+v"(tz));
      auto ld1 = [&](int m, int r, int) { return sp[m][r]; };
      float2* dst = U + (size_t)bc * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
      auto sv1 = [&](int, int, int j, float2 v) {
        const int r = j - a.out_r0;
        if ((unsigned)r < (unsigned)a.Hout) dst[u_roff(r)] = a.zacc ? cadd(dst[u_roff(r)], v) : v;
      };
      fft_pow2_io<true, PN, TT, FFT_TAIL, false, false>(lds, twl, tz, ld1, sv1);
      return;
    }
    // Plane recurrence (a uniform z-sweep such as cfg2's linspace): instead of one sincos per
    // element per plane, G_j = sp H_{z_j} advances by one complex product per plane,
    //   G_j = G_{j-1} D (1 + i eps_j sq),   D = exp(i dz sq),   eps_j = (z_j - z_{j-1}) - dz,
    // which tracks the given fp32 planes exactly: recurrence_step_ok has checked that every
    // difference is exact in fp32 and |eps_j| k <= 1e-4 rad, so 1 + i theta stands for
    // exp(i theta) to 5e-9.  D is formed in double and rounded once (<= 6e-8 per plane, 4e-6
    // over 64 planes); the first plane run is the sincos form's value bit for bit.  The planes
    // run in the order in which the column's band narrows (ascending z for cfg2; a decreasing
    // sweep runs from the range's last plane), so no element ever re-enters the band.
    // Taken when the column keeps no row with |m_x| >= PN/4 on any plane of the chunk: the
    // inverse's first-stage operands r in [4, 12) are then zero, and the registers of those 8
    // spectrum values hold the 8 step factors D (sp[0][rec_dslot(r)]); sq holds +-sq.  Both forms
    // share one z-loop and one inverse transform on the same registers (as two regions the
    // structurizer kept one form's live-ins live through the other and spilled).
    constexpr bool REC = !ZSUM && RL == 16 && MBL == 1;
    float dz = 0.f, zprev = 0.f;
    int Mprev = -2;  // below every band value (M = -1: no row of the column kept)
    // plane order: ascending, or descending where the recurrence runs the range backwards
    const int zfirst = rev ? z_hi - 1 : z_lo, zstep = rev ? -1 : 1;
    if constexpr (REC) {
      if (rec) {
        const float z0 = zl[zfirst - z_lo];
        dz = zl[zfirst + zstep - z_lo] - z0;
        zprev = z0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (r >= 4 && r < 12) continue;
          float sn, cs;
          sincos_hw(tf_mul(z0, sq[0][r]), &sn, &cs);
          sp[0][r] = cmul(sp[0][r], make_float2(cs, a.adjoint ? -sn : sn));
          const float2 d = cis_dd((double)dz * (double)sq[0][r]);
          sp[0][rec_dslot(r)] = make_float2(d.x, a.adjoint ? -d.y : d.y);
          if (a.adjoint) sq[0][r] = -sq[0][r];
          // one element's double-precision evaluation at a time (all eight interleaved need more
          // registers than the kernel has)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    for (int it = 0; it < z_hi - z_lo; ++it) {
      const int zz = zfirst + it * zstep;
      const float z = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(zl[zz - z_lo])));
      const int M = mz[zz - z_lo];
      if constexpr (REC) {
        if (rec && it > 0) {
          const float eps = tf_sub(tf_sub(z, zprev), dz);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (r >= 4 && r < 12) continue;
            sp[0][r] = cmul(sp[0][r], sp[0][rec_dslot(r)]);
          }
          // the step correction 1 + i eps sq, skipped on a scalar branch where the step is dz
          // exactly (60 of cfg2's 63 steps), where it would leave every value as it is
          if (__builtin_amdgcn_readfirstlane(__float_as_int(eps)) != 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              if (r >= 4 && r < 12) continue;
              const float2 g = sp[0][r];
              const float th = eps * sq[0][r];
              sp[0][r] = make_float2(fmaf(-th, g.y, g.x), fmaf(th, g.x, g.y));
            }
          }
        }
        zprev = z;
      }
      int tz = threadIdx.x;
      asm volatile("" : "+v"(tz));
      const int Ms = __builtin_amdgcn_readfirstlane(M);
      if constexpr (REC) {
        // the band's edge: on the chunk's first plane and wherever the band narrows (a few of
        // cfg2's planes), the elements outside it are zeroed in G itself -- they stay zero through
        // the recurrence's products, and the band never widens again (the eligibility above) --
        // so the loads below need no per-plane mask
        if (rec && Ms != Mprev) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (r >= 4 && r < 12) continue;
            // element tz + r PN/16: m_x = tz + r PN/16 (r < 4), tz + r PN/16 - PN (r >= 12)
            const bool keep = r < 4 ? tz <= Ms - r * (PN / 16) : tz >= PN - r * (PN / 16) - Ms;
            if (!keep) sp[0][r] = make_float2(0.f, 0.f);
          }
        }
        Mprev = Ms;
      }
      // the inverse's first stage (radix RL, L = 1) reads exactly the elements this thread
      // holds in sp: multiply by H_z on the fly in the loader
      // the first stage's operands r in [4, 12) are the rows PN/4 <= |m_x| < 3 PN/4: when this
      // plane's kept band M is below PN/4 (all but the few columns near m_y = 0 at cfg2) they are
      // zero for every thread, and a scalar branch skips their sincos and product
      const bool mid0 = Ms < PN / 4;
      auto ld1 = [&](int m, int r, int idx) {
        if (RL == 16 && r >= 4 && r < 12 && mid0) return make_float2(0.f, 0.f);
        if constexpr (REC) {
          if (rec) return sp[0][r];  // out-of-band elements already zero (above)
        }
        const int mx = freq_index(idx, PN);
        if (mx > M || -mx > M) return make_float2(0.f, 0.f);
        float sn, cs;
        sincos_hw(tf_mul(z, sq[m][r]), &sn, &cs);
        return cmul(sp[m][r], make_float2(cs, a.adjoint ? -sn : sn));
      };
      float2* dst = U + ((size_t)zz * a.BC + bc) * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
      auto sv1 = [&](int, int, int j, float2 v) {
        const int r = j - a.out_r0;
        // (ordinary stores: the 4 column workgroups of a U block fill its 32-B sectors in the L2;
        // streaming stores here ran K2 4.1 -> 13.8 ms)
        if ((unsigned)r < (unsigned)a.Hout) dst[u_roff(r)] = v;
      };
      fft_pow2_io<true, PN, TT, FFT_TAIL, false, false>(lds, twl, tz, ld1, sv1);
    }
  } else {
    if constexpr (ZSUM) {
      // adjoint over the chunk's planes (see the power-of-two branch)
      float2 acc[FFT_MAXV];
#pragma unroll
      for (int m = 0; m < FFT_MAXV; ++m) acc[m] = make_float2(0.f, 0.f);
      for (int zz = z_lo; zz < z_hi; ++zz) {
        const TfScalars s = tf_scalars(a, lam, zval(a, a.zoff + zz));
        const float2* colz = T + ((size_t)zz * a.BC + bc) * a.ncb * CB * a.Hin + blk(c, 0, a.Hin);
        int tm = threadIdx.x;
        asm volatile("" : "+v"(tm));
        __syncthreads();  // the previous plane's readers are done with lds
        for (int i = tm; i < Ph; i += nt) {
          const int si = i - a.in_r0;
          lds[padx(i)] = (si >= 0 && si < a.Hin) ? colz[(size_t)si * CB] : make_float2(0.f, 0.f);
        }
        __syncthreads();
        fft_lds<false>(lds, ph, tm, nt);
#pragma unroll
        for (int m = 0; m < FFT_MAXV; ++m) {
          const int i = tm + m * nt;
          if (i < Ph) acc[m] = cadd(acc[m], cmul(lds[padx(i)], tf_value(a, s, kfreq(freq_index(i, Ph), Ph, a.dx), Ky)));
        }
      }
      int tm = threadIdx.x;
      asm volatile("" : "+v"(tm));
      __syncthreads();
#pragma unroll
      for (int m = 0; m < FFT_MAXV; ++m) {
        const int i = tm + m * nt;
        if (i < Ph) lds[padx(i)] = acc[m];
      }
      __syncthreads();
      fft_lds<true>(lds, ph, tm, nt);
      float2* dst = U + (size_t)bc * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
      for (int r = tm; r < a.Hout; r += nt) {
        const float2 v = cscale(lds[padx(a.out_r0 + r)], a.scale);
        dst[u_roff(r)] = a.zacc ? cadd(dst[u_roff(r)], v) : v;
      }
      return;
    }
    for (int i = tid; i < Ph; i += nt) {
      const int s = i - a.in_r0;
      lds[padx(i)] = (s >= 0 && s < a.Hin) ? col[(size_t)s * CB] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    fft_lds<false>(lds, ph, tid, nt);
    float2 sp[FFT_MAXV];
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int m = 0; m < FFT_MAXV; ++m) {
      const int i = tid + m * nt;
      sp[m] = i < Ph ? lds[padx(i)] : make_float2(0.f, 0.f);
    }
    const float2* tcol = a.tft ? a.tft + ((size_t)(bc % a.C) * a.ncols + c) * Ph : nullptr;
    for (int zz = z_lo; zz < z_hi; ++zz) {
      const TfScalars s = tf_scalars(a, lam, zval(a, a.zoff + zz));
      int tm = threadIdx.x;
      asm volatile("" : "+v"(tm));
      __syncthreads();  // previous z's readers are done with lds
#pragma unroll
      for (int m = 0; m < FFT_MAXV; ++m) {
        const int i = tm + m * nt;
        if (i < Ph)
          lds[padx(i)] = cmul(sp[m], tcol ? (a.adjoint ? make_float2(tcol[i].x, -tcol[i].y) : tcol[i])
                                          : tf_value(a, s, kfreq(freq_index(i, Ph), Ph, a.dx), Ky));
      }
      __syncthreads();
      fft_lds<true>(lds, ph, tm, nt);
      float2* dst = U + ((size_t)zz * a.BC + bc) * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
      for (int r = tm; r < a.Hout; r += nt) dst[u_roff(r)] = cscale(lds[padx(a.out_r0 + r)], a.scale);
    }
  }
}

template <int PN>
__global__ void __launch_bounds__(1024) asm_cols(const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph,
                                                AsmArgs a) {
  asm_cols_body<PN, false>(T, U, ph, a);
}

template <int PN>
__global__ void __launch_bounds__(1024) asm_cols_zsum(const float2* __restrict__ T, float2* __restrict__ U,
                                                     FftPlan ph, AsmArgs a) {
  asm_cols_body<PN, true>(T, U, ph, a);
}

// Per (wavelength, band column) of a mixed-radix Ph: sqrt(k^2 - Kx^2 - Ky^2) of every row
// (z-independent, written on the first z-chunk) and the kept-row bound M_z of each z of the
// chunk (bisection with the exact reference-order tests, one lane per z; see asm_cols).  Every
// plane of the wavelength shares them, so the column pass does no fp32 division.
template <int PN>
__device__ __forceinline__ void tf_tables_body(const AsmArgs& a, int blk, int with_sq) {
  const int li = blk / a.ncols, c = blk - li * a.ncols;
  const float lam = a.lam[li];
  const float Ky = kfreq(c - a.J, a.Pw, a.dy);
  const size_t col = (size_t)li * a.ncols + c;
  if (with_sq) {
    const float kl = TWO_PI_F / lam;
    const float kl2 = tf_mul(kl, kl);
    const float Ky2 = tf_mul(Ky, Ky);
    for (int i = threadIdx.x; i < PN; i += blockDim.x) {
      const float Kx = kfreq(freq_index(i, PN), PN, a.dx);
      a.sqt[col * PN + i] = sqrtf(fmaxf(tf_sub(kl2, tf_add(tf_mul(Kx, Kx), Ky2)), 0.0f));
    }
  }
  if (a.nz <= 2) {
    // few planes (the DONN / QAT layers: one): every lane tests ceil((PN/2+1)/64) rows and M_z + 1
    // is the number that pass (the kept set is a prefix of |m_x|), instead of one lane's serial
    // bisection
    for (int zz = 0; zz < a.nz; ++zz) {
      const TfScalars s = tf_scalars(a, lam, zval(a, a.zoff + zz));
      int n = 0;
#pragma unroll
      for (int m0 = 0; m0 <= PN / 2; m0 += MX_T) {
        const int m = m0 + (int)threadIdx.x;
        n += __popcll(__ballot(m <= PN / 2 && tf_pass(a.bl, PN, a.dx, s, Ky, m)));
      }
      if (threadIdx.x == 0) a.mzt[col * a.nz + zz] = n - 1;
    }
    return;
  }
  for (int zz = threadIdx.x; zz < a.nz; zz += blockDim.x) {
    const TfScalars s = tf_scalars(a, lam, zval(a, a.zoff + zz));
    int lo = -1, hi = PN / 2 + 1;
    if (tf_pass(a.bl, PN, a.dx, s, Ky, 0)) {
      lo = 0;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tf_pass(a.bl, PN, a.dx, s, Ky, mid)) lo = mid;
        else hi = mid;
      }
    }
    a.mzt[col * a.nz + zz] = lo;
  }
}

template <int PN>
__global__ void __launch_bounds__(MX_T) asm_tf_tables(AsmArgs a, int with_sq) {
  tf_tables_body<PN>(a, blockIdx.x, with_sq);
}

// K2 for a compile-time mixed-radix Ph (MxPlan, blockDim MX_T): the power-of-two kernel's
// structure -- spectrum kept in registers, H_z applied in the inverse's loader from the
// per-column sqrt and the bisected |m_x| bound, cropped rows stored from the last stage -- with
// the runtime plan's numerics at the output (1 / (Ph Pw) is not a power of two here, so the
// scale is applied to each output element as asm_cols<0> does).
// MID: the 300-point layers' windows ([N/3, 2N/3) in and out: padding 2 with unpad, cfg4 / cfg5)
// as compile-time constants (asm_cols_mx_mid, the default for that geometry)
template <class MP, bool ZSUM, bool MID = false>
__device__ __forceinline__ void asm_cols_mx_body(const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph,
                                                 AsmArgs a) {
  constexpr int PN = MP::N, RL = MP::RL, MT = mx_threads(PN), NBL = PN / RL, MBL = (NBL + MT - 1) / MT;
  static_assert(MP::R0 == RL, "the inverse must start where the forward ends");
  extern __shared__ float2 lds[];
  int id, z_lo = 0, z_hi = a.nz;
  if ((int)blockIdx.x < a.kfull) {
    id = xcd_chunk(blockIdx.x, a.kfull);
  } else {
    const int t = blockIdx.x - a.kfull, part = t % a.kparts;
    id = a.kfull + t / a.kparts;
    z_lo = part * a.nz / a.kparts;
    z_hi = (part + 1) * a.nz / a.kparts;
  }
  const int bc = id / a.ncols, c = id - bc * a.ncols;
  const float2* col = T + (size_t)bc * a.ncb * CB * a.Hin + blk(c, 0, a.Hin);
  int tid = threadIdx.x;
  float2 sp[MBL][RL];
  if constexpr (MID) __builtin_assume(tid >= 0 && tid < MT);
  auto ld0 = [&](int, int, int idx) {
    const int s = idx - (MID ? PN / 3 : a.in_r0);
    return (s >= 0 && s < (MID ? PN / 3 : a.Hin)) ? col[(size_t)s * CB] : make_float2(0.f, 0.f);
  };
  auto sv0 = [&](int m, int r, int, float2 v) { sp[m][r] = v; };
  const auto twr = MP::template twiddles<MT>(ph.tw, tid);
  if constexpr (!ZSUM) MP::template run<false, MT>(lds, twr, tid, ld0, sv0);
  if (!ZSUM && a.tft) {  // RSC: tabulated transfer function FFT2(K), one z
    const float2* tcol = a.tft + ((size_t)(bc % a.C) * a.ncols + c) * PN;
    int tz = threadIdx.x;
    asm volatile("" : "+v"(tz));
    auto ld1 = [&](int m, int r, int idx) {
      const float2 t = tcol[idx];
      return cmul(sp[m][r], a.adjoint ? make_float2(t.x, -t.y) : t);
    };
    float2* dst = U + (size_t)bc * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
    auto sv1 = [&](int, int, int j, float2 v) {
      const int r = j - a.out_r0;
      if (r >= 0 && r < a.Hout) dst[u_roff(r)] = cscale(v, a.scale);
    };
    MP::template run<true, MT>(lds, twr, tz, ld1, sv1);
    return;
  }
  // kept rows |m_x| <= M_z per z and the z-independent sqrt(k^2 - K^2) of the elements this
  // thread holds: the wavelength's per-column tables (asm_tf_tables)
  const size_t tc = (size_t)(bc % a.C) * a.ncols + c;
  const int* mzc = a.mzt + tc * a.nz;
  const float* sqc = a.sqt + tc * PN;
  float sq[MBL][RL];
#pragma unroll
  for (int m = 0; m < MBL; ++m) {
    const int i = tid + m * MT;
#pragma unroll
    for (int r = 0; r < RL; ++r) sq[m][r] = (NBL % MT == 0 || i < NBL) ? sqc[i + r * NBL] : 0.f;
  }
  if constexpr (ZSUM) {
    // adjoint over the chunk's planes: sp = sum_z FFT(T_z column) conj(H_z), then one inverse
#pragma unroll
    for (int m = 0; m < MBL; ++m)
#pragma unroll
      for (int r = 0; r < RL; ++r) sp[m][r] = make_float2(0.f, 0.f);
    for (int zz = z_lo; zz < z_hi; ++zz) {
      const float z = zval(a, a.zoff + zz);
      const int M = mzc[zz];
      const float2* colz = T + ((size_t)zz * a.BC + bc) * a.ncb * CB * a.Hin + blk(c, 0, a.Hin);
      int tz = threadIdx.x;
      asm volatile("" : "+v"(tz));
      auto ldz = [&](int, int, int idx) {
        const int s = idx - a.in_r0;
        return (s >= 0 && s < a.Hin) ? colz[(size_t)s * CB] : make_float2(0.f, 0.f);
      };
      auto acc = [&](int m, int r, int j, float2 v) {
        const int mx = freq_index(j, PN);
        if (mx > M || -mx > M) return;
        float sn, cs;
        sincos_hw(tf_mul(z, sq[m][r]), &sn, &cs);
        sp[m][r] = cadd(sp[m][r], cmul(v, make_float2(cs, -sn)));
      };
      MP::template run<false, MT>(lds, twr, tz, ldz, acc);
    }
    int tz = threadIdx.x;
    asm volatile("" : "+v"(tz));
    auto ld1 = [&](int m, int r, int) { return sp[m][r]; };
    float2* dst = U + (size_t)bc * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
    auto sv1 = [&](int, int, int j, float2 v) {
      const int r = j - a.out_r0;
      if ((unsigned)r < (unsigned)a.Hout) {
        const float2 o = cscale(v, a.scale);
        dst[u_roff(r)] = a.zacc ? cadd(dst[u_roff(r)], o) : o;
      }
    };
    MP::template run<true, MT>(lds, twr, tz, ld1, sv1);
    return;
  }
  for (int zz = z_lo; zz < z_hi; ++zz) {
    const float z = zval(a, a.zoff + zz);
    const int M = mzc[zz];
    int tz = threadIdx.x;
    asm volatile("" : "+v"(tz));
    if constexpr (MID) __builtin_assume(tz >= 0 && tz < MT);
    auto ld1 = [&](int m, int r, int idx) {
      const int mx = freq_index(idx, PN);
      if (mx > M || -mx > M) return make_float2(0.f, 0.f);
      float sn, cs;
      sincos_hw(tf_mul(z, sq[m][r]), &sn, &cs);
      return cmul(sp[m][r], make_float2(cs, a.adjoint ? -sn : sn));
    };
    float2* dst = U + ((size_t)zz * a.BC + bc) * a.ncbu * CBU * u_rows(a.Hout) + blk_u(c, 0, a.Hout);
    auto sv1 = [&](int, int, int j, float2 v) {
      const int r = j - (MID ? PN / 3 : a.out_r0);
      if ((unsigned)r < (unsigned)(MID ? PN / 3 : a.Hout)) dst[u_roff(r)] = cscale(v, a.scale);
    };
    MP::template run<true, MT>(lds, twr, tz, ld1, sv1);
  }
}

template <class MP>
__global__ void __launch_bounds__(mx_threads(MP::N)) __attribute__((amdgpu_waves_per_eu(MX_WPE))) asm_cols_mx(
    const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph, AsmArgs a) {
  asm_cols_mx_body<MP, false>(T, U, ph, a);
}

template <class MP>
__global__ void __launch_bounds__(mx_threads(MP::N)) __attribute__((amdgpu_waves_per_eu(MX_WPE))) asm_cols_mx_mid(
    const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph, AsmArgs a) {
  asm_cols_mx_body<MP, false, true>(T, U, ph, a);
}

template <class MP>
__global__ void __launch_bounds__(mx_threads(MP::N)) __attribute__((amdgpu_waves_per_eu(MX_WPE))) asm_cols_mx_zsum(
    const float2* __restrict__ T, float2* __restrict__ U, FftPlan ph, AsmArgs a) {
  asm_cols_mx_body<MP, true>(T, U, ph, a);
}

// ---------------------------------------------------------------------------------------------
// K3: per output row: gather band from U, IFFT(Pw), crop -> out[z][bc][r][w]
// ---------------------------------------------------------------------------------------------
// LOSS: the stored row also feeds the |E|^2 -> normalize -> MSE sums of its batch item
// (LossAcc; Z == 1 so plane == bc), stored per workgroup in slot (c, r) of b by loss_store_part.
// MID: the crop as a compile-time window: the middle half of the padded row for the power-of-two
// sizes (out_c0 = PN / 4, Wout = PN / 2: padding scale 1 with unpad, cfg2), the middle third for
// the 300-point layers (out_c0 = Wout = 100: padding 2 with unpad, cfg4 / cfg5)
template <int PN, bool LOSS, bool MID = false>
__device__ __forceinline__ void rows_inv_body(const float2* __restrict__ U, float2* __restrict__ out, FftPlan pw,
                                              const AsmArgs& a) {
  extern __shared__ float2 lds[];
  const int row = xcd_rows(blockIdx.x, gridDim.x);  // row in [0, nz*BC*Hout)
  const int plane = row / a.Hout, r = row - plane * a.Hout;  // plane = zz*BC + bc
  const int tid = threadIdx.x, nt = blockDim.x;
  const float2* src = U + (size_t)plane * a.ncbu * CBU * u_rows(a.Hout);
  float2* dst = out + ((size_t)(a.zoff * a.BC + plane) * a.Hout + r) * a.Wout;
  LossAcc acc;
  const float* trow = nullptr;
  unsigned ibase = 0;
  int lb = 0, lc = 0;
  if constexpr (LOSS) {  // loss item lb = z B + b of the chunk's global plane
    const int gp = a.zoff * a.BC + plane;
    lb = gp / a.C;
    lc = gp - lb * a.C;
    const int tb = a.ls.tB == 1 ? 0 : lb, tc = a.ls.tC == 1 ? 0 : lc;
    trow = a.ls.target + (((size_t)tb * a.ls.tC + tc) * a.Hout + r) * a.Wout;
    ibase = (unsigned)((lc * a.Hout + r) * a.Wout);
  }
  auto put = [&](int w, float2 v) {
    // the window mask of a folded aperture (forward): the 300-point pass only
    if constexpr (is_mx(PN)) if (a.ap_side == 1 && !aperture_open(a.apm, r, w)) v = cscale(v, 0.f);
    if constexpr (PN >= 1024 && !is_mx(PN)) {
      // large planes: written once and not read back by this pipeline, so streaming (non-temporal)
      // stores that do not displace the U lines the neighbouring rows' workgroups still gather
      // (cfg2: K3 4.71 -> 4.45 ms).  The small P = 300 layers' outputs feed the next layer from L2.
      st_stream(dst + w, v);
    } else {
      dst[w] = v;
    }
    if constexpr (LOSS) acc.add(v, trow[w], ibase + (unsigned)w);
  };
  if constexpr (is_mx(PN)) {
    constexpr int MT = mx_threads(PN);
    if constexpr (MID) __builtin_assume(tid >= 0 && tid < MT);
    using MP = typename MxOf<PN>::type;
    const auto twr = MP::template twiddles<MT>(pw.tw, tid);
    auto ld = [&](int, int, int j) {
      const int c = band_col(j, PN, a.J, a.ncols);
      return c >= 0 ? src[blk_u(c, r, a.Hout)] : make_float2(0.f, 0.f);
    };
    // (MID: the layers' output window [N/3, 2N/3))
    auto sv = [&](int, int, int j, float2 v) {
      const int w = j - (MID ? PN / 3 : a.out_c0);
      if ((unsigned)w < (unsigned)(MID ? PN / 3 : a.Wout)) put(w, v);
    };
    MP::template run<true, MT>(lds, twr, tid, ld, sv);
  } else if constexpr (PN > 0) {
    // The twiddle tables' global loads go out first and their LDS writes happen after the first
    // stage's gather (the hook runs before the first exchange), so the gather does not wait behind
    // them: cfg2 K3 4.40 -> 4.28 ms (profiles/r03_k3_probes.txt)
    constexpr int TT = Geo<PN>::T;
    __builtin_assume(tid >= 0 && tid < TT);  // the launch's block size: lets the crop test fold (MID)
    const auto twf = tw_fetch<PN, TT>(pw.tw, tid);
    const TwLds twl = tw_lds_at<PN>(tw_slot<PN>(lds));
    auto tw_hook = [&]() { tw_store<PN, TT>(tw_slot<PN>(lds), twf, tid); };
    // First stage (radix 16, L = 1) reads j = i + q*NB0, i < NB0.  Its band column is
    // c = c0 + delta_q with c0 = i + J >= 0 and delta_q = q*NB0 (- PN for the negative
    // frequencies), a multiple of CBU: the blocked address is then base(c0) + delta_q*Hout,
    // one add per element instead of the full blk_u() per element.
    constexpr int NB0 = PN / pow2_v(PN);  // first stage: radix pow2_v, L = 1
    static_assert(NB0 % CBU == 0, "band offsets must be whole U blocks");
    static_assert(Geo<PN>::T == NB0, "one first-stage butterfly per thread: i = tid");
    const int c0 = tid + a.J;
    const float2* base = src + blk_u(c0, r, a.Hout);
    const long cstride = u_rows(a.Hout);  // blk_u(c + delta) - blk_u(c) = delta * cstride for CBU | delta
    // operands q in [4, 12) are the columns PN/4 <= |m_y| < 3 PN/4: outside the band for every
    // lane of most waves (all but the first and last at cfg2), which then skip their address math
    // and masked loads on one scalar branch
    static_assert(NB0 == PN / 16, "radix-16 first stage");
    const bool mid0 = __all(c0 + 4 * NB0 >= a.ncols && c0 + 11 * NB0 - PN < 0);
    auto ld = [&](int, int q, int) {
      if (q >= 4 && q < 12 && mid0) return make_float2(0.f, 0.f);
      const int delta = q * NB0 >= PN / 2 ? q * NB0 - PN : q * NB0;
      if ((unsigned)(c0 + delta) >= (unsigned)a.ncols) return make_float2(0.f, 0.f);
      return base[(long)delta * cstride];
    };
    auto sv = [&](int, int, int j, float2 v) {
      const int w = j - (MID ? PN / 4 : a.out_c0);
      if ((unsigned)w < (unsigned)(MID ? PN / 2 : a.Wout)) put(w, v);
    };
    fft_pow2_run<true, PN, TT, FFT_ROWS>(lds, twl, tid, ld, sv, tw_hook);
  } else {
    for (int j = tid; j < a.Pw; j += nt) {
      const int c = band_col(j, a.Pw, a.J, a.ncols);
      lds[padx(j)] = c >= 0 ? src[blk_u(c, r, a.Hout)] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    fft_lds<true>(lds, pw, tid, nt);
    for (int w = tid; w < a.Wout; w += nt) put(w, lds[padx(a.out_c0 + w)]);
  }
  // C Hout slots per item; loss_finish_kernel reduces them (an in-kernel finish by the last
  // workgroup of each item cost one agent-scope release fence -- an L2 writeback -- per workgroup:
  // cfg5 chained 1.10 -> 2.12 ms at batch 256, profiles/r05_experiments.txt)
  if constexpr (LOSS) loss_store_part(acc, a.ls, lb, lc * a.Hout + r);
}

template <int PN>
__global__ void __launch_bounds__(1024) THZ_ROW_ATTR asm_rows_inv(const float2* __restrict__ U, float2* __restrict__ out,
                                                    FftPlan pw, AsmArgs a) {
  rows_inv_body<PN, false>(U, out, pw, a);
}

template <int PN>
__global__ void __launch_bounds__(1024) THZ_ROW_ATTR asm_rows_inv_mid(const float2* __restrict__ U,
                                                                      float2* __restrict__ out, FftPlan pw, AsmArgs a) {
  rows_inv_body<PN, false, true>(U, out, pw, a);
}

template <int PN>
__global__ void __launch_bounds__(1024) THZ_ROW_ATTR asm_rows_inv_loss_mid(const float2* __restrict__ U,
                                                                           float2* __restrict__ out, FftPlan pw,
                                                                           AsmArgs a) {
  rows_inv_body<PN, true, true>(U, out, pw, a);
}

template <int PN>
__global__ void __launch_bounds__(1024) THZ_ROW_ATTR asm_rows_inv_loss(const float2* __restrict__ U,
                                                                       float2* __restrict__ out, FftPlan pw, AsmArgs a) {
  rows_inv_body<PN, true>(U, out, pw, a);
}


// ---------------------------------------------------------------------------------------------
// RSC (Props/RSC_Prop.py:129-215): transfer function = FFT2 of the spatial RS kernel on the
// P = N + 2 floor(N/2) grid, stored column-major [C][Pw][Ph] for the column pass.
// ---------------------------------------------------------------------------------------------
struct RscKArgs {
  int C, Ph, Pw, ncbK;
  float dx, z;
  float lam[THZ_MAX_WAVELENGTHS];
};

template <int PN>
__global__ void __launch_bounds__(1024) rsc_k_rows(float2* __restrict__ TK, FftPlan pw, RscKArgs k) {
  extern __shared__ float2 lds[];
  const int row = blockIdx.x;
  const int c = row / k.Ph, i = row - c * k.Ph;
  const float lam = k.lam[c];
  const float kk = 6.283185307179586f / lam;
  const RsPhase rph = rs_phase(lam, k.z);
  // grid x = linspace(-P dx/2, P dx/2, P) on both axes with dx (:83-84)
  const float xi = lin(-(float)k.Ph * k.dx / 2.0f, (float)k.Ph * k.dx / 2.0f, k.Ph, i);
  const float ylo = -(float)k.Pw * k.dx / 2.0f, yhi = (float)k.Pw * k.dx / 2.0f;
  float2* dst = TK + (size_t)c * k.ncbK * CB * k.Ph;
  auto load = [&](int j) { return rs_kernel(xi, lin(ylo, yhi, k.Pw, j), k.z, kk, rph); };
  auto store = [&](int j, float2 v) { dst[blk(band_col(j, k.Pw, k.Pw / 2, k.Pw), i, k.Ph)] = v; };
  const int tid = threadIdx.x, nt = blockDim.x;
  if constexpr (PN > 0) {
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), pw.tw, tid, nt);
    auto ld = [&](int, int, int j) { return load(j); };
    auto sv = [&](int, int, int j, float2 v) { store(j, v); };
    fft_pow2_run<false, PN, Geo<PN>::T, FFT_ROWS>(lds, twl, tid, ld, sv);
  } else {
    for (int j = tid; j < k.Pw; j += nt) lds[padx(j)] = load(j);
    __syncthreads();
    fft_lds<false>(lds, pw, tid, nt);
    for (int j = tid; j < k.Pw; j += nt) store(j, lds[padx(j)]);
  }
}

template <int PN>
__global__ void __launch_bounds__(1024) rsc_k_cols(const float2* __restrict__ TK, float2* __restrict__ KF,
                                                  FftPlan ph, RscKArgs k) {
  extern __shared__ float2 lds[];
  const int id = xcd_chunk(blockIdx.x, gridDim.x);
  const int c = id / k.Pw, cc = id - c * k.Pw;
  const float2* col = TK + (size_t)c * k.ncbK * CB * k.Ph + blk(cc, 0, k.Ph);
  float2* dst = KF + ((size_t)c * k.Pw + cc) * k.Ph;
  const int tid = threadIdx.x, nt = blockDim.x;
  if constexpr (PN > 0) {
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), ph.tw, tid, nt);
    auto ld = [&](int, int, int i) { return col[(size_t)i * CB]; };
    auto sv = [&](int, int, int i, float2 v) { dst[i] = v; };
    fft_pow2_run<false, PN, Geo<PN>::T, FFT_ROWS>(lds, twl, tid, ld, sv);
  } else {
    for (int i = tid; i < k.Ph; i += nt) lds[padx(i)] = col[(size_t)i * CB];
    __syncthreads();
    fft_lds<false>(lds, ph, tid, nt);
    for (int i = tid; i < k.Ph; i += nt) dst[i] = lds[padx(i)];
  }
}

// ---------------------------------------------------------------------------------------------
// Generic batched row FFT (building block / diagnostics)
// ---------------------------------------------------------------------------------------------
template <int PN>
__global__ void __launch_bounds__(1024) fft_rows_kernel(const float2* __restrict__ in, float2* __restrict__ out,
                                                       FftPlan p, int inverse, size_t stride) {
  extern __shared__ float2 lds[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t base = (size_t)blockIdx.x * stride;
  if constexpr (PN > 0) {
    const TwLds twl = load_tw_lds<PN>(tw_slot<PN>(lds), p.tw, tid, nt);
    auto ld = [&](int, int, int j) { return in[base + j]; };
    auto sv = [&](int, int, int j, float2 v) { out[base + j] = v; };
    if (inverse) fft_pow2_run<true, PN, Geo<PN>::T, 3>(lds, twl, tid, ld, sv);
    else fft_pow2_run<false, PN, Geo<PN>::T, FFT_TAIL>(lds, twl, tid, ld, sv);
  } else {
    for (int j = tid; j < p.n; j += nt) lds[padx(j)] = in[base + j];
    __syncthreads();
    if (inverse) fft_lds<true>(lds, p, tid, nt);
    else fft_lds<false>(lds, p, tid, nt);
    for (int j = tid; j < p.n; j += nt) out[base + j] = lds[padx(j)];
  }
}

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
struct AsmGeom {
  int BC, Ph, Pw, ncols, J, ncb, ncbu, Hin, Win, Hout, Wout, zc;
  int C;
  int adj;  // adjoint: T holds the z-chunk's planes, U one (summed) plane
};

static int validate(const thz_asm_desc* d) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || d->pad_h < 0 || d->pad_w < 0)
    return fail(THZ_E_ARG, "bad shape B=%d C=%d H=%d W=%d pad=(%d,%d)", d->B, d->C, d->H, d->W, d->pad_h, d->pad_w);
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d wavelengths", d->C, THZ_MAX_WAVELENGTHS);
  if (d->Z < 1 || d->Z > THZ_MAX_Z) return fail(THZ_E_UNSUPPORTED, "Z=%d outside [1, %d]", d->Z, THZ_MAX_Z);
  if (d->bandlimit < 0 || d->bandlimit > 2) return fail(THZ_E_ARG, "bad bandlimit %d", d->bandlimit);
  if (!d->wavelengths || (!d->z && !d->z_dev)) return fail(THZ_E_ARG, "null wavelengths / z");
  if (!(d->dx > 0.f) || !(d->dy > 0.f)) return fail(THZ_E_ARG, "spacing must be > 0");
  const int Ph = d->H + 2 * d->pad_h, Pw = d->W + 2 * d->pad_w;
  if (Ph > FFT_MAX_N || Pw > FFT_MAX_N)
    return fail(THZ_E_UNSUPPORTED, "padded size %dx%d exceeds %d", Ph, Pw, FFT_MAX_N);
  for (int c = 0; c < d->C; ++c)
    if (!(d->wavelengths[c] > 0.f)) return fail(THZ_E_ARG, "wavelength[%d] must be > 0", c);
  return THZ_OK;
}

// Largest |m_y| with a possibly non-zero H over all (wavelength, z); +2 columns margin for
// the fp32-vs-double evaluation.  Exact: Ky^2 <= min(k^2, (2 pi v_lim)^2); approx: |Ky| <=
// min(k, k_y_max); none: evanescent only.  All maxima sit on the Kx = 0 row.
static int band_half_width(const thz_asm_desc* d, int Ph, int Pw) {
  double kymax = 0.0;
  const double dy = d->dy, dx = d->dx;
  for (int c = 0; c < d->C; ++c) {
    const double lam = d->wavelengths[c];
    const double kl = 2.0 * M_PI / lam;
    for (int zi = 0; zi < d->Z; ++zi) {
      double lim = kl;
      if (d->z_dev) {  // the planes are read on the device: size the band for any z (evanescent bound)
        kymax = std::max(kymax, lim);
        continue;
      }
      const double z = d->z[zi];
      if (d->bandlimit == THZ_BANDLIMIT_EXACT) {
        const double dv = 1.0 / (2.0 * Ph * dy);
        const double vl = 1.0 / std::sqrt(std::pow(2.0 * dv * z, 2) + 1.0) / lam;
        lim = std::min(lim, 2.0 * M_PI * vl);
      } else if (d->bandlimit == THZ_BANDLIMIT_APPROX) {
        const double ly = Ph * dy;
        const double kym = 2.0 * M_PI / std::sqrt(std::pow(2.0 * z / ly, 2) + 1.0) / lam;
        lim = std::min(lim, kym);
      }
      kymax = std::max(kymax, lim);
    }
  }
  (void)dx;
  const double dky = 2.0 * M_PI / (Pw * dy);
  const double j = std::floor(kymax / dky) + 2.0;
  if (j >= Pw / 2) return -1;  // full band
  return (int)j;
}

static void geometry(const thz_asm_desc* d, AsmGeom* g) {
  g->BC = d->B * d->C;
  g->C = d->C;
  g->Ph = d->H + 2 * d->pad_h;
  g->Pw = d->W + 2 * d->pad_w;
  const int Ho = d->unpad ? d->H : g->Ph, Wo = d->unpad ? d->W : g->Pw;
  if (!d->adjoint) {
    g->Hin = d->H; g->Win = d->W; g->Hout = Ho; g->Wout = Wo;
  } else {
    g->Hin = Ho; g->Win = Wo; g->Hout = d->H; g->Wout = d->W;
  }
  const int J = band_half_width(d, g->Ph, g->Pw);
  if (J < 0) {
    g->ncols = g->Pw;
    g->J = g->Pw / 2;
  } else {
    g->ncols = 2 * J + 1;
    g->J = J;
  }
  g->ncb = (g->ncols + CB - 1) / CB;
  g->ncbu = (g->ncols + CBU - 1) / CBU;
  int zc = d->z_chunk > 0 ? d->z_chunk : 0;
  if (zc == 0) {
    // default: up to 64 z-planes per column pass (the forward column FFT and the T read are
    // shared by the chunk; one K2 and one K3 launch per 64 planes), U capped at 10 GiB of the
    // 288 GB HBM.  Measured on cfg2 (64 planes, round 2): z_chunk 32 / 64 -> 6830 / 7270 planes/s.
    // The Z-summing adjoint keeps the chunk's input planes in T instead (same cap).
    const double per_z = d->adjoint ? (double)g->BC * g->ncb * CB * g->Hin * sizeof(float2)
                                    : (double)g->BC * g->ncbu * CBU * g->Hout * sizeof(float2);
    zc = (int)std::max(1.0, std::min(64.0, std::floor((10240.0 * 1024 * 1024) / per_z)));
  }
  g->zc = std::min(zc, d->Z);
  g->adj = d->adjoint;
}

// Compile-time power-of-two instantiations (blockDim = n / FFT_MAXV); 0 = runtime plan.
static int pow2_kind(int n) {
  switch (n) {
    case 1024: case 2048: case 4096: case 8192: case 16384: return n;
    default: return 0;
  }
}
static int threads_for(int n) { return pow2_kind(n) ? n / pow2_v(n) : fft_threads(n); }

#define THZ_POW2_SWITCH(n, KER, ...)                                                              \
  switch (pow2_kind(n)) {                                                                          \
    case 1024: hipLaunchKernelGGL(KER<1024>, __VA_ARGS__); break;                                  \
    case 2048: hipLaunchKernelGGL(KER<2048>, __VA_ARGS__); break;                                  \
    case 4096: hipLaunchKernelGGL(KER<4096>, __VA_ARGS__); break;                                  \
    case 8192: hipLaunchKernelGGL(KER<8192>, __VA_ARGS__); break;                                  \
    case 16384: hipLaunchKernelGGL(KER<16384>, __VA_ARGS__); break;                                \
    default: hipLaunchKernelGGL(KER<0>, __VA_ARGS__); break;                                       \
  }

template <int PN>
static void add_kernels(std::vector<const void*>& ks) {
  ks.push_back((const void*)asm_rows_fwd<PN>);
  ks.push_back((const void*)asm_cols<PN>);
  if constexpr (PN == 8192) ks.push_back((const void*)asm_rows_inv_mid<PN>);
  ks.push_back((const void*)asm_cols_zsum<PN>);
  ks.push_back((const void*)asm_rows_inv<PN>);
  ks.push_back((const void*)asm_rows_inv_loss<PN>);
  ks.push_back((const void*)fft_rows_kernel<PN>);
  ks.push_back((const void*)rsc_k_rows<PN>);
  ks.push_back((const void*)rsc_k_cols<PN>);
}

// Workgroups above 64 KiB of dynamic LDS must opt in once per kernel.
static int ensure_lds_attr() {
  static std::once_flag once;
  static hipError_t err = hipSuccess;
  std::call_once(once, [] {
    const int mx = (int)fft_lds_bytes(FFT_MAX_N) + 12 * THZ_MAX_Z;
    std::vector<const void*> ks;
    add_kernels<0>(ks);
    add_kernels<1024>(ks);
    add_kernels<2048>(ks);
    add_kernels<4096>(ks);
    add_kernels<8192>(ks);
    add_kernels<16384>(ks);
    for (const void* k : ks) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      if (e != hipSuccess) err = e;
    }
  });
  if (err != hipSuccess) return fail(THZ_E_HIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize): %s",
                                     hipGetErrorString(err));
  return THZ_OK;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workgroups of the column pass resident on the whole device at once (CUs x occupancy).
// Ph / Pw with a compile-time mixed-radix kernel (asm_cols_mx, asm_rows_*<N>), else 0
static int mx_kind(int n) { return is_mx(n) ? n : 0; }
// K1 / K3: the mixed-radix instantiation or the power-of-two switch
#define THZ_ROWS_SWITCH(n, KER, G, LDSB, ...)                                                      \
  if (mx_kind(n) == Mx300::N) hipLaunchKernelGGL(KER<Mx300::N>, G, dim3(MX_T), LDSB, __VA_ARGS__); \
  else if (mx_kind(n) == Mx500::N) hipLaunchKernelGGL(KER<Mx500::N>, G, dim3(mx_threads(500)), LDSB, __VA_ARGS__); \
  else THZ_POW2_SWITCH(n, KER, G, dim3(threads_for(n)), LDSB, __VA_ARGS__)
// the mixed-radix column-pass kernels (asm_cols_mx*, templated on the plan) and their tables
#define THZ_MX_COLS(n, KER, ...)                                                                   \
  if ((n) == Mx300::N) hipLaunchKernelGGL(KER<Mx300>, __VA_ARGS__);                               \
  else hipLaunchKernelGGL(KER<Mx500>, __VA_ARGS__)
#define THZ_MX_TABLES(n, ...)                                                                      \
  if ((n) == Mx300::N) hipLaunchKernelGGL(asm_tf_tables<Mx300::N>, __VA_ARGS__);                  \
  else hipLaunchKernelGGL(asm_tf_tables<Mx500::N>, __VA_ARGS__)

// The 300-point passes with the layers' windows ([N/3, 2N/3) in and out: padding 2 with unpad,
// cfg4 / cfg5) as compile-time constants: the column pass (asm_cols_mx_mid: 80.8 vs 83.3 us per
// launch, cfg5 chained 1.097 vs 1.133 ms), K1 (asm_rows_fwd<300, true>) and K3
// (asm_rows_inv_mid<300>, asm_rows_inv_loss_mid<300>).  The A/B records: profiles/r04_experiments.txt.
static bool mx_mid(const AsmArgs& a) {
  return !a.tft && a.in_r0 == Mx300::N / 3 && a.Hin == Mx300::N / 3 && a.out_r0 == Mx300::N / 3 &&
         a.Hout == Mx300::N / 3;
}
// K3 with its crop as a compile-time window: the middle half of P = 8192 (asm_rows_inv_mid<8192>,
// padding scale 1 with unpad, cfg2: 4.00 vs 4.13 ms) or the middle third of P = 300
static bool k3_mid(int Pw, const AsmArgs& a) {
  return (Pw == 8192 && a.out_c0 == Pw / 4 && a.Wout == Pw / 2) ||
         (Pw == Mx300::N && a.out_c0 == Pw / 3 && a.Wout == Pw / 3);
}
// K1 of the 300-point layers with the input window as constants (asm_rows_fwd<300, true>)
static bool k1_mid(int Pw, const AsmArgs& a) { return Pw == Mx300::N && a.in_c0 == Pw / 3 && a.Win == Pw / 3; }
static int k2_resident(int Ph, int threads, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, size_t>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_tuple(dev, Ph, threads, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const void* k = nullptr;
  switch (pow2_kind(Ph)) {
    case 1024: k = (const void*)asm_cols<1024>; break;
    case 2048: k = (const void*)asm_cols<2048>; break;
    case 4096: k = (const void*)asm_cols<4096>; break;
    case 8192: k = (const void*)asm_cols<8192>; break;
    case 16384: k = (const void*)asm_cols<16384>; break;
    default: k = (const void*)asm_cols<0>; break;
  }
  if (mx_kind(Ph) == Mx300::N) k = (const void*)asm_cols_mx<Mx300>;
  if (mx_kind(Ph) == Mx500::N) k = (const void*)asm_cols_mx<Mx500>;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, threads, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    per_cu = cus = 0;
  const int r = per_cu * cus;
  cache[key] = r;
  return r;
}

// K2 task split: whole columns for the full dispatch rounds, the remainder split by z-range.
static int k2_tasks(const AsmGeom& g, AsmArgs* a, int threads, size_t lds) {
  const int nc = g.ncols * g.BC;
  const int G = k2_resident(g.Ph, threads, lds);
  if (G <= 0 || a->nz <= 1) {
    a->kfull = nc;
    a->kparts = 1;
    return nc;
  }
  const int full = nc / G * G, rem = nc - full;
  a->kfull = full;
  a->kparts = rem ? std::max(1, std::min(a->nz, G / rem)) : 1;
  return full + rem * a->kparts;
}

// the mixed-radix column pass's per-(wavelength, column) tables, shared by every plane
static size_t tab_sq_bytes(const AsmGeom& g) { return align256((size_t)g.C * g.ncols * g.Ph * sizeof(float)); }
static size_t tab_bytes(const AsmGeom& g) {
  return mx_kind(g.Ph) ? tab_sq_bytes(g) + align256((size_t)g.C * g.ncols * g.zc * sizeof(int)) : 0;
}
static size_t t_bytes(const AsmGeom& g) {
  return align256((size_t)(g.adj ? g.zc : 1) * g.BC * g.ncb * CB * g.Hin * sizeof(float2));
}
static size_t ws_bytes(const AsmGeom& g) {
  return t_bytes(g) + align256((size_t)(g.adj ? 1 : g.zc) * g.BC * g.ncbu * CBU * u_rows(g.Hout) * sizeof(float2)) +
         tab_bytes(g);
}

// The adjoint of a Z-plane forward (sum over planes): per z-chunk, K1 over the chunk's input
// planes and the Z-summing K2 (adding into U after the first chunk); then K3 once.
static int run_adjoint_sum(AsmArgs a, const AsmGeom& g, int Z, const void* in, void* out, float2* T, float2* U,
                           hipStream_t s, FftPlan pw, FftPlan ph, bool mx_tabs) {
  a.zsum = 1;
  a.tab_blocks = 0;
  a.kfull = g.ncols * g.BC;  // every column task runs all of its chunk's planes
  a.kparts = 1;
  const int th = threads_for(g.Ph);
  for (int z0 = 0; z0 < Z; z0 += g.zc) {
    a.zoff = z0;
    a.nz = std::min(g.zc, Z - z0);
    a.zacc = z0 > 0;
    {
      KernelTimer kt("asm_rows_fwd", s);
      if (k1_mid(g.Pw, a)) {
        hipLaunchKernelGGL((asm_rows_fwd<Mx300::N, true>), dim3(a.nz * g.BC * g.Hin), dim3(MX_T), fft_lds_bytes_io(g.Pw),
                           s, (const float2*)in, T, pw, a);
      } else {
        THZ_ROWS_SWITCH(g.Pw, asm_rows_fwd, dim3(a.nz * g.BC * g.Hin), fft_lds_bytes_io(g.Pw), s, (const float2*)in,
                        T, pw, a);
      }
      THZ_LAUNCH_CHECK();
      kt.stop();
    }
    {
      KernelTimer kt("asm_cols", s);
      if (mx_kind(g.Ph)) {
        if (mx_tabs) {
          THZ_MX_TABLES(g.Ph, dim3(g.C * g.ncols), dim3(MX_T), 0, s, a, z0 == 0);
          THZ_LAUNCH_CHECK();
        }
        const size_t lds2 = lds_floats2(g.Ph) * sizeof(float2) + 4 * THZ_MAX_Z;
        THZ_MX_COLS(g.Ph, asm_cols_mx_zsum, dim3(a.kfull), dim3(mx_threads(g.Ph)), lds2, s, (const float2*)T, U, ph, a);
      } else {
        const size_t lds2 = fft_lds_bytes(g.Ph) + 4 * THZ_MAX_Z;
        THZ_POW2_SWITCH(g.Ph, asm_cols_zsum, dim3(a.kfull), dim3(th), lds2, s, (const float2*)T, U, ph, a);
      }
      THZ_LAUNCH_CHECK();
      kt.stop();
    }
  }
  a.zoff = 0;
  a.nz = 1;
  {
    KernelTimer kt("asm_rows_inv", s);
    THZ_ROWS_SWITCH(g.Pw, asm_rows_inv, dim3(g.BC * g.Hout), fft_lds_bytes_io(g.Pw), s, (const float2*)U,
                    (float2*)out, pw, a);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  return THZ_OK;
}

// THZ_K2_RECURRENCE=0 keeps the per-plane sincos everywhere (the A/B and parity tests compare the
// two forms; read per call so a test can toggle it)
static bool plane_recurrence_disabled() {
  const char* v = std::getenv("THZ_K2_RECURRENCE");
  return v && v[0] == '0';
}

// K1 once, then (K2, K3) per z-chunk, on a prepared argument block.
static int run_pipeline(AsmArgs a, const AsmGeom& g, int Z, const void* in, void* out, float2* T, float2* U,
                        hipStream_t s, FftPlan pw, FftPlan ph, char* tabs = nullptr) {
  int e;
  if ((e = ensure_lds_attr())) return e;
  const int th = threads_for(g.Ph);
  const bool mx_tabs = mx_kind(g.Ph) && !a.tft;
  if (mx_tabs) {
    if (!tabs) return fail(THZ_E_WORKSPACE, "mixed-radix column tables need workspace");
    a.sqt = (float*)tabs;
    a.mzt = (int*)(tabs + tab_sq_bytes(g));
  }
  if (g.adj && Z > 1) return run_adjoint_sum(a, g, Z, in, out, T, U, s, pw, ph, mx_tabs);
  // square 300-point grids (cfg4 / cfg5): the first z-chunk's column tables ride along with K1
  // (tf_tables_body<PN> of K1's own size: Ph == Pw)
  a.tab_blocks = mx_tabs && g.Pw == g.Ph && g.Pw == Mx300::N ? g.C * g.ncols : 0;
  {
    KernelTimer kt("asm_rows_fwd", s);
    a.zoff = 0;
    a.nz = std::min(g.zc, Z);
    if (k1_mid(g.Pw, a)) {
      hipLaunchKernelGGL((asm_rows_fwd<Mx300::N, true>), dim3(g.BC * g.Hin + a.tab_blocks), dim3(MX_T),
                         fft_lds_bytes_io(g.Pw), s, (const float2*)in, T, pw, a);
    } else {
      THZ_ROWS_SWITCH(g.Pw, asm_rows_fwd, dim3(g.BC * g.Hin + a.tab_blocks), fft_lds_bytes_io(g.Pw), s,
                      (const float2*)in, T, pw, a);
    }
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  for (int z0 = 0; z0 < Z; z0 += g.zc) {
    a.zoff = z0;
    a.nz = std::min(g.zc, Z - z0);
    {
      KernelTimer kt("asm_cols", s);
      if (mx_kind(g.Ph)) {
        if (mx_tabs && !(z0 == 0 && a.tab_blocks)) {
          THZ_MX_TABLES(g.Ph, dim3(g.C * g.ncols), dim3(MX_T), 0, s, a, z0 == 0);
          THZ_LAUNCH_CHECK();
        }
      }
      if (mx_kind(g.Ph)) {
        const size_t lds2 = lds_floats2(g.Ph) * sizeof(float2) + 4 * THZ_MAX_Z;
        const int ntask = k2_tasks(g, &a, mx_threads(g.Ph), lds2);
        if (g.Ph == Mx300::N && mx_mid(a))
          hipLaunchKernelGGL(asm_cols_mx_mid<Mx300>, dim3(ntask), dim3(MX_T), lds2, s, (const float2*)T, U, ph, a);
        else
          THZ_MX_COLS(g.Ph, asm_cols_mx, dim3(ntask), dim3(mx_threads(g.Ph)), lds2, s, (const float2*)T, U, ph, a);
      } else {
        const size_t lds2 = fft_lds_bytes(g.Ph) + 12 * THZ_MAX_Z;  // mz, zok and the z values
        const int ntask = k2_tasks(g, &a, th, lds2);
        a.zrec = !plane_recurrence_disabled();
        THZ_POW2_SWITCH(g.Ph, asm_cols, dim3(ntask), dim3(th), lds2, s, (const float2*)T, U, ph, a);
      }
      THZ_LAUNCH_CHECK();
      kt.stop();
    }
    {
      KernelTimer kt("asm_rows_inv", s);
      if (a.ls.stats) {
        if (g.Pw == Mx300::N && k3_mid(g.Pw, a)) {
          hipLaunchKernelGGL(asm_rows_inv_loss_mid<Mx300::N>, dim3(a.nz * g.BC * g.Hout), dim3(MX_T),
                             fft_lds_bytes_io(g.Pw), s, (const float2*)U, (float2*)out, pw, a);
        } else {
          THZ_ROWS_SWITCH(g.Pw, asm_rows_inv_loss, dim3(a.nz * g.BC * g.Hout), fft_lds_bytes_io(g.Pw), s,
                          (const float2*)U, (float2*)out, pw, a);
        }
        THZ_LAUNCH_CHECK();
        if ((e = launch_loss_finish(a.ls, s))) return e;
      } else if (k3_mid(g.Pw, a)) {
        if (g.Pw == 8192)
          hipLaunchKernelGGL(asm_rows_inv_mid<8192>, dim3(a.nz * g.BC * g.Hout), dim3(threads_for(8192)),
                             fft_lds_bytes_io(8192), s, (const float2*)U, (float2*)out, pw, a);
        else
          hipLaunchKernelGGL(asm_rows_inv_mid<Mx300::N>, dim3(a.nz * g.BC * g.Hout), dim3(MX_T),
                             fft_lds_bytes_io(g.Pw), s, (const float2*)U, (float2*)out, pw, a);
      } else {
        THZ_ROWS_SWITCH(g.Pw, asm_rows_inv, dim3(a.nz * g.BC * g.Hout), fft_lds_bytes_io(g.Pw), s, (const float2*)U,
                        (float2*)out, pw, a);
      }
      THZ_LAUNCH_CHECK();
      kt.stop();
    }
  }
  return THZ_OK;
}

}  // namespace thz

using namespace thz;

extern "C" int thz_asm_band(const thz_asm_desc* d, int* ncols, int* z_chunk) {
  int e = validate(d);
  if (e) return e;
  AsmGeom g;
  geometry(d, &g);
  if (ncols) *ncols = g.ncols;
  if (z_chunk) *z_chunk = g.zc;
  return THZ_OK;
}

extern "C" int thz_asm_workspace_size(const thz_asm_desc* d, size_t* bytes) {
  int e = validate(d);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  AsmGeom g;
  geometry(d, &g);
  *bytes = ws_bytes(g);
  return THZ_OK;
}

namespace thz {
static int asm_forward_impl(const thz_asm_desc* d, const thz_doe_desc* m, const float* mh, const float* mu,
                            float* mhfull, const void* in, void* out, void* workspace, size_t workspace_bytes,
                            thz_stream_t stream, const LossSink* ls = nullptr, const thz_loss_desc* lg = nullptr,
                            const float2* lg_field = nullptr, const float* lg_target = nullptr,
                            const float* lg_stats = nullptr, const float* lg_gloss = nullptr) {
  int e = validate(d);
  if (e) return e;
  if ((!in && !lg_field) || !out) return fail(THZ_E_ARG, "null data pointer");
  AsmGeom g;
  geometry(d, &g);
  const size_t need = ws_bytes(g);
  if (!workspace || workspace_bytes < need)
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  FftPlan pw, ph;
  if ((e = get_plan(g.Pw, &pw))) return e;
  if ((e = get_plan(g.Ph, &ph))) return e;

  AsmArgs a{};
  a.BC = g.BC;
  a.C = d->C;
  a.Ph = g.Ph;
  a.Pw = g.Pw;
  const int Ho = d->unpad ? d->H : g.Ph, Wo = d->unpad ? d->W : g.Pw;
  const int o_r0 = d->unpad ? d->pad_h : 0, o_c0 = d->unpad ? d->pad_w : 0;
  if (!d->adjoint) {
    a.in_r0 = d->pad_h; a.in_c0 = d->pad_w; a.Hin = d->H; a.Win = d->W;
    a.out_r0 = o_r0; a.out_c0 = o_c0; a.Hout = Ho; a.Wout = Wo;
  } else {
    a.in_r0 = o_r0; a.in_c0 = o_c0; a.Hin = Ho; a.Win = Wo;
    a.out_r0 = d->pad_h; a.out_c0 = d->pad_w; a.Hout = d->H; a.Wout = d->W;
  }
  a.ncols = g.ncols;
  a.ncb = g.ncb;
  a.ncbu = g.ncbu;
  a.J = g.J;
  a.bl = d->bandlimit;
  a.adjoint = d->adjoint;
  a.dx = d->dx;
  a.dy = d->dy;
  a.scale = (float)(1.0 / ((double)g.Ph * (double)g.Pw));
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  if (d->z)
    for (int zi = 0; zi < d->Z; ++zi) a.zv[zi] = d->z[zi];
  a.zdev = d->z_dev;
  if (m) {
    a.mod_h = mh;
    a.mod_u = mu;
    a.mod_hfull = mhfull;
    a.mod_hs = m->hs;
    a.mod_ws = m->ws;
    a.mod_tol = m->tolerance;
    a.mod_eps = m->epsilon;
    a.mod_tand = m->tand;
    a.mod_rng = m->rng;
    a.mod_rng_stream = m->rng_stream;
  }
  if (d->window_mask) {
    const thz_aperture_desc* w = d->window_mask;
    if (w->kind != THZ_APERTURE_RECT && w->kind != THZ_APERTURE_CIRC)
      return fail(THZ_E_ARG, "window mask: bad aperture kind %d", w->kind);
    if (w->H != Ho || w->W != Wo)
      return fail(THZ_E_ARG, "window mask %dx%d does not match the output grid %dx%d", w->H, w->W, Ho, Wo);
    a.apm = aperture_args(w, Ho, Wo);
    a.ap_side = d->adjoint ? 2 : 1;
    // carried by the 300-point row passes only (the K3 storer forward, the K1 loader adjoint:
    // asm_rows_inv<300> / asm_rows_fwd<300>)
    if (mx_kind(g.Pw) != Mx300::N)
      return fail(THZ_E_UNSUPPORTED, "window mask: only the 300-point row passes fold the aperture; "
                                     "apply it separately");
    if (d->adjoint && d->Z > 1)
      return fail(THZ_E_UNSUPPORTED, "window mask: one z-plane per adjoint call");
  }
  if (ls) a.ls = *ls;
  if (lg_field) {  // the adjoint pipeline starts from the loss gradient
    a.lg_field = lg_field;
    a.lg_gloss = lg_gloss;
    a.lg_target = lg_target;
    a.lg_stats = lg_stats;
    a.lg_tB = lg->tB;
    a.lg_tC = lg->tC;
    // the loss of a Z-plane pipeline is the sum of the planes' means (thz_asm_forward_loss)
    a.lg_two_inv_n = (float)(2.0 * d->Z / ((double)lg->B * lg->C * lg->H * lg->W));
  }

  float2* T = (float2*)workspace;
  float2* U = (float2*)((char*)workspace + t_bytes(g));
  char* tabs = (char*)workspace + ws_bytes(g) - tab_bytes(g);
  return run_pipeline(a, g, d->Z, in, out, T, U, (hipStream_t)stream, pw, ph, tab_bytes(g) ? tabs : nullptr);
}
}  // namespace thz

extern "C" int thz_asm_forward(const thz_asm_desc* d, const void* in, void* out, void* workspace,
                               size_t workspace_bytes, thz_stream_t stream) {
  return asm_forward_impl(d, nullptr, nullptr, nullptr, nullptr, in, out, workspace, workspace_bytes, stream);
}

namespace thz {
// ASM_prop.create_kernel (Props/ASM_Prop.py:212-311): H of one z on the CENTRED grid of the padded
// plane, [C][Ph][Pw], the row i / column j at spectral index m = i - Ph/2 (:141-145).  The same
// fp32 scalars, masks and phase as the propagation kernels (tf_scalars / tf_value), so the table
// is exactly the transfer function they apply on the fly; only inspection reads it
// (ASM_prop.visualize_kernel).
__global__ void __launch_bounds__(256) asm_tf_export(float2* __restrict__ out, AsmArgs a) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y, c = blockIdx.z;
  if (j >= a.Pw) return;
  const TfScalars s = tf_scalars(a, a.lam[c], a.zv[0]);
  const float Kx = kfreq(i - a.Ph / 2, a.Ph, a.dx), Ky = kfreq(j - a.Pw / 2, a.Pw, a.dy);
  out[((size_t)c * a.Ph + i) * a.Pw + j] = tf_value(a, s, Kx, Ky);
}
}  // namespace thz

extern "C" int thz_asm_transfer_function(const thz_asm_desc* d, void* out, thz_stream_t stream) {
  int e = validate(d);
  if (e) return e;
  if (!out) return fail(THZ_E_ARG, "null output pointer");
  if (!d->z) return fail(THZ_E_ARG, "the transfer-function table takes a host z");
  AsmGeom g;
  geometry(d, &g);
  AsmArgs a{};
  a.C = d->C;
  a.Ph = g.Ph;
  a.Pw = g.Pw;
  a.bl = d->bandlimit;
  a.dx = d->dx;
  a.dy = d->dy;
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  a.zv[0] = d->z[0];
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("asm_tf_export", s);
  hipLaunchKernelGGL(asm_tf_export, dim3((g.Pw + 255) / 256, g.Ph, d->C), dim3(256), 0, s, (float2*)out, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_asm_forward_modulated(const thz_asm_desc* d, const thz_doe_desc* m, const void* field,
                                         const float* height, const float* noise, float* height_full, void* out,
                                         void* workspace, size_t workspace_bytes, thz_stream_t stream) {
  if (!d || !m || !height) return fail(THZ_E_ARG, "null descriptor / height");
  if (d->adjoint) return fail(THZ_E_ARG, "the fused DOE modulation is forward only");
  if (m->B != d->B || m->C != d->C || m->H != d->H || m->W != d->W)
    return fail(THZ_E_ARG, "DOE field %dx%dx%dx%d does not match the ASM input %dx%dx%dx%d", m->B, m->C, m->H, m->W,
                d->B, d->C, d->H, d->W);
  if (m->hs < 1 || m->ws < 1) return fail(THZ_E_ARG, "bad height-map size %dx%d", m->hs, m->ws);
  return asm_forward_impl(d, m, height, noise, height_full, field, out, workspace, workspace_bytes, stream);
}

extern "C" int thz_asm_adjoint_loss(const thz_asm_desc* d, const thz_loss_desc* l, const void* field,
                                     const float* target, const float* stats, const float* grad_loss,
                                     const void* grad_out, void* grad_in, void* workspace, size_t workspace_bytes,
                                     thz_stream_t stream) {
  int e = validate(d);
  if (e) return e;
  if (!l || !field || !target || !stats || !grad_loss || !grad_in)
    return fail(THZ_E_ARG, "null loss descriptor / field / target / stats / grad_loss / grad_in");
  if (!d->adjoint) return fail(THZ_E_ARG, "the fused loss adjoint takes adjoint == 1");
  const int Ho = d->unpad ? d->H : d->H + 2 * d->pad_h, Wo = d->unpad ? d->W : d->W + 2 * d->pad_w;
  if (l->B != d->Z * d->B || l->C != d->C || l->H != Ho || l->W != Wo)
    return fail(THZ_E_ARG, "loss field %dx%dx%dx%d does not match the ASM output %dx%dx%dx%d", l->B, l->C, l->H, l->W,
                d->B, d->C, Ho, Wo);
  if (!(l->tB == 1 || l->tB == l->B) || !(l->tC == 1 || l->tC == l->C))
    return fail(THZ_E_ARG, "target %dx%d does not broadcast over %dx%d", l->tB, l->tC, l->B, l->C);
  return asm_forward_impl(d, nullptr, nullptr, nullptr, nullptr, grad_out, grad_in, workspace, workspace_bytes, stream,
                          nullptr, l, (const float2*)field, target, stats, grad_loss);
}

extern "C" int thz_asm_forward_loss(const thz_asm_desc* d, const thz_doe_desc* m, const void* field,
                                    const float* height, const float* noise, float* height_full,
                                    const thz_loss_desc* l, const float* target, void* out, float* loss, float* stats,
                                    void* workspace, size_t workspace_bytes, thz_stream_t stream) {
  int e = validate(d);
  if (e) return e;
  if (!l || !target || !loss || !stats) return fail(THZ_E_ARG, "null loss descriptor / target / loss / stats");
  if (d->adjoint) return fail(THZ_E_ARG, "the fused loss is forward only (thz_asm_adjoint_loss)");
  const int Ho = d->unpad ? d->H : d->H + 2 * d->pad_h, Wo = d->unpad ? d->W : d->W + 2 * d->pad_w;
  if (l->B != d->Z * d->B || l->C != d->C || l->H != Ho || l->W != Wo)
    return fail(THZ_E_ARG, "loss field %dx%dx%dx%d does not match the ASM output %dx%dx%dx%d", l->B, l->C, l->H, l->W,
                d->B, d->C, Ho, Wo);
  if (!(l->tB == 1 || l->tB == l->B) || !(l->tC == 1 || l->tC == l->C))
    return fail(THZ_E_ARG, "target %dx%d does not broadcast over %dx%d", l->tB, l->tC, l->B, l->C);
  if (m) {
    if (!height) return fail(THZ_E_ARG, "null height map");
    if (m->B != d->B || m->C != d->C || m->H != d->H || m->W != d->W)
      return fail(THZ_E_ARG, "DOE field %dx%dx%dx%d does not match the ASM input %dx%dx%dx%d", m->B, m->C, m->H,
                  m->W, d->B, d->C, d->H, d->W);
    if (m->hs < 1 || m->ws < 1) return fail(THZ_E_ARG, "bad height-map size %dx%d", m->hs, m->ws);
  }
  const LossSink ls = loss_sink(l, target, loss, stats, l->C * l->H, d->Z);
  return asm_forward_impl(d, m, m ? height : nullptr, m ? noise : nullptr, m ? height_full : nullptr, field, out,
                          workspace, workspace_bytes, stream, &ls);
}

namespace thz {
// rows transforms of length n, row r at in/out + r * stride (in place allowed): one launch
int fft_rows_strided(const void* in, void* out, int rows, int n, size_t stride, int inverse, hipStream_t s) {
  if (!in || !out || rows < 1 || stride < (size_t)n) return fail(THZ_E_ARG, "bad fft_rows arguments");
  FftPlan p;
  int e = get_plan(n, &p);
  if (e) return e;
  if ((e = ensure_lds_attr())) return e;
  THZ_POW2_SWITCH(n, fft_rows_kernel, dim3(rows), dim3(threads_for(n)), fft_lds_bytes_io(n), s, (const float2*)in,
                  (float2*)out, p, inverse, stride);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}
}  // namespace thz

extern "C" int thz_fft_rows(const void* in, void* out, int rows, int n, int inverse, thz_stream_t stream) {
  return fft_rows_strided(in, out, rows, n, (size_t)n, inverse, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------------------------
// RSC / VRS C-ABI
// ---------------------------------------------------------------------------------------------
namespace thz {

struct RscPlan {
  AsmGeom g;
  RscKArgs k;
  size_t tk, kf, t, u;  // byte sizes
};

static int rsc_plan(const thz_rsc_desc* d, RscPlan* p) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1) return fail(THZ_E_ARG, "bad RSC shape");
  if (d->vectorial && d->B < 2) return fail(THZ_E_ARG, "vectorial RSC needs Ex, Ey planes (B >= 2)");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  if (!d->wavelengths) return fail(THZ_E_ARG, "null wavelengths");
  AsmGeom& g = p->g;
  g.Ph = d->H + 2 * (d->H / 2);
  g.Pw = d->W + 2 * (d->W / 2);
  if (g.Ph > FFT_MAX_N || g.Pw > FFT_MAX_N) return fail(THZ_E_UNSUPPORTED, "RSC grid %dx%d too large", g.Ph, g.Pw);
  g.BC = (d->vectorial ? 3 : d->B) * d->C;
  if (d->adjoint && d->vectorial) return fail(THZ_E_ARG, "RSC adjoint is per plane: vectorial must be 0");
  g.Hin = d->adjoint ? g.Ph - d->H : d->H;
  g.Win = d->adjoint ? g.Pw - d->W : d->W;
  g.Hout = d->adjoint ? d->H : g.Ph - d->H;  // ifft2(...)[..., H:, W:] (:207)
  g.Wout = d->adjoint ? d->W : g.Pw - d->W;
  g.ncols = g.Pw;
  g.J = g.Pw / 2;
  g.ncb = (g.ncols + CB - 1) / CB;
  g.ncbu = (g.ncols + CBU - 1) / CBU;
  g.zc = 1;
  g.adj = 0;
  g.C = d->C;
  RscKArgs& k = p->k;
  k.C = d->C;
  k.Ph = g.Ph;
  k.Pw = g.Pw;
  k.ncbK = g.ncb;
  k.dx = d->dx;
  k.z = d->z;
  for (int c = 0; c < d->C; ++c) k.lam[c] = d->wavelengths[c];
  p->tk = align256((size_t)d->C * k.ncbK * CB * g.Ph * sizeof(float2));
  p->kf = align256((size_t)d->C * g.Pw * g.Ph * sizeof(float2));
  p->t = align256((size_t)g.BC * g.ncb * CB * g.Hin * sizeof(float2));
  p->u = align256((size_t)g.BC * g.ncbu * CBU * u_rows(g.Hout) * sizeof(float2));
  return THZ_OK;
}

}  // namespace thz

extern "C" int thz_rsc_workspace_size(const thz_rsc_desc* d, size_t* bytes) {
  RscPlan p;
  int e = rsc_plan(d, &p);
  if (e) return e;
  if (!bytes) return fail(THZ_E_ARG, "null bytes");
  *bytes = p.tk + p.kf + p.t + p.u;
  return THZ_OK;
}

extern "C" int thz_rsc_forward(const thz_rsc_desc* d, const void* in, void* out, void* workspace,
                               size_t workspace_bytes, thz_stream_t stream) {
  RscPlan p;
  int e = rsc_plan(d, &p);
  if (e) return e;
  if (!in || !out) return fail(THZ_E_ARG, "null data pointer");
  if (!workspace || workspace_bytes < p.tk + p.kf + p.t + p.u)
    return fail(THZ_E_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, p.tk + p.kf + p.t + p.u);
  if ((e = ensure_lds_attr())) return e;
  const AsmGeom& g = p.g;
  FftPlan pw, ph;
  if ((e = get_plan(g.Pw, &pw))) return e;
  if ((e = get_plan(g.Ph, &ph))) return e;
  hipStream_t s = (hipStream_t)stream;
  char* w = (char*)workspace;
  float2* TK = (float2*)w;
  float2* KF = (float2*)(w + p.tk);
  float2* T = (float2*)(w + p.tk + p.kf);
  float2* U = (float2*)(w + p.tk + p.kf + p.t);
  {
    KernelTimer kt("rsc_kernel_fft", s);
    THZ_POW2_SWITCH(g.Pw, rsc_k_rows, dim3(d->C * g.Ph), dim3(threads_for(g.Pw)), fft_lds_bytes_io(g.Pw), s, TK, pw,
                    p.k);
    THZ_LAUNCH_CHECK();
    THZ_POW2_SWITCH(g.Ph, rsc_k_cols, dim3(d->C * g.Pw), dim3(threads_for(g.Ph)), fft_lds_bytes_io(g.Ph), s,
                    (const float2*)TK, KF, ph, p.k);
    THZ_LAUNCH_CHECK();
    kt.stop();
  }
  AsmArgs a{};
  a.BC = g.BC;
  a.C = d->C;
  a.Ph = g.Ph;
  a.Pw = g.Pw;
  if (!d->adjoint) {
    a.in_r0 = 0; a.in_c0 = 0; a.Hin = d->H; a.Win = d->W;         // U[..., :H, :W] = field (:198-200)
    a.out_r0 = d->H; a.out_c0 = d->W; a.Hout = g.Hout; a.Wout = g.Wout;
  } else {  // adjoint: gradient placed at [H:, W:], result read back from [:H, :W]
    a.in_r0 = d->H; a.in_c0 = d->W; a.Hin = g.Hin; a.Win = g.Win;
    a.out_r0 = 0; a.out_c0 = 0; a.Hout = g.Hout; a.Wout = g.Wout;
    a.adjoint = 1;
  }
  a.ncols = g.ncols;
  a.ncb = g.ncb;
  a.ncbu = g.ncbu;
  a.J = g.J;
  a.bl = THZ_BANDLIMIT_NONE;
  a.dx = d->dx;
  a.dy = d->dy;
  a.scale = (float)((double)d->dx * (double)d->dy / ((double)g.Ph * (double)g.Pw));
  a.tft = KF;
  a.vec = d->vectorial;
  a.zr = d->z;
  a.lam[0] = d->wavelengths[0];
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  a.zv[0] = d->z;
  return run_pipeline(a, g, 1, in, out, T, U, s, pw, ph);
}
