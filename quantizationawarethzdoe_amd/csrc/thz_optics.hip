// Optical elements around the DOE and the QAT loss, for gfx950.
//
//  * Gaussian source   LightSource/Gaussian_beam.py:88-160  E = A(x, y) exp(-i phi(x, y)); the
//                      per-wavelength scalars (waist, Rayleigh range, Gouy phase, spot size,
//                      curvature) are fp32 host values in the reference's op order, the per-pixel
//                      part runs here (no host-built grid, no H2D copy).
//  * thin lens         Components/Thin_Lens.py:31-58    field * exp(i ang), ang = -(pi/(lambda f)) r^2
//  * aperture          Components/Aperture.py:44-136    field * mask (rect: 'xy' grid, circ: 'ij')
//  * |E|^2 -> normalize -> MSE   utils/Helper_Functions.py:185-193 + nn.MSELoss
//                      (experiment_four_focal_spots.ipynb:336-370): one workgroup per batch item
//                      finds max / argmax of |E|^2, the squared error and the sum the backward's
//                      max-path needs; the backward is then one elementwise pass.
#include <algorithm>
#include <cmath>

#include "thz_common.hpp"
#include "thz_dev.hpp"

#pragma clang fp contract(off)

namespace thz {

struct GaussArgs {
  int C, H, W;
  float x_start, x_end, y_start, y_end;
  float x0, y0, ca, sa;
  float k[THZ_MAX_WAVELENGTHS], kz_x[THZ_MAX_WAVELENGTHS], kz_y[THZ_MAX_WAVELENGTHS];
  float two_rx[THZ_MAX_WAVELENGTHS], two_ry[THZ_MAX_WAVELENGTHS];
  float gouy_x[THZ_MAX_WAVELENGTHS], gouy_y[THZ_MAX_WAVELENGTHS];
  float amp[THZ_MAX_WAVELENGTHS], wx2[THZ_MAX_WAVELENGTHS], wy2[THZ_MAX_WAVELENGTHS];
};

__global__ void gaussian_beam_kernel(float2* __restrict__ out, GaussArgs a) {
  const int HW = a.H * a.W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HW) return;
  const int i = p / a.W, j = p - i * a.W;
  const float X = lin(a.x_start, a.x_end, a.H, i);  // meshgrid 'ij': X follows the height axis
  const float Y = lin(a.y_start, a.y_end, a.W, j);
  const float xr = X * a.ca + Y * a.sa;
  const float yr = -X * a.sa + Y * a.ca;
  const float dx = xr - a.x0, dy = yr - a.y0;
  for (int c = 0; c < a.C; ++c) {
    const float ph = ((a.kz_x[c] + (a.k[c] * (X * X)) / a.two_rx[c]) - a.gouy_x[c]) +
                     ((a.kz_y[c] + (a.k[c] * (Y * Y)) / a.two_ry[c]) - a.gouy_y[c]);
    const float A = a.amp[c] * expf(-(dx * dx) / a.wx2[c] - (dy * dy) / a.wy2[c]);
    float sn, cs;
    sincos_rad(ph, &sn, &cs);
    out[(size_t)c * HW + p] = make_float2(A * cs, -(A * sn));  // A exp(-i ph)
  }
}

struct LensArgs {
  int B, C, H, W;
  float gx0, gx1, gy0, gy1;  // linspace(-((n-1)//2), (n-1)//2, n) end points
  float dx, dy;
  float coef[THZ_MAX_WAVELENGTHS];  // pi / (lambda f), fp32
};

__global__ void __launch_bounds__(EW_THREADS) thin_lens_kernel(const float2* __restrict__ in,
                                                               float2* __restrict__ out, LensArgs a) {
  const float coef = a.coef[blockIdx.y];
  ew_scale_pairs(in, out, a.B, a.C, a.H * a.W, [&](int p) {
    const int i = p / a.W, j = p - i * a.W;
    const float xg = lin(a.gx0, a.gx1, a.H, i) * a.dx;
    const float yg = lin(a.gy0, a.gy1, a.W, j) * a.dy;
    // x^2 + y^2 rounded term by term as the reference's xg ** 2 + yg ** 2 (no fma contraction)
    const float r2 = __fadd_rn(__fmul_rn(xg, xg), __fmul_rn(yg, yg));
    float sn, cs;
    sincos_rad(-coef * r2, &sn, &cs);
    return make_float2(cs, sn);
  });
}

// the mask as a complex factor (1 or 0), evaluated once per pixel: NaN / inf propagate as in the
// reference's product field * mask
__global__ void __launch_bounds__(EW_THREADS) aperture_kernel(const float2* __restrict__ in,
                                                             float2* __restrict__ out, ApertureArgs a) {
  ew_scale_pairs(in, out, a.BC, 1, a.H * a.W, [&](int p) {
    return aperture_open(a, p / a.W, p % a.W) ? make_float2(1.f, 0.f) : make_float2(0.f, 0.f);
  });
}

// ---------------------------------------------------------------------------------------------
// |E|^2 -> normalize (per batch item, by its max) -> MSE against a broadcast target, as the
// one-pass sums of thz_dev.hpp (LossAcc / loss_store_part): a grid of (chunks, B) workgroups, one
// slot each, then loss_finish_kernel.  stats[b] = {max, argmax (as float bits), sum_i r_i I_i}, r_i = I_i/m - T_i.
// (The ASM path folds the same accumulation into its row-inverse pass: thz_asm_forward_loss.)
// ---------------------------------------------------------------------------------------------
constexpr int LOSS_THREADS = 256;
constexpr int LOSS_PER_THREAD = 8;

struct LossArgs {
  int B, C, H, W, tB, tC;
};

__device__ __forceinline__ float target_at(const float* t, const LossArgs& a, int b, int c, int p) {
  const int tb = a.tB == 1 ? 0 : b, tc = a.tC == 1 ? 0 : c;
  return t[((size_t)tb * a.tC + tc) * a.H * a.W + p];
}

__device__ __forceinline__ float intensity(float2 e) { return loss_intensity(e); }

__global__ void __launch_bounds__(LOSS_THREADS) mse_forward_kernel(const float2* __restrict__ f, LossArgs a,
                                                                   LossSink ls) {
  const int b = blockIdx.y;
  const int HW = a.H * a.W, n = a.C * HW;
  const float2* fb = f + (size_t)b * n;
  LossAcc acc;
  const int i0 = blockIdx.x * LOSS_THREADS * LOSS_PER_THREAD + threadIdx.x;
#pragma unroll
  for (int k = 0; k < LOSS_PER_THREAD; ++k) {
    const int i = i0 + k * LOSS_THREADS;
    if (i < n) {
      const int c = i / HW, p = i - c * HW;
      acc.add(fb[i], target_at(ls.target, a, b, c, p), (unsigned)i);
    }
  }
  loss_store_part(acc, ls, b, blockIdx.x);
}

// One workgroup per batch item: reduce its per_b slots (fixed order), write its statistics and
// loss term; the last workgroup to finish sums the B terms in order into the loss.
constexpr int FIN_THREADS = 256;
__global__ void __launch_bounds__(FIN_THREADS) loss_finish_kernel(LossSink ls) {
  __shared__ LossPart s_a[FIN_THREADS / 64];
  __shared__ int s_last;
  const int b = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const LossPart* pp = ls.parts() + (size_t)b * ls.per_b;
  LossAcc acc;
  for (int q = threadIdx.x; q < ls.per_b; q += FIN_THREADS) {
    const LossPart p = pp[q];
    acc.merge(LossAcc::of(p));
  }
  for (int o = 32; o > 0; o >>= 1) {
    LossAcc t;
    t.ii = __shfl_xor(acc.ii, o);
    t.it = __shfl_xor(acc.it, o);
    t.tt = __shfl_xor(acc.tt, o);
    t.key = __shfl_xor(acc.key, o);
    acc.merge(t);
  }
  if (lane == 0) s_a[wid] = acc.part();
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < FIN_THREADS / 64; ++w) acc.merge(LossAcc::of(s_a[w]));
    const float m = __uint_as_float((unsigned)(acc.key >> 32));
    const double md = m;
    ls.stats[3 * b + 0] = m;
    ls.stats[3 * b + 1] = __int_as_float((int)(0xffffffffu - (unsigned)acc.key));
    ls.stats[3 * b + 2] = (float)(acc.ii / md - acc.it);
    if (ls.B == 1) {
      // one item (cfg4): its term is the sum -- the same value the path below forms (0.0 + x and
      // x + 0.0 are exact), without its write-through store, arrival atomic and reload: three
      // dependent memory round trips of a kernel every QAT step runs
      ls.loss[0] = (float)((acc.ii / (md * md) - 2.0 * acc.it / md + acc.tt) * ls.inv_n);
      s_last = 0;
    } else {
      // the term written through to memory (an agent-scope atomic store) and its completion awaited
      // before the arrival is counted: the release the last workgroup needs, without the L2
      // write-back of an agent-scope fence (which every one of B workgroups would pay)
      __hip_atomic_store(ls.terms() + b, acc.ii / (md * md) - 2.0 * acc.it / md + acc.tt, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
      s_last = atomicAdd(ls.counter(), 1ull) == (unsigned long long)(ls.B - 1);
    }
  }
  __syncthreads();
  if (!s_last) return;
  double part = 0.0;  // B terms in order: thread t sums a contiguous run
  const int per = (ls.B + FIN_THREADS - 1) / FIN_THREADS;
  for (int q = threadIdx.x * per; q < min(ls.B, (threadIdx.x + 1) * per); ++q)
    part += __hip_atomic_load(ls.terms() + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int o = 1; o < 64; o <<= 1) {  // ordered tree over the lanes
    const double t = __shfl_down(part, o);
    if ((lane & (2 * o - 1)) == 0 && lane + o < 64) part += t;
  }
  __syncthreads();
  if (lane == 0) s_a[wid].ii = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int w = 0; w < FIN_THREADS / 64; ++w) tot += s_a[w].ii;
    ls.loss[0] = (float)(tot * ls.inv_n);
  }
}

int launch_loss_finish(const LossSink& ls, hipStream_t s) {
  hipLaunchKernelGGL(loss_finish_kernel, dim3(ls.B), dim3(FIN_THREADS), 0, s, ls);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}

// dL/dE = 2 E dL/dI;  dL/dI_j = g (r_j / m - [j == argmax] sum_i r_i I_i / m^2),  g = 2 grad / N
__global__ void mse_backward_kernel(const float2* __restrict__ f, const float* __restrict__ t,
                                    const float* __restrict__ stats, const float* __restrict__ grad_loss,
                                    float2* __restrict__ gf, LossArgs a, float two_inv_n) {
  const int HW = a.H * a.W, n = a.C * HW;
  const size_t total = (size_t)a.B * n;
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= total) return;
  const int b = (int)(q / n), i = (int)(q - (size_t)b * n);
  const int c = i / HW, p = i - c * HW;
  const float m = stats[3 * b], S = stats[3 * b + 2];
  const int am = __float_as_int(stats[3 * b + 1]);
  const float g = grad_loss[0] * two_inv_n;
  const float2 e = f[q];
  const float I = intensity(e);
  const float r = I / m - target_at(t, a, b, c, p);
  float dI = g * r / m;
  if (i == am) dI -= g * S / (m * m);
  gf[q] = make_float2(2.f * dI * e.x, 2.f * dI * e.y);
}

// ---------------------------------------------------------------------------------------------
// Field_Resampler (Addons/Field_Resampler.py:19-118): bilinear grid_sample (zeros padding,
// align_corners=True) of the complex field onto the centred output grid; adjoint by scatter.
// ---------------------------------------------------------------------------------------------
struct ResampleArgs {
  int BC, Hin, Win, Hout, Wout;
  float gx0, gx1, gy0, gy1;  // linspace(-((n-1)//2), (n-1)//2, n) end points of the output grid
  float dxo, dyo, xnorm, ynorm;
};

struct Taps {
  int x0, y0;
  float w[4];  // nw, ne, sw, se
};

// torch grid_sampler_compute_source_index (align_corners) + the bilinear weights, fp32
__device__ __forceinline__ Taps resample_taps(const ResampleArgs& a, int i, int j) {
  const float gX = lin(a.gx0, a.gx1, a.Hout, i) * a.dxo;  // height coordinate of output row i
  const float gY = lin(a.gy0, a.gy1, a.Wout, j) * a.dyo;  // width coordinate of output column j
  const float gx = gY / a.ynorm, gy = gX / a.xnorm;       // grid[..., 0] (W), grid[..., 1] (H)
  const float ix = ((gx + 1.0f) / 2.0f) * (float)(a.Win - 1);
  const float iy = ((gy + 1.0f) / 2.0f) * (float)(a.Hin - 1);
  const float fx = floorf(ix), fy = floorf(iy);
  Taps t;
  t.x0 = (int)fx;
  t.y0 = (int)fy;
  const float xe = fx + 1.0f, ye = fy + 1.0f;
  t.w[0] = (xe - ix) * (ye - iy);
  t.w[1] = (ix - fx) * (ye - iy);
  t.w[2] = (xe - ix) * (iy - fy);
  t.w[3] = (ix - fx) * (iy - fy);
  if (!(ix == ix) || !(iy == iy)) t.x0 = t.y0 = -(1 << 30);  // NaN grid: every tap out of range
  return t;
}

__global__ void resample_fwd(const float2* __restrict__ in, float2* __restrict__ out, ResampleArgs a) {
  const int HWo = a.Hout * a.Wout;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HWo) return;
  const int i = p / a.Wout, j = p - i * a.Wout;
  const Taps t = resample_taps(a, i, j);
  const int HWi = a.Hin * a.Win;
  for (int bc = 0; bc < a.BC; ++bc) {
    const float2* src = in + (size_t)bc * HWi;
    float re = 0.f, im = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = t.x0 + (k & 1), y = t.y0 + (k >> 1);
      if (x >= 0 && x < a.Win && y >= 0 && y < a.Hin) {
        const float2 v = src[(size_t)y * a.Win + x];
        re = re + v.x * t.w[k];
        im = im + v.y * t.w[k];
      }
    }
    out[(size_t)bc * HWo + p] = make_float2(re, im);
  }
}

__global__ void resample_bwd(const float2* __restrict__ g, float2* __restrict__ gin, ResampleArgs a) {
  const int HWo = a.Hout * a.Wout;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= HWo) return;
  const int i = p / a.Wout, j = p - i * a.Wout;
  const Taps t = resample_taps(a, i, j);
  const int HWi = a.Hin * a.Win;
  for (int bc = 0; bc < a.BC; ++bc) {
    const float2 gv = g[(size_t)bc * HWo + p];
    float* dst = reinterpret_cast<float*>(gin + (size_t)bc * HWi);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = t.x0 + (k & 1), y = t.y0 + (k >> 1);
      if (x >= 0 && x < a.Win && y >= 0 && y < a.Hin) {
        const size_t o = 2 * ((size_t)y * a.Win + x);
        atomicAdd(dst + o, gv.x * t.w[k]);
        atomicAdd(dst + o + 1, gv.y * t.w[k]);
      }
    }
  }
}

static bool resample_args(const thz_resample_desc* d, ResampleArgs* a) {
  if (!d || d->BC < 1 || d->Hin < 1 || d->Win < 1 || d->Hout < 1 || d->Wout < 1) return false;
  a->BC = d->BC; a->Hin = d->Hin; a->Win = d->Win; a->Hout = d->Hout; a->Wout = d->Wout;
  a->gx0 = (float)(-((d->Hout - 1) / 2));
  a->gx1 = (float)((d->Hout - 1) / 2);
  a->gy0 = (float)(-((d->Wout - 1) / 2));
  a->gy1 = (float)((d->Wout - 1) / 2);
  a->dxo = d->dx_out;
  a->dyo = d->dy_out;
  a->xnorm = d->dx_in * (float)((d->Hin - 1) / 2);  // dx * ((Hf - 1) // 2), fp32 (:82-85)
  a->ynorm = d->dy_in * (float)((d->Win - 1) / 2);
  return true;
}

static bool loss_args(const thz_loss_desc* d, LossArgs* a) {
  if (!d || d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1) return false;
  if (!(d->tB == 1 || d->tB == d->B) || !(d->tC == 1 || d->tC == d->C)) return false;
  *a = LossArgs{d->B, d->C, d->H, d->W, d->tB, d->tC};
  return true;
}

// one slot of the host ring -> the device step state; the ring is read with system-scope loads
// (pinned host memory, never cached), the counter advanced by lane 0.  Rings of <= 64 slots of
// <= 16 values: lane l reads slot l's row beside the counter load (one round trip to host memory
// instead of two in sequence), the counter's slot is broadcast from its lane.
constexpr int ADAM_THREADS = 256;
constexpr long long ADAM_PER4_FROM = 16384;  // elements: 4 per thread from here (fewer workgroups, fences)
struct AdamArgs {
  float* p[THZ_MAX_ADAM_PARAMS];
  const float* g[THZ_MAX_ADAM_PARAMS];
  float* m[THZ_MAX_ADAM_PARAMS];
  float* v[THZ_MAX_ADAM_PARAMS];
  float* step[THZ_MAX_ADAM_PARAMS];
  long long n[THZ_MAX_ADAM_PARAMS];
  int blk0[THZ_MAX_ADAM_PARAMS + 1];  // first workgroup of each parameter
  int np;
  double lr, b1, b2;
  float omb1, b2f, omb2, eps, wd, decay;  // fp32 roundings of 1 - b1, b2, 1 - b2, eps, wd, 1 - lr wd
  int decoupled;
  unsigned* done;
};

// the element update (torch's single-tensor Adam expressions, fp32) on loaded values; returns p
struct AdamElem {
  float p, g, m, v;
};
__device__ __forceinline__ void adam_update(const AdamArgs& a, AdamElem& e, float nstep, float bc2s) {
  float p = e.p, g = e.g;
  if (a.decoupled) p = p * a.decay;
  else if (a.wd != 0.0f) g = g + a.wd * p;
  const float m0 = e.m;  // lerp(m0, g, w) as ATen evaluates it
  const float w = a.omb1;
  e.m = w < 0.5f ? m0 + w * (g - m0) : g - (g - m0) * (1.0f - w);
  e.v = e.v * a.b2f + (a.omb2 * g) * g;
  e.p = p + nstep * (e.m / (sqrtf(e.v) / bc2s + a.eps));
}

// A workgroup is PER x 256 elements of one parameter: one per thread for the QAT maps (a
// one-workgroup loop over a 2,500-element map ran 2-3x longer, its loads in sequence), four for
// larger sets (the DONN's 30,000: 30 workgroups instead of 118, each with its release fence).  Thread q < np reads parameter q's step
// count and forms its scalars (fp64 bias corrections); the last workgroup to finish advances the
// counts, after every workgroup has read them.  The elements' loads are issued first, so their
// latency overlaps the step-count read and the fp64 pow of the bias corrections (before: after
// the scalars' barrier, a third dependent memory round trip on the step's critical path).
template <int PER>
__global__ void __launch_bounds__(ADAM_THREADS) adam_step_kernel(AdamArgs a) {
  __shared__ float s_ns[THZ_MAX_ADAM_PARAMS], s_bs[THZ_MAX_ADAM_PARAMS];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  const int bid = blockIdx.x;
  int q = 0;
  while (q + 1 < a.np && bid >= a.blk0[q + 1]) ++q;
  const long long i0 = (long long)(bid - a.blk0[q]) * (PER * ADAM_THREADS) + tid;
  AdamElem e[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long long i = i0 + (long long)k * ADAM_THREADS;
    if (i < a.n[q]) e[k] = AdamElem{a.p[q][i], a.g[q][i], a.m[q][i], a.v[q][i]};
  }
  float t = 0.0f;
  if (tid < a.np) {
    t = a.step[tid][0] + 1.0f;
    const double bc1 = 1.0 - pow(a.b1, (double)t), bc2 = 1.0 - pow(a.b2, (double)t);
    s_ns[tid] = (float)(-(a.lr / bc1));
    s_bs[tid] = (float)sqrt(bc2);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const long long i = i0 + (long long)k * ADAM_THREADS;
    if (i < a.n[q]) {
      adam_update(a, e[k], s_ns[q], s_bs[q]);
      a.m[q][i] = e[k].m;
      a.v[q][i] = e[k].v;
      a.p[q][i] = e[k].p;
    }
  }
  // no release fence: nothing this workgroup wrote is read by the last one, and its step-count read
  // (thread q, above) has returned before the arrival is counted (the count's value is already used)
  if (tid == 0) s_last = atomicAdd(a.done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last && tid < a.np) {
    a.step[tid][0] = t;
    if (tid == 0) a.done[0] = 0u;
  }
}

constexpr int FETCH_ROW = 16;
__global__ void __launch_bounds__(64) step_fetch_kernel(const int* ring, int depth, int width, int* state,
                                                        int* counter) {
  const int i = threadIdx.x;
  if (depth <= 64 && width <= FETCH_ROW) {
    int v[FETCH_ROW];
#pragma unroll
    for (int e = 0; e < FETCH_ROW; ++e)
      v[e] = (i < depth && e < width) ? __hip_atomic_load(ring + (size_t)i * width + e, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_SYSTEM)
                                      : 0;
    const int k = counter[0];
    const int slot = k % depth;
#pragma unroll
    for (int e = 0; e < FETCH_ROW; ++e) {
      const int t = __shfl(v[e], slot);
      if (i == e && e < width) state[e] = t;
    }
    if (i == 0) counter[0] = k + 1;
    return;
  }
  const int k = counter[0];
  const int* row = ring + (size_t)(k % depth) * width;
  for (int e = i; e < width; e += 64) state[e] = __hip_atomic_load(row + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (i == 0) counter[0] = k + 1;
}

}  // namespace thz

using namespace thz;

extern "C" int thz_gaussian_beam(const thz_gauss_desc* d, void* out, thz_stream_t stream) {
  if (!d || !out || d->C < 1 || d->H < 1 || d->W < 1 || !d->wavelengths || !d->waist_x || !d->waist_y)
    return fail(THZ_E_ARG, "bad Gaussian-beam arguments");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  GaussArgs a{};
  a.C = d->C;
  a.H = d->H;
  a.W = d->W;
  // x = linspace(-dx H / 2, dx H / 2, H) (:92-97), all fp32 as the reference's tensors
  a.x_start = (-d->dx * (float)d->H) / 2.0f;
  a.x_end = (d->dx * (float)d->H) / 2.0f;
  a.y_start = (-d->dy * (float)d->W) / 2.0f;
  a.y_end = (d->dy * (float)d->W) / 2.0f;
  a.x0 = d->x0;
  a.y0 = d->y0;
  a.ca = std::cos(d->alpha);
  a.sa = std::sin(d->alpha);
  const float PI = 3.14159265358979323846f, TWO_PI = 6.28318530717958647692f;
  for (int c = 0; c < d->C; ++c) {
    const float lam = d->wavelengths[c], w0x = d->waist_x[c], w0y = d->waist_y[c];
    const float k = TWO_PI / lam;
    const float zrx = (PI * (w0x * w0x)) / lam, zry = (PI * (w0y * w0y)) / lam;  // Rayleigh (:126-127)
    const float gx = std::atan2(d->z_w0x, zrx), gy = std::atan2(d->z_w0y, zry);   // Gouy (:130-131)
    const float qx = d->z_w0x / zrx, qy = d->z_w0y / zry;
    const float wx = w0x * std::sqrt(1.0f + qx * qx), wy = w0y * std::sqrt(1.0f + qy * qy);
    float rx = 1e12f, ry = 1e12f;  // curvature (:138-145); 1e12 at the waist
    if (d->z_w0x != 0.0f) { const float t = zrx / d->z_w0x; rx = d->z_w0x * (1.0f + t * t); }
    if (d->z_w0y != 0.0f) { const float t = zry / d->z_w0y; ry = d->z_w0y * (1.0f + t * t); }
    a.k[c] = k;
    a.kz_x[c] = k * d->z_w0x;
    a.kz_y[c] = k * d->z_w0y;
    a.two_rx[c] = 2.0f * rx;
    a.two_ry[c] = 2.0f * ry;
    a.gouy_x[c] = gx;
    a.gouy_y[c] = gy;
    a.amp[c] = (w0x / wx) * (w0y / wy);
    a.wx2[c] = wx * wx;
    a.wy2[c] = wy * wy;
  }
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("gaussian_beam", s);
  const int n = d->H * d->W;
  hipLaunchKernelGGL(gaussian_beam_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (float2*)out, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_thin_lens(const thz_lens_desc* d, const void* in, void* out, thz_stream_t stream) {
  if (!d || !in || !out || d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || !d->wavelengths)
    return fail(THZ_E_ARG, "bad thin-lens arguments");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  LensArgs a{};
  a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W;
  a.gx0 = (float)(-((d->H - 1) / 2));
  a.gx1 = (float)((d->H - 1) / 2);
  a.gy0 = (float)(-((d->W - 1) / 2));
  a.gy1 = (float)((d->W - 1) / 2);
  a.dx = d->dx;
  a.dy = d->dy;
  // pi / (lambda f) in the reference's fp32 order: torch forms python_scalar / tensor as
  // reciprocal(tensor) * scalar (Components/Thin_Lens.py:70-77), so one rounding more than a division
  const float PI = 3.14159265358979323846f;
  for (int c = 0; c < d->C; ++c) a.coef[c] = (1.0f / (d->wavelengths[c] * d->focal_length)) * PI;
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("thin_lens", s);
  const int n = d->H * d->W;
  hipLaunchKernelGGL(thin_lens_kernel, ew_grid(n, a.C, a.B), dim3(EW_THREADS), 0, s, (const float2*)in, (float2*)out,
                     a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

// CZT_prop.RS_kernel (Props/CZT_Prop.py:44-57) and RSC_prop.create_kernel (Props/RSC_Prop.py:
// 157-160): exp(i k r) z / (2 pi r^2) (1/r - i k), r = sqrt(x^2 + y^2 + z^2), on n mesh points per
// wavelength.  The phase k r is formed as (k |z|) mod 2 pi + k rho^2 / (r + |z|) with k |z| in
// double (rs_kernel), as in the CZT passes.
struct RsExportArgs {
  int n, C;
  float z;
  float lam[THZ_MAX_WAVELENGTHS];
};
__global__ void __launch_bounds__(EW_THREADS) rs_kernel_export(const float* __restrict__ x, const float* __restrict__ y,
                                                               float2* __restrict__ out, RsExportArgs a) {
  const int c = blockIdx.y;
  const float lam = a.lam[c];
  const RsPhase ph = rs_phase(lam, a.z);
  const float k = 6.283185307179586f / lam;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x)
    out[(size_t)c * a.n + i] = rs_kernel(x[i], y[i], a.z, k, ph);
}

extern "C" int thz_rs_kernel(const float* x, const float* y, int n, float z, const float* wavelengths, int C,
                             void* out, thz_stream_t stream) {
  if (!x || !y || !out || !wavelengths || n < 0 || C < 1) return fail(THZ_E_ARG, "bad RS-kernel arguments");
  if (C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", C, THZ_MAX_WAVELENGTHS);
  if (n == 0) return THZ_OK;
  RsExportArgs a{};
  a.n = n;
  a.C = C;
  a.z = z;
  for (int c = 0; c < C; ++c) a.lam[c] = wavelengths[c];
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("rs_kernel_export", s);
  const int blocks = std::min((n + EW_THREADS - 1) / EW_THREADS, 4096);
  hipLaunchKernelGGL(rs_kernel_export, dim3(blocks, C), dim3(EW_THREADS), 0, s, x, y, (float2*)out, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_aperture(const thz_aperture_desc* d, const void* in, void* out, thz_stream_t stream) {
  if (!d || !in || !out || d->BC < 1 || d->H < 1 || d->W < 1) return fail(THZ_E_ARG, "bad aperture arguments");
  if (d->kind != THZ_APERTURE_RECT && d->kind != THZ_APERTURE_CIRC)
    return fail(THZ_E_ARG, "bad aperture kind %d", d->kind);
  const ApertureArgs a = aperture_args(d, d->H, d->W);
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("aperture", s);
  const int n = d->H * d->W;
  hipLaunchKernelGGL(aperture_kernel, ew_grid(n, 1, a.BC), dim3(EW_THREADS), 0, s, (const float2*)in, (float2*)out,
                     a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" size_t thz_intensity_mse_workspace_size(const thz_loss_desc* d) {
  if (!d || d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1) return 0;
  // slots per b: the loss kernel's chunks or the fused ASM row pass's C H rows, whichever is more
  const size_t n = (size_t)d->C * d->H * d->W, per = LOSS_THREADS * LOSS_PER_THREAD;
  return LossSink::bytes(d->B, (int)std::max((n + per - 1) / per, (size_t)d->C * d->H));
}

extern "C" int thz_intensity_mse_forward(const thz_loss_desc* d, const void* field, const float* target, float* loss,
                                         float* stats, thz_stream_t stream) {
  LossArgs a;
  if (!loss_args(d, &a) || !field || !target || !loss || !stats) return fail(THZ_E_ARG, "bad loss arguments");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("intensity_mse_fwd", s);
  const int n = d->C * d->H * d->W, per = LOSS_THREADS * LOSS_PER_THREAD, chunks = (n + per - 1) / per;
  const LossSink ls = loss_sink(d, target, loss, stats, chunks);
  hipLaunchKernelGGL(mse_forward_kernel, dim3(chunks, d->B), dim3(LOSS_THREADS), 0, s, (const float2*)field, a, ls);
  THZ_LAUNCH_CHECK();
  int e = launch_loss_finish(ls, s);
  if (e) return e;
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_intensity_mse_backward(const thz_loss_desc* d, const void* field, const float* target,
                                          const float* stats, const float* grad_loss, void* grad_field,
                                          thz_stream_t stream) {
  LossArgs a;
  if (!loss_args(d, &a) || !field || !target || !stats || !grad_loss || !grad_field)
    return fail(THZ_E_ARG, "bad loss arguments");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("intensity_mse_bwd", s);
  const size_t total = (size_t)d->B * d->C * d->H * d->W;
  const double n = (double)total;
  hipLaunchKernelGGL(mse_backward_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     (const float2*)field, target, stats, grad_loss, (float2*)grad_field, a, (float)(2.0 / n));
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_resample_forward(const thz_resample_desc* d, const void* in, void* out, thz_stream_t stream) {
  ResampleArgs a;
  if (!resample_args(d, &a) || !in || !out) return fail(THZ_E_ARG, "bad resample arguments");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("resample_fwd", s);
  const int n = d->Hout * d->Wout;
  hipLaunchKernelGGL(resample_fwd, dim3((n + 255) / 256), dim3(256), 0, s, (const float2*)in, (float2*)out, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_resample_backward(const thz_resample_desc* d, const void* grad_out, void* grad_in,
                                     thz_stream_t stream) {
  ResampleArgs a;
  if (!resample_args(d, &a) || !grad_out || !grad_in) return fail(THZ_E_ARG, "bad resample arguments");
  hipStream_t s = (hipStream_t)stream;
  THZ_HIP_CHECK(hipMemsetAsync(grad_in, 0, sizeof(float2) * (size_t)d->BC * d->Hin * d->Win, s));
  const int n = d->Hout * d->Wout;
  hipLaunchKernelGGL(resample_bwd, dim3((n + 255) / 256), dim3(256), 0, s, (const float2*)grad_out,
                     (float2*)grad_in, a);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}

extern "C" int thz_step_fetch(const int* ring, int depth, int width, int* state, int* counter, thz_stream_t stream) {
  if (!ring || !state || !counter || depth < 1 || width < 1 || width > 5 + THZ_MAX_Z)
    return fail(THZ_E_ARG, "bad step-fetch arguments");
  void* dring = nullptr;
  THZ_HIP_CHECK(hipHostGetDevicePointer(&dring, const_cast<int*>(ring), 0));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(step_fetch_kernel, dim3(1), dim3(64), 0, s, (const int*)dring, depth, width, state, counter);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}

extern "C" int thz_adam_step(const thz_adam_desc* d, const thz_adam_param* params, thz_stream_t stream) {
  if (!d || !params || !d->done || d->nparams < 1 || d->nparams > THZ_MAX_ADAM_PARAMS)
    return fail(THZ_E_ARG, "bad Adam arguments");
  AdamArgs a{};
  a.np = d->nparams;
  a.lr = d->lr; a.b1 = d->beta1; a.b2 = d->beta2;
  a.omb1 = (float)(1.0 - d->beta1); a.b2f = (float)d->beta2; a.omb2 = (float)(1.0 - d->beta2);
  a.eps = (float)d->eps; a.wd = (float)d->weight_decay; a.decay = (float)(1.0 - d->lr * d->weight_decay);
  a.decoupled = d->decoupled;
  a.done = d->done;
  long long total = 0;
  for (int q = 0; q < a.np; ++q) total += params[q].n;
  const int per = total >= ADAM_PER4_FROM ? 4 : 1, chunk = per * ADAM_THREADS;
  long long blocks = 0;
  for (int q = 0; q < a.np; ++q) {
    const thz_adam_param& p = params[q];
    if (!p.param || !p.grad || !p.exp_avg || !p.exp_avg_sq || !p.step || p.n < 1) return fail(THZ_E_ARG, "bad Adam parameter %d", q);
    a.p[q] = p.param; a.g[q] = p.grad; a.m[q] = p.exp_avg; a.v[q] = p.exp_avg_sq; a.step[q] = p.step; a.n[q] = p.n;
    a.blk0[q] = (int)blocks;
    blocks += (p.n + chunk - 1) / chunk;
    if (blocks > (1 << 30)) return fail(THZ_E_UNSUPPORTED, "Adam parameters too large");
  }
  a.blk0[a.np] = (int)blocks;
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("adam_step", s);
  if (per == 4) hipLaunchKernelGGL(adam_step_kernel<4>, dim3((unsigned)blocks), dim3(ADAM_THREADS), 0, s, a);
  else hipLaunchKernelGGL(adam_step_kernel<1>, dim3((unsigned)blocks), dim3(ADAM_THREADS), 0, s, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}
