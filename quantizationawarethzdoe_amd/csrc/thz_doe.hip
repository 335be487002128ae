// Quantization-aware DOE layers (Components/QuantizedDOE.py) for gfx950.
//
//  * modulate (DOELayer.modulate, :92-126): height noise (:82-87), nearest upsampling
//    (:102-107), transmission t_c(h) = exp(-k/2 (h+b) tand sqrt(eps)) exp(-i k (h+b)(sqrt(eps)-1))
//    (:47-79) and field * t, fused in one pass over the field; its backward in one more
//    (grad_field = g conj(t); grad_h = sum_bc Re(g conj(f) conj(t gamma)), scattered to the
//    source pixel of the nearest upsampling).
//  * height-map quantizers, one thread per parameter pixel, forward and backward fused
//    (every op of the reference chain in one kernel, the full mirrored map written directly):
//      FP    FullPrecisionDOELayer      :286-292   h = hmax sigmoid(clamp(w, +-8))
//      STE   STEQuantizedDOELayer       :1239-1388 nearest LUT level, identity gradient
//      PSQ   PSQuantizedDOELayer        :1193-1223 sum of L-1 tempered sigmoids
//      SGV3  SoftGumbelQuantizedDOELayerv3 :794-860 phase-score soft Gumbel (the paper's method)
//      NGS   NaiveGumbelQuantizedDOELayer  :1022-1041 Gumbel-softmax over [h, w, L] logits
//      SGV1  SoftGumbelQuantizedDOELayer   :411-456  phase-score soft Gumbel on a raw phase weight
//    (SoftGumbelQuantizedDOELayerv2, :608-635, is SGV3 with its own threshold: the host passes the
//    mode as iter_frac 0 or 1.)
//    The Gumbel noise is injected (Exp(1) draws, -log(E) = Gumbel), so a caller can replay the
//    reference's RNG stream exactly (tests) or draw it from any generator (training).
#include <algorithm>
#include <cmath>

#include "thz_common.hpp"
#include "thz_dev.hpp"

// every fp32 operation in this file rounds as the reference's separate torch ops do
#pragma clang fp contract(off)

namespace thz {


struct ModArgs {
  int B, C, H, W, hs, ws;
  int bl;  // batch lanes per block of the backward (power of two <= 16)
  int has_noise;
  float tol, eps, tand;
  const unsigned* rng;  // device generator state (when there is no noise array)
  unsigned rng_stream;
  float lam[THZ_MAX_WAVELENGTHS];
};

__device__ __forceinline__ int nearest_src(int dst, int in, int out) { return doe_nearest_src(dst, in, out); }
__device__ __forceinline__ float noisy_h(const float* h, const float* u, int idx, const ModArgs& a) {
  return doe_noisy_h(h, a.has_noise ? u : nullptr, idx, a.tol, a.rng, a.rng_stream);
}
__device__ __forceinline__ float2 transmission(float hv, float lam, const ModArgs& a, float2* gamma) {
  return doe_transmission(hv, lam, a.eps, a.tand, gamma);
}

// grid (pixel blocks, batch stride): t_c(h) once per pixel, thread and wavelength
// two pixels per lane (16-byte accesses for even HW), the noisy height of each evaluated once and
// the transmission once per (channel, pixel), the batch strided over blockIdx.z
__global__ void __launch_bounds__(EW_THREADS) doe_modulate_fwd(const float2* __restrict__ f, const float* __restrict__ h,
                                                              const float* __restrict__ u, float2* __restrict__ out,
                                                              float* __restrict__ hfull, ModArgs a) {
  const int HW = a.H * a.W;
  const int p0 = 2 * (blockIdx.x * EW_THREADS + (int)threadIdx.x);
  if (p0 >= HW) return;
  const bool two = p0 + 1 < HW, vec = (HW & 1) == 0;
  float hv[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = two || k == 0 ? p0 + k : p0;
    const int y = p / a.W, x = p - y * a.W;
    hv[k] = noisy_h(h, u, nearest_src(y, a.hs, a.H) * a.ws + nearest_src(x, a.ws, a.W), a);
  }
  if (hfull && blockIdx.z == 0) {
    hfull[p0] = hv[0];
    if (two) hfull[p0 + 1] = hv[1];
  }
  for (int c = 0; c < a.C; ++c) {
    const float2 t0 = transmission(hv[0], a.lam[c], a, nullptr), t1 = transmission(hv[1], a.lam[c], a, nullptr);
    for (int b = blockIdx.z; b < a.B; b += gridDim.z) {
      const size_t i = ((size_t)b * a.C + c) * HW + p0;
      if (vec) {
        const float4 v = *reinterpret_cast<const float4*>(f + i);
        const float2 r0 = cmul(make_float2(v.x, v.y), t0), r1 = cmul(make_float2(v.z, v.w), t1);
        *reinterpret_cast<float4*>(out + i) = make_float4(r0.x, r0.y, r1.x, r1.y);
      } else {
        out[i] = cmul(f[i], t0);
        if (two) out[i + 1] = cmul(f[i + 1], t1);
      }
    }
  }
}

// Block = MOD_THREADS threads = (MOD_THREADS / a.bl) pixels x a.bl batch lanes (a.bl a power of two
// <= 16 chosen from B): consecutive threads take consecutive pixels, batch lane l walks
// b = l, l + bl, ...; the height gradient's batch sum is finished across the lanes in LDS in a
// fixed order (deterministic, no atomics for same-size maps).
constexpr int MOD_THREADS = 256;

__global__ void __launch_bounds__(MOD_THREADS) doe_modulate_bwd(const float2* __restrict__ g,
                                                                const float2* __restrict__ f,
                                                                const float* __restrict__ h,
                                                                const float* __restrict__ u,
                                                                float2* __restrict__ gf, float* __restrict__ gh,
                                                                ModArgs a) {
  __shared__ float red[MOD_THREADS];
  const int HW = a.H * a.W;
  const int PX = MOD_THREADS / a.bl;
  const int px = threadIdx.x % PX, lane = threadIdx.x / PX;
  const int p = blockIdx.x * PX + px;
  const bool live = p < HW;
  float acc = 0.f;
  int src = 0;
  if (live) {
    const int y = p / a.W, x = p - y * a.W;
    src = nearest_src(y, a.hs, a.H) * a.ws + nearest_src(x, a.ws, a.W);
    const float hv = noisy_h(h, u, src, a);
    for (int c = 0; c < a.C; ++c) {
      float2 gam;
      const float2 t = transmission(hv, a.lam[c], a, &gam);
      float2 gt = make_float2(0.f, 0.f);  // sum_b g conj(f), this lane's share
      for (int b = lane; b < a.B; b += a.bl) {
        const size_t i = ((size_t)b * a.C + c) * HW + p;
        const float2 gv = g[i];
        if (gf) gf[i] = make_float2(gv.x * t.x + gv.y * t.y, gv.y * t.x - gv.x * t.y);
        if (gh) {
          const float2 fv = f[i];
          gt.x += gv.x * fv.x + gv.y * fv.y;
          gt.y += gv.y * fv.x - gv.x * fv.y;
        }
      }
      if (gh) {
        const float2 dt = cmul(t, gam);  // dt/dh
        acc += gt.x * dt.x + gt.y * dt.y;  // Re(gt conj(dt))
      }
    }
  }
  if (gh) {
    red[threadIdx.x] = acc;
    __syncthreads();
    if (live && lane == 0) {
      float s = red[px];
      for (int l = 1; l < a.bl; ++l) s += red[l * PX + px];
      if (a.hs == a.H && a.ws == a.W) gh[src] = s;
      else atomicAdd(gh + src, s);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// quantizers
// ---------------------------------------------------------------------------------------------
struct QArgs {
  int kind, hq, wq, mirror, L;
  float hmax, clampv, tau, iter_frac, c_s, s, beta, phase_scale;
  const float* dyn;  // device (tau, s, beta) overriding the three above (graph replay)
  const unsigned* rng;  // device generator state: the Exp(1) noise drawn here when expo == nullptr
  unsigned rng_stream;
  float lut[THZ_MAX_LUT];
  float plut_w[THZ_MAX_LUT];  // wrapped phase LUT (SGV3)
};

// Loops over the LUT levels run to the compile-time bound with a guard, so the per-level arrays
// (logits, Gumbel draws, y) stay in registers instead of dynamically indexed scratch memory.
#define THZ_FOR_LEVELS(l, n) _Pragma("unroll") for (int l = 0; l < THZ_MAX_LUT; ++l) if (l < (n))

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

#pragma clang fp contract(off)
// torch.remainder(a, b) for b > 0 (fmod with the sign of the divisor)
__device__ __forceinline__ float rem_pos(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && m < 0.0f) m += b;
  return m;
}
__device__ __forceinline__ float wrap_pi(float x) {
  const float PI = 3.1415927410125732f, TWO_PI = 6.2831854820251465f;
  return rem_pos(x + PI, TWO_PI) - PI;
}
// SGV3 scores (score_phase(func='sigmoid') * c_s * s, :794-817, :833) and d score / d phase
__device__ __forceinline__ void sgv3_score(const QArgs& a, float sv, float phase, int l, float* score, float* dscore) {
  const float PI = 3.1415927410125732f, TWO_PI = 6.2831854820251465f;
  const float wp = wrap_pi(phase);
  float d = wp - a.plut_w[l];
  d = rem_pos(d + PI, TWO_PI) - PI;
  d = d / PI;
  const float z = sv * d;
  const float sg = sigm(z);
  const float sc = sg * (1.0f - sg) * 4.0f;
  *score = (sc * a.c_s) * sv;
  // d/dphase: 4 sg (1-sg)(1-2sg) * s/pi * c_s * s
  *dscore = 4.0f * sg * (1.0f - sg) * (1.0f - 2.0f * sg) * (sv / PI) * a.c_s * sv;
}

// quadrant pixel (i, j) -> its up to four mirror positions in the full map (:28-35)
template <class F>
__device__ __forceinline__ void for_mirrors(const QArgs& a, int i, int j, F fn) {
  if (!a.mirror) {
    fn(i * a.wq + j);
    return;
  }
  const int W = 2 * a.wq;
  const int r0 = a.hq - 1 - i, r1 = a.hq + i;
  const int c0 = a.wq - 1 - j, c1 = a.wq + j;
  fn(r0 * W + c0);
  fn(r0 * W + c1);
  fn(r1 * W + c0);
  fn(r1 * W + c1);
}

// gumbel_softmax(logits, tau, hard) over L values: returns the hard index, y_soft in y
__device__ __forceinline__ int gumbel_soft(const float* logits, const float* expo, int L, float tau, float* y) {
  float mx = -INFINITY;
  THZ_FOR_LEVELS(l, L) {
    y[l] = (logits[l] + (-logf(expo[l]))) / tau;
    mx = fmaxf(mx, y[l]);
  }
  float sum = 0.f;
  THZ_FOR_LEVELS(l, L) {
    y[l] = expf(y[l] - mx);
    sum += y[l];
  }
  int arg = 0;
  float best = -1.f;
  THZ_FOR_LEVELS(l, L) {
    y[l] = y[l] / sum;
    if (y[l] > best) {
      best = y[l];
      arg = l;
    }
  }
  return arg;
}

// straight-through value sum_l lut_l * ((onehot_l - y_l) + y_l)
__device__ __forceinline__ float st_value(const QArgs& a, const float* y, int arg) {
  float q = 0.f;
  THZ_FOR_LEVELS(l, a.L) q += a.lut[l] * (((l == arg ? 1.0f : 0.0f) - y[l]) + y[l]);
  return q;
}

// the schedule values of this launch: the descriptor's, or the graph-replay device buffer's.
// The kernels keep QArgs unmodified (a written by-value struct is copied to scratch memory).
struct QDyn {
  float tau, s, beta;
};
__device__ __forceinline__ QDyn get_dyn(const QArgs& a) {
  return a.dyn ? QDyn{a.dyn[0], a.dyn[1], a.dyn[2]} : QDyn{a.tau, a.s, a.beta};
}

// quantized height of quadrant pixel p (the quantizer chain of QuantizedDOE.py for a.kind); the
// soft samples y go to ysave when it is non-null
__device__ __forceinline__ float quant_fwd_px(const QArgs& a, const QDyn& q, const float* __restrict__ w,
                                              const float* __restrict__ expo, int p, int n,
                                              float* __restrict__ ysave) {
  float out;
  float y[THZ_MAX_LUT];
  if (a.kind == THZ_Q_NGS) {
    float ex[THZ_MAX_LUT];
    THZ_FOR_LEVELS(l, a.L) ex[l] = expo ? expo[(size_t)p * a.L + l] : rng_exp1(a.rng, a.rng_stream, (unsigned)(p * a.L + l));
    const int arg = gumbel_soft(w + (size_t)p * a.L, ex, a.L, q.tau, y);
    out = st_value(a, y, arg);
    if (ysave) THZ_FOR_LEVELS(l, a.L) ysave[(size_t)p * a.L + l] = y[l];
  } else if (a.kind == THZ_Q_SGV1) {
    // the weight is the phase itself (:411-445): scores of w, Gumbel pick, LUT value
    float logits[THZ_MAX_LUT], ex[THZ_MAX_LUT];
    THZ_FOR_LEVELS(l, a.L) {
      float dsc;
      sgv3_score(a, q.s, w[p], l, &logits[l], &dsc);
      ex[l] = expo ? expo[(size_t)l * n + p] : rng_exp1(a.rng, a.rng_stream, (unsigned)(l * n + p));
    }
    const int arg = gumbel_soft(logits, ex, a.L, q.tau, y);
    out = st_value(a, y, arg);
    if (ysave) THZ_FOR_LEVELS(l, a.L) ysave[(size_t)l * n + p] = y[l];
  } else {
    const float wc = fminf(fmaxf(w[p], -a.clampv), a.clampv);
    const float hm = a.hmax * sigm(wc);
    out = hm;
    if (a.kind == THZ_Q_STE) {
      int arg = 0;
      float best = INFINITY;
      THZ_FOR_LEVELS(l, a.L) {
        const float dd = fabsf(hm - a.lut[l]);
        if (dd < best) {
          best = dd;
          arg = l;
        }
      }
      out = a.lut[arg];
    } else if (a.kind == THZ_Q_PSQ) {
      const float delta = (a.hmax - 0.0f) / (float)(a.L - 1);
      const float xn = (hm - 0.0f) / delta - 0.5f;
      float sm = 0.f;
      THZ_FOR_LEVELS(l, a.L - 1) sm += sigm(q.tau * (xn - (float)l));
      out = 0.0f + delta * sm;
    } else if (a.kind == THZ_Q_SGV3 && a.iter_frac > 0.3f) {
      const float phase = a.phase_scale * hm;
      float logits[THZ_MAX_LUT], ex[THZ_MAX_LUT];
      THZ_FOR_LEVELS(l, a.L) {
        float dsc;
        sgv3_score(a, q.s, phase, l, &logits[l], &dsc);
        ex[l] = expo ? expo[(size_t)l * n + p] : rng_exp1(a.rng, a.rng_stream, (unsigned)(l * n + p));
      }
      const int arg = gumbel_soft(logits, ex, a.L, q.tau, y);
      const float qv = st_value(a, y, arg);
      out = a.iter_frac <= 0.8f ? (1.0f - q.beta) * hm + q.beta * qv : qv;
      if (ysave) THZ_FOR_LEVELS(l, a.L) ysave[(size_t)l * n + p] = y[l];
    }
  }
  return out;
}

__global__ void quant_fwd(QArgs a, const float* __restrict__ w, const float* __restrict__ expo,
                          float* __restrict__ hfull, float* __restrict__ ysave) {
  const QDyn q = get_dyn(a);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = a.hq * a.wq;
  if (p >= n) return;
  const int i = p / a.wq, j = p - i * a.wq;
  const float out = quant_fwd_px(a, q, w, expo, p, n, ysave);
  for_mirrors(a, i, j, [&](int o) { hfull[o] = out; });
}

// The Gumbel kinds' forward with the L levels of a pixel on G adjacent lanes (G = the power of two
// >= L): lane l forms level l's logit and Exp(1) draw -- the long part of the chain (score wraps,
// draw, log) -- and the softmax runs on values gathered from the group in level order, so every
// operation and its order is quant_fwd_px's while each lane's chain is about 1 / L as long.  quant_fwd's one-pixel-per-thread form ran 7.2 us at cfg4 (2,500 pixels,
// 10 workgroups: a latency chain, not throughput).
template <int G>
__global__ void __launch_bounds__(256) quant_fwd_lv(QArgs a, const float* __restrict__ w,
                                                    const float* __restrict__ expo, float* __restrict__ hfull,
                                                    float* __restrict__ ysave) {
  const QDyn q = get_dyn(a);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int p = t / G, l = t % G;
  const int n = a.hq * a.wq;
  const int base = (int)(threadIdx.x & 63) - l;  // the group's first lane
  const bool live = p < n && l < a.L;
  const int pc = p < n ? p : n - 1, lc = l < a.L ? l : 0;  // in-range loads for the idle lanes
  float logit, ex, hm = 0.f;
  if (a.kind == THZ_Q_NGS) {
    logit = w[(size_t)pc * a.L + lc];
    ex = expo ? expo[(size_t)pc * a.L + lc] : rng_exp1(a.rng, a.rng_stream, (unsigned)(pc * a.L + lc));
  } else {
    float dsc, ph;
    if (a.kind == THZ_Q_SGV1) {
      ph = w[pc];
    } else {
      const float wc = fminf(fmaxf(w[pc], -a.clampv), a.clampv);
      hm = a.hmax * sigm(wc);
      ph = a.phase_scale * hm;
    }
    sgv3_score(a, q.s, ph, lc, &logit, &dsc);
    ex = expo ? expo[(size_t)lc * n + pc] : rng_exp1(a.rng, a.rng_stream, (unsigned)(lc * n + pc));
  }
  // gumbel_soft over the group, in level order
  const float yl = (logit + (-logf(ex))) / q.tau;
  float mx = -INFINITY;
  THZ_FOR_LEVELS(j, a.L) mx = fmaxf(mx, __shfl(yl, base + j));
  const float el = expf(yl - mx);
  float sum = 0.f;
  THZ_FOR_LEVELS(j, a.L) sum += __shfl(el, base + j);
  const float yv = el / sum;
  float y[THZ_MAX_LUT];
  int arg = 0;
  float best = -1.f;
  THZ_FOR_LEVELS(j, a.L) {
    y[j] = __shfl(yv, base + j);
    if (y[j] > best) {
      best = y[j];
      arg = j;
    }
  }
  const float qv = st_value(a, y, arg);
  float out = qv;
  if (a.kind == THZ_Q_SGV3) out = a.iter_frac <= 0.8f ? (1.0f - q.beta) * hm + q.beta * qv : qv;
  if (live && ysave) ysave[a.kind == THZ_Q_NGS ? (size_t)p * a.L + l : (size_t)l * n + p] = yv;
  if (l == 0 && p < n) {
    const int i = p / a.wq, jj = p - i * a.wq;
    for_mirrors(a, i, jj, [&](int o) { hfull[o] = out; });
  }
}

// dL/dw of quadrant pixel p from G = dL/dh summed over its mirror positions (the chain of
// quant_fwd's pixel, reversed); NGS writes its L logits' gradients
__device__ __forceinline__ void quant_bwd_px(const QArgs& a, const QDyn& q, const float* __restrict__ w,
                                             const float* __restrict__ ysave, int p, int n, float G,
                                             float* __restrict__ gw) {
  // The softmax backward in torch's form and rounding order (_softmax_backward_data:
  // y_l (dy_l - sum_k dy_k y_k), the straight-through's dy_l = G lut_l formed first).  At a
  // saturated softmax the difference keeps only the digits beyond the ulp of dy_l, as the
  // reference's own does; a centred form sum_k y_k (dy_l - dy_k), exact there, multiplies the
  // saturated level's rounding-noise score derivative by its now nonzero weight and moved a drawn
  // case 10 % from fp64 where the reference sits at 7.5e-6 (profiles/r06_experiments.txt 10).
  if (a.kind == THZ_Q_NGS) {
    // d logits_l = y_l (dy_l - sum_k y_k dy_k) / tau, dy_l = G lut_l
    float dot = 0.f;
    THZ_FOR_LEVELS(l, a.L) dot += (G * a.lut[l]) * ysave[(size_t)p * a.L + l];
    THZ_FOR_LEVELS(l, a.L) {
      const float yl = ysave[(size_t)p * a.L + l];
      gw[(size_t)p * a.L + l] = yl * (G * a.lut[l] - dot) / q.tau;
    }
    return;
  }
  if (a.kind == THZ_Q_SGV1) {
    float dot = 0.f;
    THZ_FOR_LEVELS(l, a.L) dot += (G * a.lut[l]) * ysave[(size_t)l * n + p];
    float dphase = 0.f;
    THZ_FOR_LEVELS(l, a.L) {
      const float yl = ysave[(size_t)l * n + p];
      float sc, dsc;
      sgv3_score(a, q.s, w[p], l, &sc, &dsc);
      dphase += yl * (G * a.lut[l] - dot) / q.tau * dsc;
    }
    gw[p] = dphase;
    return;
  }
  const float wv = w[p];
  const float wc = fminf(fmaxf(wv, -a.clampv), a.clampv);
  const float sg = sigm(wc);
  const float hm = a.hmax * sg;
  float dhm = G;  // FP and STE (identity straight-through)
  if (a.kind == THZ_Q_PSQ) {
    const float delta = (a.hmax - 0.0f) / (float)(a.L - 1);
    const float xn = (hm - 0.0f) / delta - 0.5f;
    float d = 0.f;
    THZ_FOR_LEVELS(l, a.L - 1) {
      const float s2 = sigm(q.tau * (xn - (float)l));
      d += s2 * (1.0f - s2) * q.tau;
    }
    dhm = G * d;  // delta * sum(tau sig') / delta
  } else if (a.kind == THZ_Q_SGV3 && a.iter_frac > 0.3f) {
    const bool blend = a.iter_frac <= 0.8f;
    const float gq = blend ? q.beta * G : G;
    float dot = 0.f;
    THZ_FOR_LEVELS(l, a.L) dot += (gq * a.lut[l]) * ysave[(size_t)l * n + p];
    const float phase = a.phase_scale * hm;
    float dphase = 0.f;
    THZ_FOR_LEVELS(l, a.L) {
      const float yl = ysave[(size_t)l * n + p];
      const float dlogit = yl * (gq * a.lut[l] - dot) / q.tau;
      float sc, dsc;
      sgv3_score(a, q.s, phase, l, &sc, &dsc);
      dphase += dlogit * dsc;
    }
    dhm = (blend ? (1.0f - q.beta) * G : 0.0f) + dphase * a.phase_scale;
  }
  const bool inside = wv >= -a.clampv && wv <= a.clampv;  // clamp passes the gradient on [min, max]
  gw[p] = inside ? dhm * a.hmax * sg * (1.0f - sg) : 0.0f;
}

__global__ void quant_bwd(QArgs a, const float* __restrict__ w, const float* __restrict__ ysave,
                          const float* __restrict__ gfull, float* __restrict__ gw) {
  const QDyn q = get_dyn(a);
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = a.hq * a.wq;
  if (p >= n) return;
  const int i = p / a.wq, j = p - i * a.wq;
  float G = 0.f;
  for_mirrors(a, i, j, [&](int o) { G += gfull[o]; });
  quant_bwd_px(a, q, w, ysave, p, n, G, gw);
}

// The DOE layer's whole backward in one pass, for a height map of the field's own size (no
// upsampling): modulate backward (grad_field = g conj(t) for every (b, c); dL/dh per full-map
// pixel, the batch summed over a.bl lanes in LDS exactly as doe_modulate_bwd does) and the
// quantizer's backward of the quadrant pixel those full-map pixels mirror (for_mirrors order), so
// grad_height never goes to memory.  Block = MOD_THREADS threads = PXQ quadrant pixels x nm mirror
// positions x a.bl batch lanes (thread = (lane * nm + k) * PXQ + px), so a mirrored map keeps
// one thread per (full-map pixel, lane) as the two-kernel form has; results bit-identical to
// doe_modulate_bwd followed by quant_bwd.
__global__ void __launch_bounds__(MOD_THREADS) doe_modulate_quant_bwd(const float2* __restrict__ g,
                                                                      const float2* __restrict__ f,
                                                                      const float* __restrict__ h,
                                                                      const float* __restrict__ u,
                                                                      float2* __restrict__ gf, ModArgs a, QArgs qa,
                                                                      const float* __restrict__ w,
                                                                      const float* __restrict__ ysave,
                                                                      float* __restrict__ gw) {
  __shared__ float red[MOD_THREADS];
  const int HW = a.H * a.W;
  const int n = qa.hq * qa.wq;
  const int nm = qa.mirror ? 4 : 1;
  const int PXQ = MOD_THREADS / (nm * a.bl);
  const int px = threadIdx.x % PXQ, k = (threadIdx.x / PXQ) % nm, lane = threadIdx.x / (PXQ * nm);
  const int p = blockIdx.x * PXQ + px;
  const bool live = p < n;
  float acc = 0.f;
  if (live) {
    const int i = p / qa.wq, j = p - i * qa.wq;
    int o = 0, kk = 0;
    for_mirrors(qa, i, j, [&](int oo) {
      if (kk++ == k) o = oo;
    });
    const float hv = noisy_h(h, u, o, a);
    for (int c = 0; c < a.C; ++c) {
      float2 gam;
      const float2 t = transmission(hv, a.lam[c], a, &gam);
      float2 gt = make_float2(0.f, 0.f);  // sum_b g conj(f), this lane's share
      for (int b = lane; b < a.B; b += a.bl) {
        const size_t e = ((size_t)b * a.C + c) * HW + o;
        const float2 gv = g[e];
        if (gf) gf[e] = make_float2(gv.x * t.x + gv.y * t.y, gv.y * t.x - gv.x * t.y);
        const float2 fv = f[e];
        gt.x += gv.x * fv.x + gv.y * fv.y;
        gt.y += gv.y * fv.x - gv.x * fv.y;
      }
      const float2 dt = cmul(t, gam);  // dt/dh
      acc += gt.x * dt.x + gt.y * dt.y;  // Re(gt conj(dt))
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (live && k == 0 && lane == 0) {
    float G = 0.f;  // quant_bwd's sum over the mirror positions of doe_modulate_bwd's lane sums
    for (int m = 0; m < nm; ++m) {
      float s = red[m * PXQ + px];
      for (int l = 1; l < a.bl; ++l) s += red[(l * nm + m) * PXQ + px];
      G += s;
    }
    quant_bwd_px(qa, get_dyn(qa), w, ysave, p, n, G, gw);
  }
}

static int qargs(const thz_quant_desc* d, QArgs* a) {
  if (!d) return fail(THZ_E_ARG, "null descriptor");
  if (d->kind < THZ_Q_FP || d->kind > THZ_Q_SGV1) return fail(THZ_E_ARG, "bad quantizer kind %d", d->kind);
  if (d->hq < 1 || d->wq < 1) return fail(THZ_E_ARG, "bad quantizer size");
  if (d->L < 1 || d->L > THZ_MAX_LUT) return fail(THZ_E_UNSUPPORTED, "LUT levels %d outside [1, %d]", d->L, THZ_MAX_LUT);
  if (!d->lut) return fail(THZ_E_ARG, "null LUT");
  if (d->kind == THZ_Q_PSQ && d->L < 2) return fail(THZ_E_ARG, "PSQ needs >= 2 levels");
  a->kind = d->kind;
  a->hq = d->hq;
  a->wq = d->wq;
  a->mirror = d->mirror;
  a->L = d->L;
  a->hmax = d->hmax;
  a->clampv = d->clamp;
  a->tau = d->tau;
  a->iter_frac = d->iter_frac;
  a->c_s = d->c_s;
  a->s = d->s;
  a->beta = d->beta;
  a->phase_scale = d->phase_scale;
  a->dyn = d->dyn;
  a->rng = d->rng;
  a->rng_stream = d->rng_stream;
  for (int l = 0; l < d->L; ++l) {
    a->lut[l] = d->lut[l];
    // (phase_lut + pi) % 2pi - pi of the reference's LUT phases (:802), host fp32
    const float PI = 3.1415927410125732f, TWO_PI = 6.2831854820251465f;
    const float ph = d->phase_scale * d->lut[l];
    float m = std::fmod(ph + PI, TWO_PI);
    if (m != 0.0f && m < 0.0f) m += TWO_PI;
    a->plut_w[l] = m - PI;
  }
  return THZ_OK;
}

}  // namespace thz

using namespace thz;

extern "C" int thz_doe_modulate_forward(const thz_doe_desc* d, const void* field, const float* height,
                                        const float* noise, void* out, float* height_full, thz_stream_t stream) {
  if (!d || !field || !height || !out) return fail(THZ_E_ARG, "null argument");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1 || d->hs < 1 || d->ws < 1) return fail(THZ_E_ARG, "bad shape");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  ModArgs a{};
  a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W; a.hs = d->hs; a.ws = d->ws;
  a.has_noise = noise != nullptr;
  a.tol = d->tolerance; a.eps = d->epsilon; a.tand = d->tand;
  a.rng = d->rng;
  a.rng_stream = d->rng_stream;
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("doe_modulate_fwd", s);
  const int n = d->H * d->W;
  hipLaunchKernelGGL(doe_modulate_fwd, ew_grid(n, 1, d->B), dim3(EW_THREADS), 0, s, (const float2*)field, height,
                     noise, (float2*)out, height_full, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_doe_modulate_backward(const thz_doe_desc* d, const void* grad_out, const void* field,
                                         const float* height, const float* noise, void* grad_field,
                                         float* grad_height, thz_stream_t stream) {
  if (!d || !grad_out || !field || !height) return fail(THZ_E_ARG, "null argument");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  ModArgs a{};
  a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W; a.hs = d->hs; a.ws = d->ws;
  a.has_noise = noise != nullptr;
  a.tol = d->tolerance; a.eps = d->epsilon; a.tand = d->tand;
  a.rng = d->rng;
  a.rng_stream = d->rng_stream;
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("doe_modulate_bwd", s);
  if (grad_height && (d->hs != d->H || d->ws != d->W))
    THZ_HIP_CHECK(hipMemsetAsync(grad_height, 0, sizeof(float) * d->hs * d->ws, s));
  const int n = d->H * d->W;
  a.bl = 1;
  while (a.bl < 16 && 2 * a.bl <= d->B) a.bl *= 2;
  const int px = MOD_THREADS / a.bl;
  hipLaunchKernelGGL(doe_modulate_bwd, dim3((n + px - 1) / px), dim3(MOD_THREADS), 0, s, (const float2*)grad_out,
                     (const float2*)field, height, noise, (float2*)grad_field, grad_height, a);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_quant_forward(const thz_quant_desc* d, const float* weight, const float* noise_exp,
                                 float* height_full, float* y_soft, thz_stream_t stream) {
  QArgs a;
  int e = qargs(d, &a);
  if (e) return e;
  const bool gumbel =
      d->kind == THZ_Q_NGS || d->kind == THZ_Q_SGV1 || (d->kind == THZ_Q_SGV3 && d->iter_frac > 0.3f);
  if (!weight || !height_full || (gumbel && ((!noise_exp && !d->rng) || !y_soft)))
    return fail(THZ_E_ARG, "null argument (Gumbel kinds need noise_exp or rng, and y_soft)");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("quant_fwd", s);
  const int n = d->hq * d->wq;
  if (gumbel && a.L > 1) {  // the levels on adjacent lanes
    if (a.L <= 4)
      hipLaunchKernelGGL(quant_fwd_lv<4>, dim3((4 * n + 255) / 256), dim3(256), 0, s, a, weight, noise_exp, height_full, y_soft);
    else if (a.L <= 8)
      hipLaunchKernelGGL(quant_fwd_lv<8>, dim3((8 * n + 255) / 256), dim3(256), 0, s, a, weight, noise_exp, height_full, y_soft);
    else
      hipLaunchKernelGGL(quant_fwd_lv<16>, dim3((16 * n + 255) / 256), dim3(256), 0, s, a, weight, noise_exp, height_full, y_soft);
  } else {
    hipLaunchKernelGGL(quant_fwd, dim3((n + 255) / 256), dim3(256), 0, s, a, weight, noise_exp, height_full, y_soft);
  }
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_doe_quant_backward(const thz_doe_desc* d, const thz_quant_desc* q, const void* grad_out,
                                      const void* field, const float* height, const float* noise, const float* weight,
                                      const float* y_soft, void* grad_field, float* grad_weight, thz_stream_t stream) {
  if (!d || !grad_out || !field || !height || !weight || !grad_weight) return fail(THZ_E_ARG, "null argument");
  if (d->B < 1 || d->C < 1 || d->H < 1 || d->W < 1) return fail(THZ_E_ARG, "bad shape");
  if (d->C > THZ_MAX_WAVELENGTHS) return fail(THZ_E_UNSUPPORTED, "C=%d > %d", d->C, THZ_MAX_WAVELENGTHS);
  QArgs qa;
  int e = qargs(q, &qa);
  if (e) return e;
  const int Hf = q->mirror ? 2 * q->hq : q->hq, Wf = q->mirror ? 2 * q->wq : q->wq;
  if (d->hs != d->H || d->ws != d->W || Hf != d->H || Wf != d->W)
    return fail(THZ_E_UNSUPPORTED, "fused DOE backward needs the quantized map at the field's size (%dx%d map, %dx%d "
                "height, %dx%d field)", Hf, Wf, d->hs, d->ws, d->H, d->W);
  const bool gumbel = q->kind == THZ_Q_NGS || q->kind == THZ_Q_SGV1 || (q->kind == THZ_Q_SGV3 && q->iter_frac > 0.3f);
  if (gumbel && !y_soft) return fail(THZ_E_ARG, "null y_soft (Gumbel kinds)");
  ModArgs a{};
  a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W; a.hs = d->hs; a.ws = d->ws;
  a.has_noise = noise != nullptr;
  a.tol = d->tolerance; a.eps = d->epsilon; a.tand = d->tand;
  a.rng = d->rng;
  a.rng_stream = d->rng_stream;
  for (int c = 0; c < d->C; ++c) a.lam[c] = d->wavelengths[c];
  a.bl = 1;
  while (a.bl < 16 && 2 * a.bl <= d->B) a.bl *= 2;  // doe_modulate_bwd's lanes: the same batch sums
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("doe_modulate_quant_bwd", s);
  const int n = q->hq * q->wq, px = MOD_THREADS / ((q->mirror ? 4 : 1) * a.bl);
  hipLaunchKernelGGL(doe_modulate_quant_bwd, dim3((n + px - 1) / px), dim3(MOD_THREADS), 0, s,
                     (const float2*)grad_out, (const float2*)field, height, noise, (float2*)grad_field, a, qa, weight,
                     y_soft, grad_weight);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_quant_backward(const thz_quant_desc* d, const float* weight, const float* y_soft,
                                  const float* grad_full, float* grad_weight, thz_stream_t stream) {
  QArgs a;
  int e = qargs(d, &a);
  if (e) return e;
  if (!weight || !grad_full || !grad_weight) return fail(THZ_E_ARG, "null argument");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("quant_bwd", s);
  const int n = d->hq * d->wq;
  hipLaunchKernelGGL(quant_bwd, dim3((n + 255) / 256), dim3(256), 0, s, a, weight, y_soft, grad_full, grad_weight);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

// ---------------------------------------------------------------------------------------------
// Rotationally symmetric layers (QuantizedDOE.py:1399-1623): radial profile [R] -> quadrant
// bins floor(sqrt(x^2 + y^2)) (< R-1, else 0) -> mirrored 2R x 2R map -> centre crop [H, W].
// ---------------------------------------------------------------------------------------------
namespace thz {
__device__ __forceinline__ int radial_bin(int i, int j, int R, int H, int W) {
  const int fi = R - H / 2 + i, fj = R - W / 2 + j;  // centre crop start (:1427-1429)
  const int qx = fi < R ? R - 1 - fi : fi - R;
  const int qy = fj < R ? R - 1 - fj : fj - R;
  const float d = sqrtf((float)(qx * qx + qy * qy));
  // bin 0 (r < 1) is filled for every R, bins k >= 1 for r < R - 1 (:1421-1423): at R = 1 the
  // single quadrant pixel still takes profile[0]
  return d < fmaxf(1.0f, (float)(R - 1)) ? (int)floorf(d) : -1;
}

__global__ void radial_fwd(const float* __restrict__ prof, float* __restrict__ out, int R, int H, int W) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= H * W) return;
  const int b = radial_bin(p / W, p % W, R, H, W);
  out[p] = b >= 0 ? prof[b] : 0.0f;
}

__global__ void radial_bwd(const float* __restrict__ g, float* __restrict__ gprof, int R, int H, int W) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= H * W) return;
  const int b = radial_bin(p / W, p % W, R, H, W);
  if (b >= 0) atomicAdd(gprof + b, g[p]);
}

// The rotationally symmetric layers' backward from the map gradient to the weight in one kernel:
// one workgroup per profile bin b gathers dL/dmap over the pixels of its annulus (radial_bin ==
// b; per map row the candidate columns come from the quadrant distance bounds, each candidate
// re-tested with radial_bin) in a fixed order -- no atomics, no zeroed buffer -- and applies the
// quantizer's backward to profile pixel b (quant_bwd_px).  Replaces radial_bwd's memset + atomic
// scatter and the quant_bwd launch.
constexpr int RQ_THREADS = 64;
__global__ void __launch_bounds__(RQ_THREADS) radial_quant_bwd(const float* __restrict__ g, QArgs qa, int R, int H,
                                                               int W, const float* __restrict__ w,
                                                               const float* __restrict__ ysave,
                                                               float* __restrict__ gw) {
  const int b = blockIdx.x;
  const int r0 = R - H / 2, c0 = R - W / 2;  // centre-crop offsets (radial_bin)
  float acc = 0.f;
  for (int i = threadIdx.x; i < H; i += RQ_THREADS) {
    const int fi = r0 + i;
    const int qx = fi < R ? R - 1 - fi : fi - R;
    if (qx > b + 1) continue;
    // quadrant columns qy with b <= sqrt(qx^2 + qy^2) < b + 1, one column of margin each side
    const int lo2 = b * b - qx * qx;
    const int qlo = lo2 > 0 ? max(0, (int)sqrtf((float)lo2) - 1) : 0;
    const int qhi = (int)sqrtf((float)((b + 1) * (b + 1) - qx * qx)) + 1;
    for (int qy = qlo; qy <= qhi; ++qy) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {  // fj = R - 1 - qy (left half), R + qy (right half)
        const int j = (side == 0 ? R - 1 - qy : R + qy) - c0;
        if (j >= 0 && j < W && radial_bin(i, j, R, H, W) == b) acc += g[(size_t)i * W + j];
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (threadIdx.x == 0) quant_bwd_px(qa, get_dyn(qa), w, ysave, b, R, acc, gw);
}
}  // namespace thz

extern "C" int thz_radial_forward(const float* profile, int R, int H, int W, float* out, thz_stream_t stream) {
  if (!profile || !out || R < 1 || H < 1 || W < 1 || H > 2 * R || W > 2 * R)
    return fail(THZ_E_ARG, "bad radial map arguments R=%d H=%d W=%d", R, H, W);
  hipLaunchKernelGGL(radial_fwd, dim3((H * W + 255) / 256), dim3(256), 0, (hipStream_t)stream, profile, out, R, H, W);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}

extern "C" int thz_radial_quant_backward(const thz_quant_desc* q, const float* grad_map, int R, int H, int W,
                                         const float* weight, const float* y_soft, float* grad_weight,
                                         thz_stream_t stream) {
  if (!grad_map || !weight || !grad_weight || R < 1 || H < 1 || W < 1 || H > 2 * R || W > 2 * R)
    return fail(THZ_E_ARG, "bad radial map arguments R=%d H=%d W=%d", R, H, W);
  QArgs qa;
  int e = qargs(q, &qa);
  if (e) return e;
  if (q->mirror || q->hq * q->wq != R) return fail(THZ_E_ARG, "the radial profile quantizer is %dx%d (mirror %d), "
                                                   "not the R = %d profile", q->hq, q->wq, q->mirror, R);
  const bool gumbel = q->kind == THZ_Q_NGS || q->kind == THZ_Q_SGV1 || (q->kind == THZ_Q_SGV3 && q->iter_frac > 0.3f);
  if (gumbel && !y_soft) return fail(THZ_E_ARG, "null y_soft (Gumbel kinds)");
  hipStream_t s = (hipStream_t)stream;
  KernelTimer kt("radial_quant_bwd", s);
  hipLaunchKernelGGL(radial_quant_bwd, dim3(R), dim3(RQ_THREADS), 0, s, grad_map, qa, R, H, W, weight, y_soft,
                     grad_weight);
  THZ_LAUNCH_CHECK();
  kt.stop();
  return THZ_OK;
}

extern "C" int thz_radial_backward(const float* grad_out, int R, int H, int W, float* grad_profile,
                                   thz_stream_t stream) {
  if (!grad_out || !grad_profile || R < 1 || H < 1 || W < 1 || H > 2 * R || W > 2 * R)
    return fail(THZ_E_ARG, "bad radial map arguments");
  hipStream_t s = (hipStream_t)stream;
  THZ_HIP_CHECK(hipMemsetAsync(grad_profile, 0, sizeof(float) * R, s));
  hipLaunchKernelGGL(radial_bwd, dim3((H * W + 255) / 256), dim3(256), 0, s, grad_out, grad_profile, R, H, W);
  THZ_LAUNCH_CHECK();
  return THZ_OK;
}
