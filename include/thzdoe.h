/*
 * thzdoe.h -- C-ABI of libthzdoe.so, the MI355X (gfx950) hot path of
 * QuantizationAwareTHzDOE: band-limited angular-spectrum (ASM), chirp-z (CZT) and
 * Rayleigh-Sommerfeld (RSC) complex-field propagators and the quantized-DOE phase
 * modulation.
 *
 * Conventions (all entry points):
 *   - extern "C", C types only; no exception crosses the boundary.
 *   - every entry returns int: THZ_OK (0) or a THZ_E_* code; thz_last_error()
 *     returns a thread-local message describing the last failure.
 *   - complex data is interleaved (re, im) float32, i.e. the memory of
 *     torch.complex64; all data/workspace pointers are DEVICE pointers owned by
 *     the caller (PyTorch's caching allocator).  The library allocates nothing per
 *     call; it keeps immutable per-device twiddle tables built lazily under a mutex
 *     (so the first call for a new length must not be inside a stream capture).
 *   - calls enqueue asynchronously on `stream` and never synchronise the device.
 *   - per-call physical scalars (wavelengths, z) are HOST arrays; they travel as
 *     kernel arguments, so calls are hipGraph-capturable after warm-up.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   thz_asm_*        Props/ASM_Prop.py:17-378    ASM_prop.forward (+ autograd adjoint)
 *   thz_czt_*        Props/CZT_Prop.py:11-314    CZT_prop.forward / VCZT_prop
 *   thz_rsc_*        Props/RSC_Prop.py:15-321    RSC_prop.forward / VRS_prop.forward
 *   thz_doe_*        Components/QuantizedDOE.py:44-126  DOELayer.modulate (+ backward)
 *   thz_quant_*      Components/QuantizedDOE.py:181-1388 quantized height maps (+ backward)
 *   thz_fft_*        utils/Helper_Functions.py:99-160 ft2/ift2 (centred ortho FFT)
 */
#ifndef THZDOE_H_
#define THZDOE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define THZ_OK 0
#define THZ_E_ARG 1         /* invalid argument / shape */
#define THZ_E_UNSUPPORTED 2 /* size outside what the kernels support */
#define THZ_E_WORKSPACE 3   /* workspace too small */
#define THZ_E_HIP 4         /* HIP runtime error (message in thz_last_error) */

#define THZ_BANDLIMIT_NONE 0
#define THZ_BANDLIMIT_EXACT 1  /* Matsushima eqs. 18-19, Props/ASM_Prop.py:296-301 */
#define THZ_BANDLIMIT_APPROX 2 /* Matsushima eqs. 21-22, Props/ASM_Prop.py:302-306 */

#define THZ_MAX_WAVELENGTHS 64
#define THZ_MAX_Z 256

typedef void* thz_stream_t; /* hipStream_t */

/* ABI of this header.  Bumped whenever a descriptor struct changes layout (round 2 appended
 * rng / rng_stream to thz_doe_desc and thz_quant_desc; 4 added thz_asm_transfer_function and
 * thz_rs_kernel, which the bindings require; 5 appended thz_asm_desc.window_mask, 6 thz_asm_desc.z_dev,
 * 7 added thz_doe_quant_backward and thz_radial_quant_backward, 8 thz_step_fetch and
 * thz_adam_step):
 * a caller compares thz_abi_version()
 * with the THZ_ABI_VERSION it was compiled against before its first call, since a shorter
 * struct from an older header would make the library read past it.  Descriptors are plain C
 * structs: zero-initialise them (memset / `= {0}` / ctypes defaults) so fields a caller does not
 * know about stay 0 (no noise buffer and no device generator means no noise). */
#define THZ_ABI_VERSION 8

/* Library identity. */
const char* thz_version(void);
const char* thz_last_error(void);
int thz_abi_version(void);

/*
 * Angular-spectrum propagation, Props/ASM_Prop.py:314-378 (forward) and its
 * adjoint (autograd backward, == ASM with conj(H)).
 *
 * Forward : in  [B, C, H, W]     -> out [Z, B, C, Ho, Wo]
 * Adjoint : in  [Z, B, C, Ho, Wo] -> out [B, C, H, W] = sum over z of plane z's adjoint (the
 *           autograd backward of a Z-plane forward; the column pass sums the planes' spectra,
 *           one inverse column transform and one row pass in all)
 * with Ho = H, Wo = W when unpad != 0 (CenterCrop, :359-361) else Ho = H+2 pad_h,
 * Wo = W + 2 pad_w (do_unpad_after_pad=False).  pad_h = floor(s_h H / 2) as in
 * compute_padding (:119-136); do_padding=False is pad_h = pad_w = 0.
 * wavelengths[C] and z[Z] are host float arrays (metres); dx, dy = field.spacing.
 */
typedef struct thz_asm_desc {
  int B, C, H, W;
  int pad_h, pad_w;
  int unpad;
  int bandlimit;            /* THZ_BANDLIMIT_* */
  int Z;                    /* 1 .. THZ_MAX_Z */
  int adjoint;              /* 0 forward, 1 adjoint (sums the Z planes) */
  int z_chunk;              /* z-planes per column pass; 0 = library default */
  float dx, dy;
  const float* wavelengths; /* host [C] */
  const float* z;           /* host [Z] */
  /* optional (NULL = none, ABI 5): an aperture on the output grid (ApertureElement after ASM_prop,
   * Components/Aperture.py:104-136, e.g. the DONN's layers, experiment_DONN_3_layers.ipynb:109-200),
   * applied in the row-inverse pass's stores (forward) or in the row pass's loads of the adjoint's
   * input (the adjoint of mask * ASM is ASM^H * mask).  Its BC is ignored; H, W must be the
   * output grid's (unpad ? H, W : the padded plane); the field is multiplied by 1 / 0, so NaN / inf
   * propagate as in the reference's field * mask.  Carried by the 300-point padded row length only
   * (the DONN / QAT layer geometry); other geometries return THZ_E_UNSUPPORTED (apply
   * thz_aperture separately), as does an adjoint with Z > 1. */
  const struct thz_aperture_desc* window_mask;
  /* optional (NULL = none, ABI 6): the Z plane distances in DEVICE memory [Z], read by the kernels
   * in place of z[] -- a captured HIP graph then replays with whatever the caller writes there
   * before each replay (the extended-depth-of-focus loop re-draws its five planes every iteration,
   * experiment_extend_depth_of_focus.ipynb cell 22).  The spectral band is then sized for any z
   * (the evanescent bound |Ky| <= k; the band limit still masks per element), and z[] (host) may be
   * NULL.  The caller keeps the values fixed between a forward and its adjoint. */
  const float* z_dev;
} thz_asm_desc;

/* Workspace: the row-pass spectrum T [BC][ncols][H], one z-chunk of column-pass output
 * U [zc][BC][ncols][Ho] (both complex64; the adjoint holds a z-chunk of input planes in T,
 * [zc][BC][ncols][Ho], and one summed plane in U), and for a 300-point padded height the
 * mixed-radix column pass's per-(wavelength, column) tables (sqrt row values and
 * kept-row bounds).  Contents need not persist between calls. */
int thz_asm_workspace_size(const thz_asm_desc* d, size_t* bytes);
int thz_asm_forward(const thz_asm_desc* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                    thz_stream_t stream);
/* Plan facts for diagnostics / bench byte counts: number of spectral columns the kernels
 * keep (|m_y| <= J; ncols = 2J+1, or Pw when nothing is cut) and z-planes per column pass. */
int thz_asm_band(const thz_asm_desc* d, int* ncols, int* z_chunk);
/* The transfer function the ASM kernels apply on the fly, materialised for inspection:
 * ASM_prop.create_kernel (Props/ASM_Prop.py:212-311; used by visualize_kernel, :198-210).
 * out [C, Ph, Pw] complex64 (device) on the CENTRED frequency grid of the padded plane
 * (row i <-> Kx = 2 pi ((i - Ph/2) / Ph) / dx, :141-145, 244-245), H = exp(i z sqrt(k^2 - K^2))
 * with the evanescent cut (:262) and the desc's band limit (:264-309), z = d->z[0].
 * Uses C, H, W, pad_h, pad_w, bandlimit, dx, dy, wavelengths, z of the descriptor. */
int thz_asm_transfer_function(const thz_asm_desc* d, void* out, thz_stream_t stream);

/*
 * Chirp-z (Bluestein) Rayleigh-Sommerfeld propagation with output zoom,
 * Props/CZT_Prop.py:252-314 (forward).
 *   in  [B, C, H, W] complex64, spacing (dx, dy)
 *   out [B, C, outW, outH] (the reference's transposed result; outH must equal outW,
 *        as the reference's final F0 * U broadcast requires, :248)
 * wavelengths[C] host floats; z, output spacing (odx, ody) as in forward(field, outputHeight,
 * outputWidth, outputPixel_dx, outputPixel_dy).
 * THZ_E_ARG when H + outW - 1 or W + outH - 1 is a power of two: the reference's Bluestein
 * slice keeps one row too few there and raises (Props/CZT_Prop.py:206,211).
 */
typedef struct thz_czt_desc {
  int B, C, H, W;
  int outH, outW;
  float dx, dy;
  float odx, ody;
  float z;
  const float* wavelengths; /* host [C] */
  int adjoint;              /* 1: the adjoint (autograd backward): in [B, C, outW, outH] ->
                               out [B, C, H, W]; conj chirps / filter / RS kernels, passes reversed */
} thz_czt_desc;

int thz_czt_workspace_size(const thz_czt_desc* d, size_t* bytes);
int thz_czt_forward(const thz_czt_desc* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                    thz_stream_t stream);

/*
 * Rayleigh-Sommerfeld convolution, Props/RSC_Prop.py:170-215 (RSC_prop.forward), and its
 * vectorial form VRS_prop.forward (:265-321, vectorial != 0: planes 0/1 of the input are
 * Ex/Ey, Ez = (Ex x + Ey y)/r is formed in the kernel, output has 3 planes).
 *   in  [B, C, H, W] -> out [Bo, C, Ph - H, Pw - W], Ph = H + 2 floor(H/2) (the reference's
 *   ifft2(...)[..., H:, W:] window, :207), Bo = vectorial ? 3 : B.
 * The spatial kernel grid uses dx on both axes (:83-84) and the spectrum is scaled by dx*dy.
 */
typedef struct thz_rsc_desc {
  int B, C, H, W;
  int vectorial;
  float dx, dy;
  float z;
  const float* wavelengths; /* host [C] */
  int adjoint;              /* 1: the adjoint (autograd backward) of the scalar convolution:
                               in [B, C, Ph - H, Pw - W] -> out [B, C, H, W], conj(FFT2(K)),
                               windows exchanged; vectorial must be 0 (VRS backward applies it
                               per plane and folds the Ez chain on the host side) */
} thz_rsc_desc;

int thz_rsc_workspace_size(const thz_rsc_desc* d, size_t* bytes);
int thz_rsc_forward(const thz_rsc_desc* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                    thz_stream_t stream);

/* The Rayleigh-Sommerfeld kernel exp(i k r) z / (2 pi r^2) (1/r - i k), r = sqrt(x^2 + y^2 + z^2),
 * k = 2 pi / lambda_c, on n mesh points: CZT_prop.RS_kernel (Props/CZT_Prop.py:44-57) and the
 * spatial kernel of RSC_prop.create_kernel (Props/RSC_Prop.py:144-167).  x[n], y[n] device
 * floats (the meshes), wavelengths[C] host floats; out [C][n] complex64 (device). */
int thz_rs_kernel(const float* x, const float* y, int n, float z, const float* wavelengths, int C, void* out,
                  thz_stream_t stream);

/*
 * DOE modulation, DOELayer.modulate (Components/QuantizedDOE.py:92-126):
 *   h' = height + (noise - 0.5) * 2 * tolerance   (noise = the rand_like draw, NULL = no noise, :82-87)
 *   h_full = nearest-upsample(h') to [H, W]        (:102-107)
 *   out[b,c] = field[b,c] * exp(-k_c/2 (h+b) tand sqrt(eps)) exp(-i k_c (h+b)(sqrt(eps)-1))  (:47-79)
 * field/out [B, C, H, W] complex64; height/noise [hs, ws] float32 (device).  height_full, if
 * non-NULL, receives h_full [H, W].  Backward: grad_field = g conj(t) (NULL to skip) and
 * grad_height [hs, ws] = sum_bc Re(g conj(field) conj(dt/dh)) (NULL to skip).
 */
typedef struct thz_doe_desc {
  int B, C, H, W;
  int hs, ws;                /* height-map size (upsampled to H, W if different) */
  float tolerance, epsilon, tand;
  const float* wavelengths;  /* host [C] */
  const unsigned* rng;       /* optional DEVICE [2] = (seed, step): with noise == NULL the kernels draw
                                the U[0,1) height noise per height pixel from a counter-based generator
                                (hash of seed, step, rng_stream, index; forward and backward agree) */
  unsigned rng_stream;
} thz_doe_desc;

int thz_doe_modulate_forward(const thz_doe_desc* d, const void* field, const float* height, const float* noise,
                             void* out, float* height_full, thz_stream_t stream);
int thz_doe_modulate_backward(const thz_doe_desc* d, const void* grad_out, const void* field, const float* height,
                              const float* noise, void* grad_field, float* grad_height, thz_stream_t stream);

/*
 * Fused DOE -> ASM step: the ASM forward of thz_doe_modulate_forward(field) in one
 * pipeline -- the row pass applies the noisy, upsampled transmission t_c(h) in its loader, so the
 * modulated field never goes to memory.  Replaces DOELayer.modulate (Components/QuantizedDOE.py:
 * 92-126) followed by ASM_prop.forward (Props/ASM_Prop.py:314-378).  d: the ASM descriptor (forward,
 * adjoint == 0); m: the DOE descriptor of the same [B, C, H, W] field.  height_full (optional)
 * receives the noisy upsampled height map [H, W].  The backward composes the ASM adjoint and
 * thz_doe_modulate_backward.
 */
int thz_asm_forward_modulated(const thz_asm_desc* d, const thz_doe_desc* m, const void* field, const float* height,
                              const float* noise, float* height_full, void* out, void* workspace,
                              size_t workspace_bytes, thz_stream_t stream);

/*
 * Height-map quantizers of the QAT layers (forward value + custom backward), one fused kernel
 * each way.  weight: [hq, wq] (FP/STE/PSQ/SGV3) or [hq, wq, L] logits (NGS).  height_full:
 * [2hq, 2wq] when mirror (num_unit set, _copy_quad_to_full :28-35) else [hq, wq].
 * noise_exp: the Exp(1) draw F.gumbel_softmax consumes ([L, hq, wq] for SGV1 and for SGV3
 * when iter_frac > 0.3, [hq, wq, L] for NGS); y_soft (same shape) is saved for the backward.
 * SoftGumbelQuantizedDOELayerv2 (:608-635) is SGV3 with iter_frac passed as 0 or 1.
 */
#define THZ_Q_FP 0    /* FullPrecisionDOELayer            :286-292   */
#define THZ_Q_STE 1   /* STEQuantizedDOELayer             :1239-1388 */
#define THZ_Q_PSQ 2   /* PSQuantizedDOELayer              :1193-1223 */
#define THZ_Q_SGV3 3  /* SoftGumbelQuantizedDOELayerv3    :794-860   */
#define THZ_Q_NGS 4   /* NaiveGumbelQuantizedDOELayer     :1022-1041 */
#define THZ_Q_SGV1 5  /* SoftGumbelQuantizedDOELayer      :411-456 (weight = phase) */
#define THZ_MAX_LUT 16

typedef struct thz_quant_desc {
  int kind;
  int hq, wq;
  int mirror;
  int L;
  const float* lut;   /* host [L] */
  float hmax;         /* height_constraint_max */
  float clamp;        /* weight clamp: 8 (FP/STE/PSQ), 10 (SGV3) */
  float tau;          /* temperature of the layer's schedule */
  float iter_frac;    /* SGV3 schedule phase */
  float c_s;          /* SGV3 score boost */
  float s;            /* SGV3 steepness tau_max / tau */
  float beta;         /* SGV3 blend (iter_frac - 0.3) / 0.5 */
  float phase_scale;  /* SGV3 2 pi / lambda_min * (sqrt(eps) - 1), fp32 */
  const float* dyn;   /* optional DEVICE [3] = (tau, s, beta) read by the kernels instead of the
                         fields above, so one captured HIP graph serves every schedule step */
  const unsigned* rng; /* optional DEVICE [2] = (seed, step): with noise_exp == NULL the Gumbel
                          kinds draw their Exp(1) noise in the kernel (see thz_doe_desc.rng) */
  unsigned rng_stream;
} thz_quant_desc;

int thz_quant_forward(const thz_quant_desc* d, const float* weight, const float* noise_exp, float* height_full,
                      float* y_soft, thz_stream_t stream);
int thz_quant_backward(const thz_quant_desc* d, const float* weight, const float* y_soft, const float* grad_full,
                       float* grad_weight, thz_stream_t stream);

/*
 * The whole backward of a quantized DOE layer whose height map has the field's size (no nearest
 * upsampling): thz_doe_modulate_backward followed by thz_quant_backward in ONE kernel, the height
 * gradient never written (DOELayer.modulate :92-126 and the quantizer's backward, e.g. v3
 * :794-860).  d: the modulation (hs == H, ws == W); q: the quantizer that produced `height`
 * (its full map, mirrored or not, must be [H, W]).  grad_field (NULL to skip) as
 * thz_doe_modulate_backward, grad_weight as thz_quant_backward; bit-identical to the two calls.
 * THZ_E_UNSUPPORTED for an upsampled map (use the two calls).
 */
int thz_doe_quant_backward(const thz_doe_desc* d, const thz_quant_desc* q, const void* grad_out, const void* field,
                           const float* height, const float* noise, const float* weight, const float* y_soft,
                           void* grad_field, float* grad_weight, thz_stream_t stream);

/*
 * Radial profile -> 2-D height map of the rotationally symmetric layers
 * (Components/QuantizedDOE.py:1409-1433): quadrant pixel (x, y) takes profile[floor(r)] for
 * r = sqrt(x^2 + y^2) < R - 1 (0 beyond), mirrored to 2R x 2R and centre-cropped to [H, W].
 */
int thz_radial_forward(const float* profile, int R, int H, int W, float* out, thz_stream_t stream);
int thz_radial_backward(const float* grad_out, int R, int H, int W, float* grad_profile, thz_stream_t stream);
/* The rotationally symmetric layer's backward from the map gradient to its weight in one kernel:
 * thz_radial_backward then thz_quant_backward of the profile quantizer q (hq * wq == R, mirror 0;
 * weight / y_soft as thz_quant_backward), the profile gradient gathered per bin in a fixed order
 * (deterministic; thz_radial_backward scatters with atomics). */
int thz_radial_quant_backward(const thz_quant_desc* q, const float* grad_map, int R, int H, int W, const float* weight,
                              const float* y_soft, float* grad_weight, thz_stream_t stream);

/*
 * Optical elements around the DOE, generated / applied on the device.
 *
 * Guassian_beam.forward (LightSource/Gaussian_beam.py:88-160): out [1, C, H, W] complex64.
 * waist_x / waist_y: host [C] fp32 beam waists (given, or BeamWaistCorruagtedTK :67-85).
 */
typedef struct thz_gauss_desc {
  int C, H, W;
  float dx, dy;                /* field spacing */
  const float* wavelengths;    /* host [C] */
  const float* waist_x;        /* host [C] */
  const float* waist_y;        /* host [C] */
  float x0, y0;                /* beam centre */
  float z_w0x, z_w0y;          /* waist positions */
  float alpha;                 /* amplitude rotation (rad) */
} thz_gauss_desc;
int thz_gaussian_beam(const thz_gauss_desc* d, void* out, thz_stream_t stream);

/* Thin_LensElement.forward (Components/Thin_Lens.py:31-85): out = in * exp(-i pi r^2 / (lambda f)). */
typedef struct thz_lens_desc {
  int B, C, H, W;
  float dx, dy, focal_length;
  const float* wavelengths;    /* host [C] */
} thz_lens_desc;
int thz_thin_lens(const thz_lens_desc* d, const void* in, void* out, thz_stream_t stream);

/* ApertureElement.forward (Components/Aperture.py:44-136): out = in * mask (in == out allowed). */
#define THZ_APERTURE_RECT 1
#define THZ_APERTURE_CIRC 2
typedef struct thz_aperture_desc {
  int BC, H, W, kind;
  float dx, dy;
  float half_w, half_h;        /* rect: open where |x| <= half_w and |y| <= half_h (fp32) */
  float radius;                /* circ: open where sqrt(x^2 + y^2) <= radius */
} thz_aperture_desc;
int thz_aperture(const thz_aperture_desc* d, const void* in, void* out, thz_stream_t stream);

/*
 * QAT loss (experiment_four_focal_spots.ipynb:336-370): mean((normalize(|E|^2) - target)^2) with
 * normalize dividing each batch item by its max (utils/Helper_Functions.py:185-193).
 * target [tB, tC, H, W] broadcast over B / C (tB in {1, B}, tC in {1, C}).
 * stats: device workspace of thz_intensity_mse_workspace_size bytes (max, argmax, max-path sum
 * per batch item, kept for the backward); loss: device [1]; grad_loss: device [1].
 */
typedef struct thz_loss_desc {
  int B, C, H, W;
  int tB, tC;
} thz_loss_desc;
size_t thz_intensity_mse_workspace_size(const thz_loss_desc* d);
int thz_intensity_mse_forward(const thz_loss_desc* d, const void* field, const float* target, float* loss,
                              float* stats, thz_stream_t stream);
int thz_intensity_mse_backward(const thz_loss_desc* d, const void* field, const float* target, const float* stats,
                               const float* grad_loss, void* grad_field, thz_stream_t stream);

/*
 * Fused ASM -> loss step: ASM forward of one z-plane (optionally of the DOE
 * modulation of field, as thz_asm_forward_modulated; m == NULL: plain ASM, height / noise /
 * height_full ignored) whose row-inverse pass also accumulates the QAT loss above over the rows
 * it stores, so the output field is not read back.  Replaces ASM_prop.forward (Props/
 * ASM_Prop.py:314-378) followed by the notebook's loss (experiment_four_focal_spots.ipynb:
 * 336-370, normalize = utils/Helper_Functions.py:185-193).  l describes the ASM output
 * [B, C, Ho, Wo]; out, loss and stats are what thz_asm_forward and thz_intensity_mse_forward
 * return (stats: thz_intensity_mse_workspace_size bytes, valid for thz_intensity_mse_backward).
 * Z > 1 planes (the multi-plane notebooks, e.g. plot_data/example_2 / example_3): l describes the
 * Z x B plane-major items [Z B, C, Ho, Wo] (each normalised by its own max; target tB in {1, Z B})
 * and the loss is the SUM over the planes of each plane's mean -- the notebooks' summed MSEs.
 */
/*
 * Its backward's first half in one pipeline: the ASM adjoint (d->adjoint == 1; Z >= 1 with l as above,
 * the Z-summing adjoint) of the loss
 * gradient dL/dE = 2 E dL/dI at the forward output `field` (thz_intensity_mse_backward's formula,
 * from the same target, stats and device grad_loss [1]), plus grad_out when non-NULL (the
 * cotangent of the output field itself).  The row pass forms the gradient as it loads each row.
 */
int thz_asm_adjoint_loss(const thz_asm_desc* d, const thz_loss_desc* l, const void* field, const float* target,
                         const float* stats, const float* grad_loss, const void* grad_out, void* grad_in,
                         void* workspace, size_t workspace_bytes, thz_stream_t stream);
int thz_asm_forward_loss(const thz_asm_desc* d, const thz_doe_desc* m, const void* field, const float* height,
                         const float* noise, float* height_full, const thz_loss_desc* l, const float* target,
                         void* out, float* loss, float* stats, void* workspace, size_t workspace_bytes,
                         thz_stream_t stream);

/*
 * Field_Resampler.forward (Addons/Field_Resampler.py:74-118): bilinear grid_sample (zeros
 * padding, align_corners=True) of [BC, Hin, Win] complex64 onto the centred output grid
 * linspace(-((n-1)//2), (n-1)//2, n) * d_out, normalised by d_in * ((n_in - 1) // 2).
 * The backward scatters grad_out with the same weights (grad_in is zeroed first).
 */
typedef struct thz_resample_desc {
  int BC, Hin, Win, Hout, Wout;
  float dx_in, dy_in, dx_out, dy_out;
} thz_resample_desc;
int thz_resample_forward(const thz_resample_desc* d, const void* in, void* out, thz_stream_t stream);
int thz_resample_backward(const thz_resample_desc* d, const void* grad_out, void* grad_in, thz_stream_t stream);

/*
 * Batched 1-D FFT along the contiguous axis (the building block of ft2/ift2,
 * utils/Helper_Functions.py:150, without shifts): in/out [rows, n], unnormalised,
 * inverse != 0 for the backward transform.  n <= 16384, any factorisation.
 */
int thz_fft_rows(const void* in, void* out, int rows, int n, int inverse, thz_stream_t stream);

/*
 * Double precision (complex128).  The reference computes in the field's precision: a complex128
 * field or float64 wavelength tensor runs ASM / CZT / RSC in fp64 and returns complex128
 * (DataType/ElectricField.py:85-90; test_czt.py:12 runs RSC + CZT that way).  These entries are
 * the fp32 ones with double scalars and complex128 buffers (interleaved double (re, im), identical
 * to torch.complex128); same shapes, windows and error codes.  Transform lengths (padded sizes,
 * Bluestein np2) up to 8192.  The fp64 ASM adjoint takes one z-plane (Z == 1).
 */
typedef struct thz_asm_desc64 {
  int B, C, H, W;
  int pad_h, pad_w;
  int unpad;
  int bandlimit;             /* THZ_BANDLIMIT_* */
  int Z;                     /* 1 .. THZ_MAX_Z; 1 for the adjoint */
  int adjoint;
  double dx, dy;
  const double* wavelengths; /* host [C] */
  const double* z;           /* host [Z] */
} thz_asm_desc64;
int thz_asm64_workspace_size(const thz_asm_desc64* d, size_t* bytes);
int thz_asm64_forward(const thz_asm_desc64* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                      thz_stream_t stream);

typedef struct thz_czt_desc64 {
  int B, C, H, W;
  int outH, outW;
  double dx, dy;
  double odx, ody;
  double z;
  const double* wavelengths; /* host [C] */
  int adjoint;
} thz_czt_desc64;
int thz_czt64_workspace_size(const thz_czt_desc64* d, size_t* bytes);
int thz_czt64_forward(const thz_czt_desc64* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                      thz_stream_t stream);

typedef struct thz_rsc_desc64 {
  int B, C, H, W;
  int vectorial;
  double dx, dy;
  double z;
  const double* wavelengths; /* host [C] */
  int adjoint;
} thz_rsc_desc64;
int thz_rsc64_workspace_size(const thz_rsc_desc64* d, size_t* bytes);
int thz_rsc64_forward(const thz_rsc_desc64* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                      thz_stream_t stream);

/* Batched 1-D FFT of complex128 rows (as thz_fft_rows), n <= 8192. */
int thz_fft64_rows(const void* in, void* out, int rows, int n, int inverse, thz_stream_t stream);

/*
 * Per-step state of the graph-replayed trainers (not part of the reference: qat.py StepState, the
 * schedule values tau / s / beta, the device generator's seed and step, the multi-plane systems'
 * plane distances, as int32 bit patterns).  ring: [depth][width] int32 in pinned host memory
 * (hipHostMalloc'd, device-mapped), one slot filled by the host per replay; counter: device int32 [1],
 * the fetches so far.  Copies slot (counter mod depth) into state (device [width] int32) and
 * increments counter -- a step's graph captures it as its first node, so every replay reads the
 * slot its host call filled without a host->device copy command between replays.  The caller
 * rewrites a slot only after the replay that read it has run.  1 <= width <= 5 + THZ_MAX_Z.
 */
int thz_step_fetch(const int* ring, int depth, int width, int* state, int* counter, thz_stream_t stream);

/*
 * One Adam / AdamW step over up to THZ_MAX_ADAM_PARAMS fp32 parameters in one launch (the trainers'
 * optimiser, quantizationawarethzdoe_amd/optim.py; the reference's notebooks step torch.optim.Adam /
 * AdamW, e.g. plot_data/example_1/experiment_four_focal_spots.ipynb cells 22, 33, 52).  Per element,
 * torch's single-tensor update with t = *step + 1 (each parameter's own device step count,
 * incremented by the launch); the scalars (1 - b1, 1 - b2, 1 - lr wd, the bias corrections) formed
 * in fp64 and rounded to fp32, as torch forms them in Python:
 *   decoupled (AdamW): p *= 1 - lr wd;   else g += wd p
 *   m = lerp(m, g, 1 - b1);   v = v b2 + (1 - b2) g g
 *   p += -(lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 * done: device u32 [1], zero before the first launch (the launch leaves it zero): the last
 * workgroup to finish advances the step counts, after every workgroup has read them.
 */
#define THZ_MAX_ADAM_PARAMS 16
typedef struct thz_adam_param {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;      /* device [1] */
  long long n;      /* elements */
} thz_adam_param;
typedef struct thz_adam_desc {
  double lr, beta1, beta2, eps, weight_decay;
  int decoupled;    /* 1: AdamW */
  int nparams;      /* 1 .. THZ_MAX_ADAM_PARAMS */
  unsigned* done;   /* device [1] */
} thz_adam_desc;
int thz_adam_step(const thz_adam_desc* d, const thz_adam_param* params, thz_stream_t stream);

/*
 * Per-kernel HIP-event timing used by bench.py (not part of the reference): when
 * enabled every kernel launch is bracketed by two events on its own stream;
 * thz_timing_read() synchronises on the pending events and returns the summed
 * duration and launch count for one kernel name ("asm_rows_fwd", "asm_cols", ...).
 */
int thz_timing_enable(int on);
int thz_timing_reset(void);
int thz_timing_read(const char* kernel, double* total_ms, long* launches);

#ifdef __cplusplus
}
#endif
#endif /* THZDOE_H_ */
