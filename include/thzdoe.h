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

/* Library identity. */
const char* thz_version(void);
const char* thz_last_error(void);

/*
 * Angular-spectrum propagation, Props/ASM_Prop.py:314-378 (forward) and its
 * adjoint (autograd backward, == ASM with conj(H)).
 *
 * Forward : in  [B, C, H, W]            -> out [Z, B, C, Ho, Wo]
 * Adjoint : in  [Z, B, C, Ho, Wo] (Z==1) -> out [B, C, H, W]
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
  int adjoint;              /* 0 forward, 1 adjoint (requires Z == 1) */
  int z_chunk;              /* z-planes per column pass; 0 = library default */
  float dx, dy;
  const float* wavelengths; /* host [C] */
  const float* z;           /* host [Z] */
} thz_asm_desc;

int thz_asm_workspace_size(const thz_asm_desc* d, size_t* bytes);
int thz_asm_forward(const thz_asm_desc* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                    thz_stream_t stream);
/* Plan facts for diagnostics / bench byte counts: number of spectral columns the kernels
 * keep (|m_y| <= J; ncols = 2J+1, or Pw when nothing is cut) and z-planes per column pass. */
int thz_asm_band(const thz_asm_desc* d, int* ncols, int* z_chunk);

/*
 * Chirp-z (Bluestein) Rayleigh-Sommerfeld propagation with output zoom,
 * Props/CZT_Prop.py:252-314 (forward).
 *   in  [B, C, H, W] complex64, spacing (dx, dy)
 *   out [B, C, outW, outH] (the reference's transposed result; outH must equal outW,
 *        as the reference's final F0 * U broadcast requires, :248)
 * wavelengths[C] host floats; z, output spacing (odx, ody) as in forward(field, outputHeight,
 * outputWidth, outputPixel_dx, outputPixel_dy).
 */
typedef struct thz_czt_desc {
  int B, C, H, W;
  int outH, outW;
  float dx, dy;
  float odx, ody;
  float z;
  const float* wavelengths; /* host [C] */
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
} thz_rsc_desc;

int thz_rsc_workspace_size(const thz_rsc_desc* d, size_t* bytes);
int thz_rsc_forward(const thz_rsc_desc* d, const void* in, void* out, void* workspace, size_t workspace_bytes,
                    thz_stream_t stream);

/*
 * Batched 1-D FFT along the contiguous axis (the building block of ft2/ift2,
 * utils/Helper_Functions.py:150, without shifts): in/out [rows, n], unnormalised,
 * inverse != 0 for the backward transform.  n <= 16384, any factorisation.
 */
int thz_fft_rows(const void* in, void* out, int rows, int n, int inverse, thz_stream_t stream);

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
