/*
 * Host-side checks of libthzdoe's C-ABI that need no GPU: descriptor validation of every entry
 * point (null pointers, bad shapes, broadcast rules, workspace too small), the error codes and
 * thread-local messages, and the workspace / band queries.  Built and run against the
 * AddressSanitizer build of the library (make -C quantizationawarethzdoe_amd/csrc asan), so
 * any host out-of-bounds access or leak on these paths aborts the run.  No kernel is launched.
 */
#include <stdio.h>
#include <string.h>

#include "../../include/thzdoe.h"

static int fails = 0;
#define EXPECT(cond, what)                                          \
  do {                                                              \
    if (!(cond)) {                                                  \
      fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, \
              __LINE__, what, thz_last_error());                    \
      ++fails;                                                      \
    }                                                               \
  } while (0)

int main(void) {
  EXPECT(thz_version() && strlen(thz_version()) > 0, "version string");
  EXPECT(thz_abi_version() == THZ_ABI_VERSION, "ABI version matches the header");
  float wl[2] = {1e-3f, 1.2e-3f}, zs[3] = {0.02f, 0.05f, 0.12f};

  /* ASM: workspace and band queries on valid descriptors, rejections on bad ones */
  thz_asm_desc a;
  memset(&a, 0, sizeof a);
  a.B = 1; a.C = 2; a.H = 100; a.W = 120; a.pad_h = 100; a.pad_w = 120; a.unpad = 1;
  a.bandlimit = THZ_BANDLIMIT_EXACT; a.Z = 3; a.dx = 1e-3f; a.dy = 1e-3f; a.wavelengths = wl; a.z = zs;
  size_t ws = 0;
  EXPECT(thz_asm_workspace_size(&a, &ws) == THZ_OK && ws > 0, "asm workspace size");
  int ncols = 0, zc = 0;
  EXPECT(thz_asm_band(&a, &ncols, &zc) == THZ_OK && ncols > 0 && ncols <= 360 && zc >= 1 && zc <= 3, "asm band");
  EXPECT(thz_asm_workspace_size(NULL, &ws) != THZ_OK, "asm null descriptor");
  EXPECT(thz_asm_workspace_size(&a, NULL) != THZ_OK, "asm null size pointer");
  thz_asm_desc b = a;
  b.H = 0;
  EXPECT(thz_asm_workspace_size(&b, &ws) != THZ_OK && strlen(thz_last_error()) > 0, "asm bad shape");
  b = a; b.Z = 0;
  EXPECT(thz_asm_workspace_size(&b, &ws) != THZ_OK, "asm Z = 0");
  b = a; b.Z = THZ_MAX_Z + 1;
  EXPECT(thz_asm_workspace_size(&b, &ws) != THZ_OK, "asm Z too large");
  b = a; b.adjoint = 1;  /* the adjoint sums the Z planes: the workspace holds a chunk of input planes */
  size_t ws_adj = 0;
  EXPECT(thz_asm_workspace_size(&b, &ws_adj) == THZ_OK && ws_adj > 0, "asm adjoint over Z planes");
  b = a; b.C = THZ_MAX_WAVELENGTHS + 1;
  EXPECT(thz_asm_workspace_size(&b, &ws) != THZ_OK, "asm too many wavelengths");
  EXPECT(thz_asm_forward(&a, NULL, NULL, NULL, 0, NULL) != THZ_OK, "asm forward null data");
  char dummy[64];
  EXPECT(thz_asm_forward(&a, dummy, dummy, dummy, 8, NULL) == THZ_E_WORKSPACE, "asm workspace too small");
  /* ABI 6: device-resident planes (z_dev) need no host z; the band is then sized for any z */
  b = a; b.z = NULL; b.z_dev = (const float*)dummy;
  int ncols_dev = 0, zc_dev = 0;
  EXPECT(thz_asm_band(&b, &ncols_dev, &zc_dev) == THZ_OK && ncols_dev >= ncols && zc_dev == zc, "asm z_dev band");
  b = a; b.z = NULL;
  EXPECT(thz_asm_workspace_size(&b, &ws) == THZ_E_ARG, "asm without host or device z");
  b = a; b.z = NULL; b.z_dev = (const float*)dummy;
  EXPECT(thz_asm_transfer_function(&b, dummy, NULL) == THZ_E_ARG, "transfer function needs a host z");
  /* inspection entries: rejections before any launch */
  EXPECT(thz_asm_transfer_function(NULL, dummy, NULL) != THZ_OK, "transfer function null descriptor");
  EXPECT(thz_asm_transfer_function(&a, NULL, NULL) == THZ_E_ARG, "transfer function null output");
  b = a; b.W = -1;
  EXPECT(thz_asm_transfer_function(&b, dummy, NULL) != THZ_OK, "transfer function bad shape");
  EXPECT(thz_rs_kernel(NULL, (const float*)dummy, 4, 0.1f, wl, 2, dummy, NULL) == THZ_E_ARG, "rs kernel null mesh");
  EXPECT(thz_rs_kernel((const float*)dummy, (const float*)dummy, 4, 0.1f, wl, 0, dummy, NULL) == THZ_E_ARG,
         "rs kernel no wavelength");
  EXPECT(thz_rs_kernel((const float*)dummy, (const float*)dummy, 4, 0.1f, wl, THZ_MAX_WAVELENGTHS + 1, dummy, NULL) ==
             THZ_E_UNSUPPORTED, "rs kernel too many wavelengths");
  EXPECT(thz_rs_kernel((const float*)dummy, (const float*)dummy, 0, 0.1f, wl, 2, dummy, NULL) == THZ_OK,
         "rs kernel on an empty mesh is a no-op");

  /* fused entries: shape agreement is checked before anything runs */
  thz_doe_desc m;
  memset(&m, 0, sizeof m);
  m.B = 1; m.C = 2; m.H = 100; m.W = 100; m.hs = 100; m.ws = 100;
  EXPECT(thz_asm_forward_modulated(&a, &m, dummy, (const float*)dummy, NULL, NULL, dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "modulated: DOE field shape must match the ASM input");
  thz_loss_desc l;
  memset(&l, 0, sizeof l);
  l.B = 1; l.C = 2; l.H = 100; l.W = 120; l.tB = 1; l.tC = 1;
  EXPECT(thz_asm_forward_loss(&a, NULL, dummy, NULL, NULL, NULL, &l, (const float*)dummy, dummy, (float*)dummy,
                              (float*)dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "loss: needs Z == 1");
  b = a; b.Z = 1;
  l.tC = 3;
  EXPECT(thz_asm_forward_loss(&b, NULL, dummy, NULL, NULL, NULL, &l, (const float*)dummy, dummy, (float*)dummy,
                              (float*)dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "loss: target must broadcast");
  l.tC = 1; l.W = 99;
  EXPECT(thz_asm_forward_loss(&b, NULL, dummy, NULL, NULL, NULL, &l, (const float*)dummy, dummy, (float*)dummy,
                              (float*)dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "loss: shape must match the ASM output");
  l.W = 120;
  EXPECT(thz_asm_adjoint_loss(&b, &l, dummy, (const float*)dummy, (const float*)dummy, (const float*)dummy, NULL,
                              dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "loss adjoint: needs adjoint == 1");
  b.adjoint = 1;
  EXPECT(thz_asm_adjoint_loss(&b, &l, NULL, (const float*)dummy, (const float*)dummy, (const float*)dummy, NULL,
                              dummy, dummy, 1 << 20, NULL) != THZ_OK,
         "loss adjoint: null field");
  b.adjoint = 0;
  EXPECT(thz_intensity_mse_workspace_size(&l) >= 3 * sizeof(float), "loss workspace size");
  EXPECT(thz_intensity_mse_workspace_size(NULL) == 0, "loss workspace null");
  EXPECT(thz_intensity_mse_forward(&l, NULL, NULL, NULL, NULL, NULL) != THZ_OK, "loss forward null pointers");

  /* CZT and RSC */
  thz_czt_desc c;
  memset(&c, 0, sizeof c);
  c.B = 1; c.C = 2; c.H = 256; c.W = 256; c.outH = 64; c.outW = 64; c.dx = 5e-4f; c.dy = 5e-4f;
  c.odx = 2.5e-4f; c.ody = 2.5e-4f; c.z = 0.5f; c.wavelengths = wl;
  EXPECT(thz_czt_workspace_size(&c, &ws) == THZ_OK && ws > 0, "czt workspace size");
  thz_czt_desc c2 = c;
  c2.outW = 32;
  EXPECT(thz_czt_workspace_size(&c2, &ws) != THZ_OK, "czt non-square output");
  c2 = c; c2.wavelengths = NULL;
  EXPECT(thz_czt_workspace_size(&c2, &ws) != THZ_OK, "czt null wavelengths");
  /* m + M - 1 a power of two (12 + 21 - 1 = 32): the reference's Bluestein slice raises there */
  c2 = c; c2.H = 12; c2.W = 12; c2.outH = 21; c2.outW = 21;
  EXPECT(thz_czt_workspace_size(&c2, &ws) == THZ_E_ARG && strstr(thz_last_error(), "power of two"),
         "czt power-of-two Bluestein length refused");
  c2.outH = 20; c2.outW = 20; /* 31: fine */
  EXPECT(thz_czt_workspace_size(&c2, &ws) == THZ_OK, "czt Bluestein length 31 accepted");
  c2.W = 13; /* the W pass: 13 + 20 - 1 = 32 */
  EXPECT(thz_czt_workspace_size(&c2, &ws) == THZ_E_ARG, "czt power-of-two length on the W pass refused");
  {
    double wl64[1] = {1e-3};
    thz_czt_desc64 c64;
    memset(&c64, 0, sizeof c64);
    c64.B = 1; c64.C = 1; c64.H = 12; c64.W = 12; c64.outH = 21; c64.outW = 21; c64.dx = 5e-4; c64.dy = 5e-4;
    c64.odx = 2.5e-4; c64.ody = 2.5e-4; c64.z = 0.5; c64.wavelengths = wl64;
    EXPECT(thz_czt64_workspace_size(&c64, &ws) == THZ_E_ARG, "fp64 czt power-of-two Bluestein length refused");
    c64.outH = 20; c64.outW = 20;
    EXPECT(thz_czt64_workspace_size(&c64, &ws) == THZ_OK, "fp64 czt Bluestein length 31 accepted");
  }
  thz_rsc_desc r;
  memset(&r, 0, sizeof r);
  r.B = 1; r.C = 1; r.H = 64; r.W = 64; r.dx = 1e-3f; r.dy = 1e-3f; r.z = 0.3f; r.wavelengths = wl;
  EXPECT(thz_rsc_workspace_size(&r, &ws) == THZ_OK && ws > 0, "rsc workspace size");
  thz_rsc_desc r2 = r;
  r2.H = 0;
  EXPECT(thz_rsc_workspace_size(&r2, &ws) != THZ_OK, "rsc bad shape");
  r2 = r; r2.vectorial = 1; r2.adjoint = 1;
  EXPECT(thz_rsc_workspace_size(&r2, &ws) != THZ_OK, "rsc vectorial adjoint");

  /* elementwise entries */
  EXPECT(thz_gaussian_beam(NULL, NULL, NULL) != THZ_OK, "gaussian null");
  EXPECT(thz_thin_lens(NULL, NULL, NULL, NULL) != THZ_OK, "lens null");
  EXPECT(thz_aperture(NULL, NULL, NULL, NULL) != THZ_OK, "aperture null");
  EXPECT(thz_doe_modulate_forward(NULL, NULL, NULL, NULL, NULL, NULL, NULL) != THZ_OK, "modulate null");
  EXPECT(thz_quant_forward(NULL, NULL, NULL, NULL, NULL, NULL) != THZ_OK, "quant null");
  EXPECT(thz_doe_quant_backward(NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL) != THZ_OK,
         "fused DOE backward null");
  {  /* an upsampled height map is refused before any launch */
    float wl = 1e-3f, lut[4] = {0.f, 0.25e-3f, 0.5e-3f, 0.75e-3f};
    thz_doe_desc dd;
    memset(&dd, 0, sizeof dd);
    dd.B = 1; dd.C = 1; dd.H = 100; dd.W = 100; dd.hs = 50; dd.ws = 50; dd.epsilon = 2.66f;
    dd.wavelengths = &wl;
    thz_quant_desc qd;
    memset(&qd, 0, sizeof qd);
    qd.kind = THZ_Q_FP; qd.hq = 50; qd.wq = 50; qd.L = 4; qd.lut = lut; qd.hmax = 1e-3f;
    EXPECT(thz_doe_quant_backward(&dd, &qd, dummy, dummy, (const float*)dummy, NULL, (const float*)dummy, NULL, NULL,
                                  (float*)dummy, NULL) == THZ_E_UNSUPPORTED,
           "fused DOE backward refuses an upsampled map");
  }
  EXPECT(thz_resample_forward(NULL, NULL, NULL, NULL) != THZ_OK, "resample null");
  EXPECT(thz_radial_forward(NULL, 0, 0, 0, NULL, NULL) != THZ_OK, "radial bad");
  EXPECT(thz_radial_quant_backward(NULL, NULL, 0, 0, 0, NULL, NULL, NULL, NULL) != THZ_OK, "radial quant bad");
  EXPECT(thz_fft_rows(NULL, NULL, 0, 1024, 0, NULL) != THZ_OK, "fft rows bad");
  int ring[4] = {0}, cnt = 0;
  EXPECT(thz_step_fetch(NULL, 1, 1, NULL, NULL, NULL) != THZ_OK, "step fetch null");
  EXPECT(thz_step_fetch(ring, 1, 6 + THZ_MAX_Z, ring, &cnt, NULL) != THZ_OK, "step fetch width > 5 + THZ_MAX_Z");
  thz_adam_desc ad;
  memset(&ad, 0, sizeof ad);
  EXPECT(thz_adam_step(NULL, NULL, NULL) != THZ_OK, "adam null");
  EXPECT(thz_adam_step(&ad, NULL, NULL) != THZ_OK, "adam no params");
  double ms = -1.0;
  long n = -1;
  EXPECT(thz_timing_reset() == THZ_OK && thz_timing_read("asm_cols", &ms, &n) == THZ_OK && n == 0,
         "timing registry empty after reset");

  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("abi host checks passed\n");
  return 0;
}
