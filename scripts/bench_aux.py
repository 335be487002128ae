#!/usr/bin/env python3
"""Measurement of the SURVEY §8(f) kernels beside the propagators: the source / lens / aperture
((f)2), the resampler ((f)3), the DOE modulation (A10) and the QAT loss (A14, (f)1).  Each is
timed with HIP events on torch's current stream (the stream the kernels are enqueued on) over 50
launches at a size large enough to stream from HBM ([1, 32, 2048, 2048] complex64 = 1 GiB, or the
batch of the workload), and reported against the 8 TB/s HBM peak with its algorithmic bytes:
  gaussian_beam 8 N (write) | thin_lens, aperture 16 N (read + write) | resample 8 (N_in + N_out)
  modulate 16 N + 4 HW (field in, out; height) | intensity MSE forward 8 N + 4 N (field, target).
One JSON object per kernel on stdout (profiles/r02_aux_kernels.json keeps a run)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantizationawarethzdoe_amd import _lib, doe, optics  # noqa: E402

PEAK = 8.0e12
dev = torch.device("cuda:0")
C0 = 2.998e8


def timed(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def report(name, shape, nbytes, t):
    gbs = nbytes / t / 1e9
    print(json.dumps({"kernel": name, "shape": list(shape), "alg_bytes": int(nbytes), "us": round(t * 1e6, 2),
                      "GB_s": round(gbs, 1), "frac_hbm_peak": round(gbs * 1e9 / PEAK, 3)}), flush=True)


C, H, W = 32, 2048, 2048
N = C * H * W
wl = [C0 / f for f in torch.linspace(220e9, 330e9, C).tolist()]
x = optics.gaussian_beam(H, W, 0.5e-3, 0.5e-3, wl, [20e-3] * C, [20e-3] * C, device=dev)
report("gaussian_beam", x.shape, 8 * N,
       timed(lambda: optics.gaussian_beam(H, W, 0.5e-3, 0.5e-3, wl, [20e-3] * C, [20e-3] * C, device=dev)))
with torch.no_grad():
    report("thin_lens", x.shape, 16 * N, timed(lambda: optics.thin_lens(x, 0.5e-3, 0.5e-3, 0.127, wl)))
    report("aperture_rect", x.shape, 16 * N, timed(lambda: optics.aperture(x, _lib.APERTURE_RECT, 0.5e-3, 0.5e-3, 0.3, 0.3)))
    Ho = Wo = 1024
    report("resample", (1, C, Ho, Wo), 8 * (N + C * Ho * Wo),
           timed(lambda: optics.resample(x, Ho, Wo, 0.5e-3, 0.5e-3, 0.75e-3, 0.75e-3)))
    h = torch.rand(H, W, device=dev) * 1e-3
    u = torch.rand(H, W, device=dev)
    report("doe_modulate", x.shape, 16 * N + 8 * H * W,
           timed(lambda: doe.modulate(x, h, wl, 2.66, 0.03, tolerance=1e-5, noise=u)))
    # the QAT loss on a cfg5-sized batch (256 x 1 x 100 x 100) and a streaming-sized field
    for shp in ((256, 1, 100, 100), (32, 1, 2048, 2048)):
        f = torch.randn(shp, dtype=torch.complex64, device=dev)
        t = torch.rand((1,) + tuple(shp[1:]), device=dev)
        n = f.numel()
        report("intensity_mse_fwd", shp, 8 * n + 4 * n, timed(lambda: optics.intensity_mse(f, t)))
