#!/usr/bin/env python3
"""Generate tests/golden/cfg3_check.npz: the REFERENCE's own output on the cfg3 workload
(Props/CZT_Prop.py:252-314: a 2048^2 field, dx_in = 0.5 mm, 32 wavelengths c0 / linspace(220,
330 GHz, 32), z = 0.5 m, zoomed to 512^2 at dx_out = 0.25 mm), run in fp64 by the SURVEY.md §8(c)
procedure and in fp32 as shipped.

The input is a seeded white complex field (``cfg3_input``), not SURVEY §8(d)'s Gaussian beam: for a
centred Gaussian the reference's CZT returns almost nothing (|E| <= 2e-8 in fp64 from a unit-peak
beam at this geometry, and the same at the test_czt.py geometry), so its fp32 output is pure
rounding noise (5e3 relative to fp64) and no signature of it can grade anything.  A white field
has energy at every spatial frequency the zoom window samples.

Only a signature of each 512^2 output plane is kept (bench.py's cfg3 line and
tests/test_czt_gpu.py compare against it): the energy sum |E|^2, the sub-grid E[::8, ::8] and the
full row 256, per wavelength.  The reference processes the wavelength channels independently, so
it is called on 8 wavelengths at a time to bound host memory.

Runs only in the build container (imports /root/reference through ``_refimport``)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_cfg3_check.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from _refimport import import_reference  # noqa: E402

from bench import cfg3_input  # noqa: E402  (the input planes the bench times)


C0 = 2.998e8
N, DX, Z = 2048, 0.5e-3, 0.5
OUT, ODX = 512, 0.25e-3
NLAM = 32
SUB = 8
ROW = 256
GROUP = 8


def wavelengths32():
    """The fp32 wavelengths bench.py passes (float(fp32(c0 / f)))."""
    freqs = torch.linspace(220e9, 330e9, NLAM, dtype=torch.float64)
    return [float(torch.tensor(C0 / float(f), dtype=torch.float32)) for f in freqs]


def main():
    ref = import_reference()
    torch.set_num_threads(8)
    lam_all = wavelengths32()
    arrays = {"lam": np.array(lam_all, dtype=np.float32), "z": np.float64(Z), "dx": np.float32(DX),
              "odx": np.float32(ODX), "sub": np.int64(SUB), "row": np.int64(ROW)}
    sig = {tag: {"energy": [], "sub": [], "row": []} for tag in ("64", "32")}
    for g0 in range(0, NLAM, GROUP):
        lam = lam_all[g0:g0 + GROUP]
        x = torch.stack([cfg3_input(g0 + i) for i in range(len(lam))])[None]
        for f64 in (True, False):
            tag = "64" if f64 else "32"
            old = torch.get_default_dtype()
            torch.set_default_dtype(torch.float64 if f64 else torch.float32)
            try:
                data = x.to(torch.complex128) if f64 else x
                field = ref.ElectricField(data=data, wavelengths=lam, spacing=DX, device="cpu")
                if f64:
                    field._wavelengths = field._wavelengths.double()
                    field._spacing = field._spacing.double()
                prop = ref.CZT.CZT_prop(z_distance=Z, device="cpu")
                with contextlib.redirect_stdout(io.StringIO()):
                    out = prop.forward(field, outputHeight=OUT, outputWidth=OUT, outputPixel_dx=ODX,
                                       outputPixel_dy=ODX).data.detach()[0].to(torch.complex128).numpy()
            finally:
                torch.set_default_dtype(old)
            sig[tag]["energy"].append(np.sum(np.abs(out) ** 2, axis=(-2, -1)))
            sig[tag]["sub"].append(out[:, ::SUB, ::SUB].copy())
            sig[tag]["row"].append(out[:, ROW].copy())
            print(f"wavelengths {g0}..{g0 + len(lam) - 1} fp{tag}: energy {sig[tag]['energy'][-1][0]:.9e}",
                  flush=True)
            del out
    for tag in ("64", "32"):
        for k in ("energy", "sub", "row"):
            arrays[f"{k}{tag}"] = np.concatenate(sig[tag][k], 0)
    s64, s32 = arrays["sub64"], arrays["sub32"]
    arrays["rel32vs64"] = np.array([np.linalg.norm(s32[i] - s64[i]) / np.linalg.norm(s64[i]) for i in range(NLAM)])
    print("reference fp32 vs fp64 rel-L2 per wavelength (sub-grid): max", arrays["rel32vs64"].max())
    np.savez_compressed(os.path.join(HERE, "cfg3_check.npz"), **arrays)


if __name__ == "__main__":
    main()
