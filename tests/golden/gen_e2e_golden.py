#!/usr/bin/env python3
"""Generate tests/golden/e2e_golden.npz: designed 4-level height maps pushed through the REFERENCE's
whole four-focal-spots system (experiment_four_focal_spots.ipynb:198-260: Guassian_beam with the
fitted horn waist -> ASM 127 mm -> thin lens f = 127 mm -> 80 mm aperture -> FixDOEElement
(tolerance 0) -> ASM 200 mm), then the QAT loss MSE(normalize(|E|^2), target) against the nine-PSF
target of define_FoM (nb :89-181) and its gradient with respect to the height map; fp64 by the
SURVEY.md §8(c) procedure and fp32 as shipped.  This is the deterministic end-to-end golden of
SURVEY §4 / §8(c): FixDOEElement(tolerance=0) -> ASM has no RNG in its output.

Cases:

* the REFERENCE's own trained maps (edoe_4levels.npy and plot_data/example_1/splitter_{ours, STE,
  PSQ, GS, full_precision}.npy): the 80 x 80 centre crops that the notebook's
  ``best_setup.doe.save(crop_size=[80, 80])`` wrote (experiment_four_focal_spots.ipynb cells 13, 29,
  39, 48, 56; Components/QuantizedDOE.py:253-267).  The files are numpy OBJECT arrays (a pickled
  dict); they are read by ``refdoe_parse.parse_pickled_npy``, a token parser that executes nothing
  from the file (no pickle loader runs on them).  ``ref_<name>_pad100``: the crop zero-padded back
  to the 100 x 100 DOE -- the system's 80 mm aperture (80 x 80 pixels) zeroes the field outside
  the crop before the DOE, so this reproduces the trained DOE's detector field exactly;
  ``ref_ours_80``: the 80 x 80 crop as a user would load it, upsampled by the FixDOE's nearest
  interpolation (QuantizedDOE.py:102-107).
* two maps designed here the way a 4-level splitter is: the phase of the superposition of the
  tilted plane waves that focus on the target's spots at f = 200 mm, quantised to 4 levels of
  lambda / (4 (n - 1)) height: ``splitter4_80`` (80 x 80, 4 spots at (+-20, +-20) mm, upsampled
  to the 100 x 100 field) and ``splitter9_100`` (100 x 100, the target's 9 spots).

Runs only in the build container (imports /root/reference through ``_refimport``)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_e2e_golden.py
"""
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refimport import import_reference  # noqa: E402

C0 = 2.998e8
MM = 1e-3
F0 = 300e9
EPS, TAND = 2.66, 0.03
FOCI9 = [(-20, -20), (20, 20), (-20, 20), (20, -20), (0, 0), (0, -20), (-20, 0), (0, 20), (20, 0)]
FOCI4 = [(-20, -20), (20, 20), (-20, 20), (20, -20)]


def designed_map(n, foci_mm, lam, f=200 * MM, dxy=1 * MM):
    """4-level height map [n, n] (float32, metres): phase of sum_k exp(i (2 pi / lam (x sin_x + y sin_y)
    + theta_k)) over the spots (theta_k = pi k^2 / K: spread spot phases, as splitter designs use to
    keep the sum from being real -- with equal phases the symmetric 4-spot sum has only 2 levels),
    level = floor(phase / (pi / 2)), height = level * lam / (4 (n - 1))."""
    x = (np.arange(n) - (n - 1) / 2) * dxy
    X, Y = np.meshgrid(x, x, indexing="ij")
    acc = np.zeros((n, n), np.complex128)
    for k, (a, b) in enumerate(foci_mm):
        r = np.sqrt((a * MM) ** 2 + (b * MM) ** 2 + f ** 2)
        acc += np.exp(1j * (2 * np.pi / lam * (X * a * MM + Y * b * MM) / r + np.pi * k * k / len(foci_mm)))
    phase = np.mod(np.angle(acc), 2 * np.pi)
    level = np.minimum(np.floor(phase / (np.pi / 2)), 3)
    return (level * lam / (4 * (np.sqrt(EPS) - 1))).astype(np.float32)


def fom(ref, resolution, dxy, lam, focal, pos, dt):
    """define_FoM of the notebook (nb :89-181) on the CPU, in dtype dt."""
    h, w = resolution
    Lx, Ly = dxy * w, dxy * h
    effL = torch.sqrt(torch.tensor(Lx ** 2 + Ly ** 2, dtype=dt))
    NA = torch.sin(torch.atan(effL / (2 * focal)))
    fwhm = lam / (2 * NA)
    xg, yg = torch.meshgrid(torch.linspace(-Lx / 2, Lx / 2, steps=w, dtype=dt),
                            torch.linspace(-Ly / 2, Ly / 2, steps=h, dtype=dt), indexing="ij")
    xp, yp = torch.tensor(pos, dtype=dt)
    psf = torch.exp(-((xg - xp) ** 2 + (yg - yp) ** 2) / ((fwhm * 2) ** 2))
    return ref.HF.normalize(psf.unsqueeze(0).unsqueeze(0))


def run(ref, hmap, f64, force_max=None):
    """The system's field, loss and height gradient; ``force_max`` = (i, j) divides by the intensity
    of that pixel instead of normalize()'s max (the same value when the pixel is a maximum, and
    the gradient torch's max routes to that index)."""
    GB = ref.import_module("LightSource.Gaussian_beam")
    TL = ref.import_module("Components.Thin_Lens")
    AP = ref.import_module("Components.Aperture")
    dt = torch.float64 if f64 else torch.float32
    old = torch.get_default_dtype()
    torch.set_default_dtype(dt)
    try:
        lam = C0 / F0
        with contextlib.redirect_stdout(io.StringIO()):
            src = GB.Guassian_beam(height=100, width=100, beam_waist_x=None, beam_waist_y=None, wavelengths=lam,
                                   spacing=1 * MM, device="cpu")
            f0 = src()
            if f64:
                f0._data = f0._data.to(torch.complex128)
                f0._wavelengths = f0._wavelengths.double()
                f0._spacing = f0._spacing.double()
            asm1 = ref.ASM.ASM_prop(z_distance=0.127, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True,
                                    device="cpu")
            lens = TL.Thin_LensElement(focal_length=0.127)
            ap = AP.ApertureElement(aperture_type='rect', aperture_size=0.08)
            field_in = ap(lens(asm1(f0)))
            doe = ref.DOE.FixDOEElement(height_map=torch.from_numpy(hmap).to(dt), tolerance=0.0,
                                        material=[EPS, TAND], device="cpu")
            asm3 = ref.ASM.ASM_prop(z_distance=200 * MM, bandlimit_type='exact', padding_scale=2,
                                    bandlimit_kernel=True, device="cpu")
            out = asm3(doe(field_in))
        target = sum(fom(ref, [100, 100], 1 * MM, lam, 200 * MM, [a * MM, b * MM], dt) for a, b in FOCI9)
        inten = torch.abs(out.data) ** 2
        if force_max is None:
            amp = ref.HF.normalize(inten)
        else:
            amp = inten / inten[0, 0, force_max[0], force_max[1]]
        loss = torch.nn.MSELoss()(amp, target)
        loss.backward()
        return dict(field_in=field_in.data.detach().numpy(), out=out.data.detach().numpy(), loss=float(loss.detach()),
                    grad=doe.height_map.grad.detach().numpy().copy(), target=target.detach().numpy())
    finally:
        torch.set_default_dtype(old)


def main():
    ref = import_reference()
    torch.set_num_threads(8)
    lam32 = float(np.float32(C0 / F0))
    cases = {"splitter4_80": designed_map(80, FOCI4, lam32), "splitter9_100": designed_map(100, FOCI9, lam32)}
    sources = {}
    from refdoe_parse import parse_pickled_npy
    refmaps = [("edoe_4levels", "edoe_4levels.npy")] + [
        (n, f"plot_data/example_1/splitter_{n}.npy") for n in ("ours", "STE", "PSQ", "GS", "full_precision")]
    for name, rel in refmaps:
        d = parse_pickled_npy(os.path.join(ref.root, rel))
        t = np.asarray(d["thickness"], dtype=np.float32)
        assert t.shape == (80, 80) and abs(float(d["dxy"]) - 1e-3) < 1e-12
        cases[f"ref_{name}_pad100"] = np.pad(t, 10)
        sources[f"ref_{name}_pad100"] = rel
        if name == "ours":
            cases["ref_ours_80"] = t
            sources["ref_ours_80"] = rel
    arrays, meta = {}, []
    for name, h in cases.items():
        arrays[f"{name}__h"] = h
        for f64 in (True, False):
            tag = "64" if f64 else "32"
            r = run(ref, h, f64)
            arrays[f"{name}__out{tag}"] = r["out"]
            arrays[f"{name}__loss{tag}"] = np.float64(r["loss"])
            arrays[f"{name}__grad{tag}"] = r["grad"]
            if name == "splitter4_80":
                arrays[f"field_in{tag}"] = r["field_in"]
                arrays[f"target{tag}"] = r["target"]
            print(f"{name} fp{tag}: loss {r['loss']:.9e}", flush=True)
        # tied maxima (the trained maps are mirror-symmetric): normalize()'s max is a tie-break of
        # rounding, and its gradient term moves with it -- store the fp64 gradient for every pixel
        # within 1e-9 of the maximum, so the GPU test can grade the one its own max picked
        I64 = np.abs(arrays[f"{name}__out64"][0, 0]) ** 2
        tied = np.argwhere(I64 >= I64.max() * (1 - 1e-9))
        ties = []
        if len(tied) > 1:
            for i, j in tied:
                arrays[f"{name}__gradtie_{i}_{j}"] = run(ref, h, True, force_max=(int(i), int(j)))["grad"]
                ties.append([int(i), int(j)])
        o32, o64 = arrays[f"{name}__out32"], arrays[f"{name}__out64"]
        rel = float(np.linalg.norm(o32 - o64) / np.linalg.norm(o64))
        lv = sorted(set(np.round(h.ravel() * 1e6).tolist()))
        meta.append(dict(name=name, shape=list(h.shape), levels=lv if len(lv) <= 8 else f"{len(lv)} distinct",
                         rel32vs64=rel, source=sources.get(name, "designed here"), tied_max=ties,
                         loss64=float(arrays[f"{name}__loss64"])))
        print(f"  {name}: reference fp32 vs fp64 field rel-L2 {rel:.2e}")
    np.savez_compressed(os.path.join(HERE, "e2e_golden.npz"), **arrays)
    with open(os.path.join(HERE, "e2e_manifest.json"), "w") as fh:
        json.dump(dict(cases=meta, f_ghz=F0 / 1e9, material=[EPS, TAND], foci_mm=FOCI9), fh, indent=1)


if __name__ == "__main__":
    main()
