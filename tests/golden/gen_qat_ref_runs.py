#!/usr/bin/env python3
"""Seeded 6,000-iteration runs of the REFERENCE itself (CPU, this container) of the QAT methods of the
four-focal-spots and extended-DOF notebooks (Missing #2: the HIP path sat 1.3-2.6x
above the published extended-DOF curves with nothing to say whether the port or the curve is off).  The published curves
(plot_data/example_{1,3}/loss_curve_*.npy) are ONE unseeded CUDA run each; these runs give the
spread of the same code over seeds, which tests/test_qat_quality_gpu.py grades the HIP runs against.

Systems, exactly as the notebook cells (see gen_qat_multi.py / gen_golden.gen_qat for the optics):
  * edof (plot_data/example_3/experiment_extend_depth_of_focus.ipynb cells 1-3 and "full" 6-8,
    "Ours" 22-24, STE 35-37, GQ 44-46, PSQ 52-54): Gaussian source -> ASM 127 mm (padding 4) -> lens
    [-> ASM 127 mm: "full" only] -> 80 mm aperture -> the rotationally symmetric layer of the cell
    (doe_params of cell 1, optim_params c_s 100, tau 2.5 -> 1.5 except PSQ's c_s 300, tau 400 -> 1)
    -> five ASM planes at 50..90 mm re-drawn after every forward; loss = sum of the five
    MSE(normalize(|E|^2), PSF(f = 100 mm)); lr 0.02, AdamW ("Ours", STE, "full") or Adam (GQ, PSQ).
  * dual (plot_data/example_2/experiment_dual_plane_hologram.ipynb cells 2-8 "Ours", 16-18 "full",
    39-41 GQ, 46-48 PSQ, 53-55 STE): the same optics with padding 2, the second 127 mm propagation
    before the aperture in every cell but "Ours" (cell 6 comments it out), tolerance 50 um, tan d
    0.003, num_unit None, planes at 100 and 150 mm against the two Aalto logos (the package's decoded
    copy, data/dual_plane_targets.npz, made by gen_qat_multi.py from the notebook's cells 3-4); loss =
    the two MSEs summed; lr 0.01, AdamW ("Ours", "full", GQ) or Adam (PSQ, STE; c_s 300, tau 800 -> 1).
  * four_focal (experiment_four_focal_spots.ipynb "Ours" 6-8, "full" 19-22, GS 31-33, PSQ 41-43,
    STE 50-52): the 9-spot target at 200 mm, padding 2, num_unit 2; GS c_s 100, tau 5.5 -> 1.0;
    PSQ and STE c_s 300, tau 400 -> 1 (cell 42's dict, still in force at cell 51); lr 0.02, Adam
    ("Ours", PSQ) or AdamW ("full", GS, STE).
iter_frac = itr / 6000.  Seed s: torch.manual_seed(s) before the layer is built (its weight init)
and before the loop (the Gumbel / fabrication noise), random.seed(s) (the planes' jitter).

Output: tests/golden/qat_ref_runs.json, per "system/method": one entry per seed with the final,
minimum, argmin, mean of the last 100 iterations and the loss every 200 iterations (the same
statistics as scripts/qat_quality.stats).  Runs only in the build container:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_qat_ref_runs.py --system edof --method Ours --seed 0
"""
import argparse
import contextlib
import fcntl
import io
import json
import os
import random
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refimport import import_reference  # noqa: E402

C0 = 2.998e8
MM = 1e-3
TRACE_ITERS = list(range(0, 6000, 200)) + [5999]
OUT = os.path.join(HERE, "qat_ref_runs.json")
FOCI = [(-20, -20), (20, 20), (-20, 20), (20, -20), (0, 0), (0, -20), (-20, 0), (0, 20), (20, 0)]


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def fom(ref, resolution, dxy, wavelength, focal_length, position):
    """The notebooks' define_FoM (cell 2), restated on CPU."""
    h, w = resolution
    Lx, Ly = dxy * w, dxy * h
    effL = torch.sqrt(torch.tensor(Lx ** 2 + Ly ** 2))
    NA = torch.sin(torch.atan(effL / (2 * focal_length)))
    fwhm = wavelength / (2 * NA)
    xg, yg = torch.meshgrid(torch.linspace(-Lx / 2, Lx / 2, steps=w), torch.linspace(-Ly / 2, Ly / 2, steps=h),
                            indexing="ij")
    x0, y0 = torch.tensor(position)
    psf = torch.exp(-((xg - x0) ** 2 + (yg - y0) ** 2) / ((fwhm * 2) ** 2))
    return ref.HF.normalize(psf.unsqueeze(0).unsqueeze(0))


def optics_before_doe(ref, pad):
    """source -> ASM 127 mm -> lens f = 127 mm -> 80 mm rect aperture (field_before_DOE)."""
    G = ref.import_module("LightSource.Gaussian_beam")
    TL = ref.import_module("Components.Thin_Lens")
    AP = ref.import_module("Components.Aperture")
    src = G.Guassian_beam(height=100, width=100, beam_waist_x=None, beam_waist_y=None, wavelengths=C0 / 300e9,
                          spacing=1 * MM, device="cpu")
    asm1 = ref.ASM.ASM_prop(z_distance=0.127, bandlimit_type='exact', padding_scale=pad, bandlimit_kernel=True,
                            device="cpu")
    lens = TL.Thin_LensElement(focal_length=0.127)
    ap = AP.ApertureElement(aperture_type='rect', aperture_size=0.08)
    f0 = quiet(src)
    if isinstance(f0, tuple):
        f0 = f0[0]
    f1 = quiet(asm1, f0)
    if isinstance(f1, tuple):
        f1 = f1[0]
    return ap(lens(f1))


def stats(curve):
    c = np.asarray(curve, dtype=np.float64)
    return {"final": float(c[-1]), "min": float(c.min()), "argmin": int(c.argmin()),
            "mean_last100": float(c[-100:].mean()), "trace": [float(c[i]) for i in TRACE_ITERS if i < len(c)]}


# method -> (layer class, optim_params (None: the system's cell-1 dict), optimiser, second 127 mm
# propagation before the aperture): the notebook cells named in the module docstring
FOUR_FOCAL = {
    "Ours": ("SoftGumbelQuantizedDOELayerv3", None, "adam", False),
    "full": ("FullPrecisionDOELayer", None, "adamw", False),
    "GS": ("NaiveGumbelQuantizedDOELayer", dict(c_s=100, tau_max=5.5, tau_min=1.0), "adamw", False),
    "PSQ": ("PSQuantizedDOELayer", dict(c_s=300, tau_max=400, tau_min=1), "adam", False),
    "STE": ("STEQuantizedDOELayer", dict(c_s=300, tau_max=400, tau_min=1), "adamw", False),
}
EDOF = {
    "Ours": ("RotationallySymmetricScoreGumbelSoftQuantizedDOELayer", None, "adamw", False),
    "full": ("RotationallySymmetricFullPrecisionDOELayer", None, "adamw", True),
    "STE": ("RotationallySymmetricSTEQuantizedDOELayer", None, "adamw", False),
    "GQ": ("RotationallySymmetricNaiveGumbelQuantizedDOELayer", None, "adam", False),
    "PSQ": ("RotationallySymmetricPSQuantizedQuantizedDOELayer", dict(c_s=300, tau_max=400, tau_min=1), "adam", False),
}


DUAL = {
    "Ours": ("SoftGumbelQuantizedDOELayerv3", None, "adamw", False),
    "full": ("FullPrecisionDOELayer", None, "adamw", True),
    "GQ": ("NaiveGumbelQuantizedDOELayer", None, "adamw", True),
    "PSQ": ("PSQuantizedDOELayer", dict(c_s=300, tau_max=800, tau_min=1), "adam", True),
    "STE": ("STEQuantizedDOELayer", dict(c_s=300, tau_max=800, tau_min=1), "adam", True),
}


def optics_before_doe2(ref, pad, second):
    """optics_before_doe with the optional second ASM 127 mm after the lens (cells whose
    field_before_DOE runs asm_prop2)."""
    if not second:
        return optics_before_doe(ref, pad)
    G = ref.import_module("LightSource.Gaussian_beam")
    TL = ref.import_module("Components.Thin_Lens")
    AP = ref.import_module("Components.Aperture")
    src = G.Guassian_beam(height=100, width=100, beam_waist_x=None, beam_waist_y=None, wavelengths=C0 / 300e9,
                          spacing=1 * MM, device="cpu")
    kw = dict(bandlimit_type='exact', padding_scale=pad, bandlimit_kernel=True, device="cpu")
    asm1 = ref.ASM.ASM_prop(z_distance=0.127, **kw)
    asm2 = ref.ASM.ASM_prop(z_distance=0.127, **kw)
    lens = TL.Thin_LensElement(focal_length=0.127)
    ap = AP.ApertureElement(aperture_type='rect', aperture_size=0.08)
    unt = (lambda f: f[0] if isinstance(f, tuple) else f)
    f = unt(quiet(src))
    f = lens(unt(quiet(asm1, f)))
    return ap(unt(quiet(asm2, f)))


def make_layer(ref, cls, doe_params, optim_params):
    """The cell's layer: the full-precision layers take no optim_params (QuantizedDOE.py:182-184)."""
    if "FullPrecision" in cls:
        return getattr(ref.DOE, cls)(doe_params, device="cpu")
    return getattr(ref.DOE, cls)(doe_params, optim_params, device="cpu")


def run(system, method, seed, iters):
    ref = import_reference()
    HF = ref.HF
    mse = torch.nn.MSELoss()
    if system == "edof":
        doe_params = dict(doe_size=[100, 100], doe_dxy=1 * MM, doe_level=4, look_up_table=None, num_unit=None,
                          height_constraint_max=1 * MM, tolerance=10e-6, material=[2.66, 0.03])
        cls, op, optname, second = EDOF[method]
        optim_params = op or dict(c_s=100, tau_max=2.5, tau_min=1.5)
        target = fom(ref, [100, 100], 1 * MM, C0 / 300e9, 100 * MM, [0.0, 0.0])
        field_in = optics_before_doe2(ref, 4, second)
        torch.manual_seed(seed)
        doe = make_layer(ref, cls, doe_params, optim_params)
        props = [ref.ASM.ASM_prop(z_distance=z * MM, bandlimit_type='exact', padding_scale=4, bandlimit_kernel=True,
                                  device="cpu") for z in (50, 60, 70, 80, 90)]
        jitter = [(50, 0, 5), (60, -5, 5), (70, -5, 5), (80, -5, 5), (90, -5, 0)]
        targets = [target] * 5
    elif system == "dual":
        doe_params = dict(doe_size=[100, 100], doe_dxy=1 * MM, doe_level=4, look_up_table=None, num_unit=None,
                          height_constraint_max=1 * MM, tolerance=0.05 * MM, material=[2.66, 0.003])
        cls, op, optname, second = DUAL[method]
        optim_params = op or dict(c_s=100, tau_max=2.5, tau_min=1.5)
        tt = np.load(os.path.join(os.path.dirname(os.path.dirname(HERE)), "quantizationawarethzdoe_amd", "data",
                                  "dual_plane_targets.npz"))["targets"].astype(np.float32)
        field_in = optics_before_doe2(ref, 2, second)
        torch.manual_seed(seed)
        doe = make_layer(ref, cls, doe_params, optim_params)
        props = [ref.ASM.ASM_prop(z_distance=z * MM, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True,
                                  device="cpu") for z in (100, 150)]
        jitter = None
        targets = [torch.from_numpy(tt[i]).reshape(1, 1, 100, 100) for i in range(2)]
    elif system == "four_focal":
        doe_params = dict(doe_size=[100, 100], doe_dxy=1 * MM, doe_level=4, look_up_table=None, num_unit=2,
                          height_constraint_max=1 * MM, tolerance=10e-6, material=[2.66, 0.03])
        cls, op, optname, second = FOUR_FOCAL[method]
        optim_params = op or dict(c_s=100, tau_max=2.5, tau_min=1.5)
        wl = C0 / 300e9
        target = sum(fom(ref, [100, 100], 1 * MM, wl, 200 * MM, [a * MM, b * MM]) for a, b in FOCI)
        field_in = optics_before_doe2(ref, 2, second)
        torch.manual_seed(seed)
        doe = make_layer(ref, cls, doe_params, optim_params)
        props = [ref.ASM.ASM_prop(z_distance=200 * MM, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True,
                                  device="cpu")]
        jitter = None
        targets = [target]
    else:
        raise SystemExit(f"unknown system {system}")
    lr = 0.01 if system == "dual" else 0.02
    opt = (torch.optim.AdamW if optname == "adamw" else torch.optim.Adam)(doe.parameters(), lr=lr)
    torch.manual_seed(seed)
    random.seed(seed)
    losses = []
    t0 = time.time()
    for itr in range(iters):
        mid = doe(field_in, itr / iters)
        outs = [quiet(p, mid) for p in props]
        if jitter is not None:  # cell 22's forward: the planes move after the five propagations
            for p, (c, lo, hi) in zip(props, jitter):
                p.z = c * MM + random.uniform(lo * MM, hi * MM)
        loss = sum(mse(HF.normalize(torch.abs(o.data) ** 2), t) for o, t in zip(outs, targets))
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
        if itr % 500 == 0:
            print(f"{system}/{method} seed {seed} itr {itr} loss {losses[-1]:.4e} ({time.time() - t0:.0f} s)",
                  file=sys.stderr, flush=True)
    st = stats(losses)
    st.update(seed=seed, iters=iters, seconds=round(time.time() - t0, 1), threads=torch.get_num_threads(),
              finite=bool(np.all(np.isfinite(losses))))
    return st


def merge(key, entry):
    """Add one run to the JSON (a lock file serialises concurrent generators)."""
    with open(OUT + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        data = {}
        if os.path.exists(OUT):
            with open(OUT) as fh:
                data = json.load(fh)
        data.setdefault("source", "the reference itself on CPU (tests/golden/gen_qat_ref_runs.py), torch "
                        + torch.__version__)
        runs = data.setdefault("runs", {}).setdefault(key, [])
        runs[:] = [r for r in runs if r["seed"] != entry["seed"]] + [entry]
        runs.sort(key=lambda r: r["seed"])
        with open(OUT, "w") as fh:
            json.dump(data, fh, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", required=True, choices=["edof", "four_focal", "dual"])
    ap.add_argument("--method", required=True)
    ap.add_argument("--seed", type=int, required=True)
    ap.add_argument("--iters", type=int, default=6000)
    ap.add_argument("--threads", type=int, default=2)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    entry = run(args.system, args.method, args.seed, args.iters)
    merge(f"{args.system}/{args.method}", entry)
    print(json.dumps({k: entry[k] for k in ("final", "min", "mean_last100", "seconds")}), file=sys.stderr)


if __name__ == "__main__":
    main()
