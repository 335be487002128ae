#!/usr/bin/env python3
"""Reproduce the reference's published QAT quality: each of its three QAT systems trained for 6,000
iterations with each quantisation method of its notebook, several seeds each, on the HIP path
(graph-replayed trainer), compared with the reference's own loss curves (tests/golden/qat_curves.json,
made by tests/golden/gen_qat_curves.py from /root/reference/plot_data/example_{1,2,3}/loss_curve_*.npy).

Systems and methods (notebook cells; lr and optimiser as each cell):
  * four_focal (plot_data/example_1, experiment_four_focal_spots.ipynb): v3 "Ours" (cells 6-8:
    SoftGumbelQuantizedDOELayerv3, c_s 100, tau 2.5 -> 1.5, Adam), "full" (cells 19-22:
    FullPrecisionDOELayer, AdamW), "GS" (cells 31-33: NaiveGumbel, c_s 100, tau 5.5 -> 1.0, AdamW),
    "PSQ" (cells 41-43: c_s 300, tau 400 -> 1, Adam), "STE" (cells 50-52: AdamW); lr 0.02.
  * dual (plot_data/example_2, experiment_dual_plane_hologram.ipynb): "Ours" (cells 6-8, AdamW),
    "full" (16-18, AdamW), "GQ" (39-41: NaiveGumbel with cell 2's c_s 100, tau 2.5 -> 1.5, AdamW),
    "PSQ" (46-48: c_s 300, tau 800 -> 1, Adam), "STE" (53-55, Adam); lr 0.01; every method but
    "Ours" with the second 127 mm propagation before the aperture.
  * edof (plot_data/example_3, experiment_extend_depth_of_focus.ipynb): the rotationally symmetric
    layers, "Ours" (22-24, AdamW), "full" (6-8, AdamW, second propagation), "STE" (35-37, AdamW),
    "GQ" (44-46, Adam), "PSQ" (52-54: c_s 300, tau 400 -> 1, Adam); lr 0.02; five planes re-drawn
    every iteration.
iter_frac = itr / 6000 everywhere.  The four-focal notebook's GS and STE cells ran 30,000 iterations
(its "_more_iterations" files); the 6,000-entry curves compared here are the 6,000-iteration runs.

    python scripts/qat_quality.py [--system four_focal] [--seeds 5] [--methods Ours,STE,...] [--out FILE]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# method -> (layer class, optim_params or None, optimiser)
SYSTEMS = {
    "four_focal": {
        "curves": "methods", "lr": 0.02,
        "methods": {
            "Ours": ("SoftGumbelQuantizedDOELayerv3", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}, "adam"),
            "full": ("FullPrecisionDOELayer", None, "adamw"),
            "GS": ("NaiveGumbelQuantizedDOELayer", {"c_s": 100, "tau_max": 5.5, "tau_min": 1.0}, "adamw"),
            "PSQ": ("PSQuantizedDOELayer", {"c_s": 300, "tau_max": 400, "tau_min": 1}, "adam"),
            "STE": ("STEQuantizedDOELayer", {"c_s": 300, "tau_max": 400, "tau_min": 1}, "adamw"),
        }},
    "dual": {
        "curves": "example_2", "lr": 0.01,
        "methods": {
            "Ours": ("SoftGumbelQuantizedDOELayerv3", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}, "adamw"),
            "full": ("FullPrecisionDOELayer", None, "adamw"),
            "GQ": ("NaiveGumbelQuantizedDOELayer", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}, "adamw"),
            "PSQ": ("PSQuantizedDOELayer", {"c_s": 300, "tau_max": 800, "tau_min": 1}, "adam"),
            "STE": ("STEQuantizedDOELayer", {"c_s": 300, "tau_max": 800, "tau_min": 1}, "adam"),
        }},
    "edof": {
        "curves": "example_3", "lr": 0.02,
        "methods": {
            "Ours": ("RotationallySymmetricScoreGumbelSoftQuantizedDOELayer",
                     {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}, "adamw"),
            "full": ("RotationallySymmetricFullPrecisionDOELayer", None, "adamw"),
            "STE": ("RotationallySymmetricSTEQuantizedDOELayer", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5},
                    "adamw"),
            "GQ": ("RotationallySymmetricNaiveGumbelQuantizedDOELayer", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5},
                   "adam"),
            "PSQ": ("RotationallySymmetricPSQuantizedQuantizedDOELayer", {"c_s": 300, "tau_max": 400, "tau_min": 1},
                    "adam"),
        }},
}
# backwards-compatible name of the four-focal-spots table
METHODS = SYSTEMS["four_focal"]["methods"]
TRACE_ITERS = list(range(0, 6000, 200)) + [5999]


def stats(curve):
    c = np.asarray(curve, dtype=np.float64)
    return {"final": float(c[-1]), "min": float(c.min()), "argmin": int(c.argmin()),
            "mean_last100": float(c[-100:].mean()), "trace": [float(c[i]) for i in TRACE_ITERS if i < len(c)]}


def reference(system, name):
    with open(os.path.join(ROOT, "tests", "golden", "qat_curves.json")) as fh:
        ref = json.load(fh)
    key = SYSTEMS[system]["curves"]
    return (ref[key] if key == "methods" else ref[key]["methods"])[name]


def run_method(name, seed, iters=6000, device="cuda:0", system="four_focal"):
    from quantizationawarethzdoe_amd import qat
    from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
    spec = SYSTEMS[system]
    cls_name, op, opt = spec["methods"][name]
    dev = torch.device(device)
    torch.manual_seed(seed)
    if system == "four_focal":
        _, op0 = qat.default_params()
        model = qat.FourFocalSpotsSystem(doe_class=getattr(Q, cls_name), optim_params=op or op0, device=dev)
        target = qat.four_focal_spots_target(device=dev)
    elif system == "dual":
        model = qat.DualPlaneSystem(doe_class=getattr(Q, cls_name), optim_params=op, device=dev)
        target = qat.logo_targets(device=dev)
    else:
        model = qat.ExtendedDOFSystem(doe_class=getattr(Q, cls_name), optim_params=op, seed=seed, device=dev)
        target = qat.edof_target(device=dev)
    trainer = qat.QATTrainer(model, target, lr=spec["lr"], max_itrs=iters, graph=True, optimizer=opt)
    losses, dt = trainer.train(iters, log_every=0)
    return losses.double().numpy(), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--system", default="four_focal", choices=list(SYSTEMS))
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--methods", default=None)
    ap.add_argument("--iters", type=int, default=6000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    spec = SYSTEMS[args.system]
    out = args.out or os.path.join(ROOT, "gpurun_out", f"qat_quality_{args.system}.json")
    res = {"system": args.system, "iters": args.iters, "seeds": args.seeds, "methods": {}}
    for name in (args.methods.split(",") if args.methods else list(spec["methods"])):
        runs = []
        for seed in range(args.seeds):
            curve, dt = run_method(name, seed, args.iters, system=args.system)
            st = stats(curve)
            st.update(seed=seed, seconds=round(dt, 3), ms_per_it=round(dt / args.iters * 1e3, 4),
                      finite=bool(np.all(np.isfinite(curve))))
            runs.append(st)
            print(f"{args.system} {name} seed {seed}: final {st['final']:.3e} min {st['min']:.3e} "
                  f"last100 {st['mean_last100']:.3e} ({dt:.1f} s)", flush=True)
        med = {k: float(np.median([r[k] for r in runs])) for k in ("final", "min", "mean_last100")}
        r = reference(args.system, name)
        res["methods"][name] = {"runs": runs, "median": med, "reference": {k: r[k] for k in ("final", "min", "mean_last100")},
                                "ratio_to_reference": {k: med[k] / r[k] for k in med}}
        print(f"{args.system} {name}: median final {med['final']:.3e} (ref {r['final']:.3e}), min {med['min']:.3e} "
              f"(ref {r['min']:.3e}), last100 {med['mean_last100']:.3e} (ref {r['mean_last100']:.3e})", flush=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
