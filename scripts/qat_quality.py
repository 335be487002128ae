#!/usr/bin/env python3
"""Reproduce the reference's published QAT quality: the four-focal-spots system trained for 6,000
iterations with each quantisation method of experiment_four_focal_spots.ipynb, several seeds each,
on the HIP path (graph-replayed trainer), compared with the reference's own loss curves
(tests/golden/qat_curves.json, made by tests/golden/gen_qat_curves.py from
/root/reference/plot_data/example_1/loss_curve_*.npy).

Methods (notebook cells): v3 "Ours" (cell 6-8: SoftGumbelQuantizedDOELayerv3, c_s 100, tau 2.5 ->
1.5, Adam), "full" (cells 19-22: FullPrecisionDOELayer, AdamW), "GS" (cells 31-33: NaiveGumbel,
c_s 100, tau 5.5 -> 1.0, AdamW), "PSQ" (cells 41-43: c_s 300, tau 400 -> 1, Adam), "STE" (cells
50-52: AdamW).  lr 0.02 and iter_frac = itr / 6000 everywhere.  The notebook's GS and STE cells
ran 30,000 iterations (its "_more_iterations" files); the 6,000-entry curves compared here are the
6,000-iteration runs, so 6,000 iterations with iter_frac = itr / 6000 are run.

    python scripts/qat_quality.py [--seeds 5] [--methods Ours,STE,...] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METHODS = {
    "Ours": ("SoftGumbelQuantizedDOELayerv3", {"c_s": 100, "tau_max": 2.5, "tau_min": 1.5}, "adam"),
    "full": ("FullPrecisionDOELayer", None, "adamw"),
    "GS": ("NaiveGumbelQuantizedDOELayer", {"c_s": 100, "tau_max": 5.5, "tau_min": 1.0}, "adamw"),
    "PSQ": ("PSQuantizedDOELayer", {"c_s": 300, "tau_max": 400, "tau_min": 1}, "adam"),
    "STE": ("STEQuantizedDOELayer", {"c_s": 300, "tau_max": 400, "tau_min": 1}, "adamw"),
}
TRACE_ITERS = list(range(0, 6000, 200)) + [5999]


def stats(curve):
    c = np.asarray(curve, dtype=np.float64)
    return {"final": float(c[-1]), "min": float(c.min()), "argmin": int(c.argmin()),
            "mean_last100": float(c[-100:].mean()), "trace": [float(c[i]) for i in TRACE_ITERS]}


def run_method(name, seed, iters=6000, device="cuda:0"):
    from quantizationawarethzdoe_amd import qat
    from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
    cls_name, op, opt = METHODS[name]
    torch.manual_seed(seed)
    dp, op0 = qat.default_params()
    system = qat.FourFocalSpotsSystem(doe_class=getattr(Q, cls_name), optim_params=op or op0,
                                      device=torch.device(device))
    trainer = qat.QATTrainer(system, qat.four_focal_spots_target(device=torch.device(device)), lr=0.02,
                             max_itrs=iters, graph=True, optimizer=opt)
    losses, dt = trainer.train(iters, log_every=0)
    return losses.double().numpy(), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--methods", default=",".join(METHODS))
    ap.add_argument("--iters", type=int, default=6000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "qat_quality.json"))
    args = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "qat_curves.json")) as fh:
        ref = json.load(fh)
    res = {"iters": args.iters, "seeds": args.seeds, "methods": {}}
    for name in args.methods.split(","):
        runs = []
        for seed in range(args.seeds):
            curve, dt = run_method(name, seed, args.iters)
            st = stats(curve)
            st.update(seed=seed, seconds=round(dt, 3), ms_per_it=round(dt / args.iters * 1e3, 4))
            runs.append(st)
            print(f"{name} seed {seed}: final {st['final']:.3e} min {st['min']:.3e} last100 {st['mean_last100']:.3e} "
                  f"({dt:.1f} s)", flush=True)
        med = {k: float(np.median([r[k] for r in runs])) for k in ("final", "min", "mean_last100")}
        r = ref["methods"][name]
        res["methods"][name] = {"runs": runs, "median": med, "reference": {k: r[k] for k in ("final", "min", "mean_last100")},
                                "ratio_to_reference": {k: med[k] / r[k] for k in med}}
        print(f"{name}: median final {med['final']:.3e} (ref {r['final']:.3e}), min {med['min']:.3e} "
              f"(ref {r['min']:.3e}), last100 {med['mean_last100']:.3e} (ref {r['mean_last100']:.3e})", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
