#!/usr/bin/env python3
"""Generate tests/golden/qat_curves.json: summary numbers of the REFERENCE's published QAT loss
curves, /root/reference/plot_data/example_1/loss_curve_{Ours, STE, PSQ, GS, full}.npy and
example_{2, 3}/loss_curve_{Ours, STE, PSQ, GQ, full}.npy (plain float64
[6000] arrays, read with np.load(allow_pickle=False); written by experiment_four_focal_spots.ipynb
cells 13, 28, 39, 48, 56), and the notebook's printed trace of the v3 run (cell 8 output: the loss
every 200 iterations).  Final, minimum, argmin, mean of the last 100 iterations, and the loss every
200 iterations.  Runs only in the build container; the GPU box reads the JSON.

    python tests/golden/gen_qat_curves.py
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("THZ_REFERENCE", "/root/reference")
TRACE_ITERS = list(range(0, 6000, 200)) + [5999]


def main():
    if not os.path.isdir(REF):
        raise SystemExit(f"reference tree {REF} is absent")
    out = {"source": "plot_data/example_1/loss_curve_*.npy (np.load allow_pickle=False)", "trace_iters": TRACE_ITERS,
           "methods": {}}
    for name in ("Ours", "STE", "PSQ", "GS", "full"):
        c = np.load(os.path.join(REF, "plot_data", "example_1", f"loss_curve_{name}.npy"), allow_pickle=False)
        assert c.shape == (6000,) and c.dtype == np.float64
        out["methods"][name] = {"final": float(c[-1]), "min": float(c.min()), "argmin": int(c.argmin()),
                                "mean_last100": float(c[-100:].mean()), "trace": [float(c[i]) for i in TRACE_ITERS]}
    # the dual-plane hologram (example 2, its GS run is named GQ) and the extended depth of focus
    # (example 3): the same statistics per method
    for ex in ("example_2", "example_3"):
        out[ex] = {"source": f"plot_data/{ex}/loss_curve_*.npy (np.load allow_pickle=False)", "methods": {}}
        for name in ("Ours", "STE", "PSQ", "GQ", "full"):
            c = np.load(os.path.join(REF, "plot_data", ex, f"loss_curve_{name}.npy"), allow_pickle=False)
            assert c.shape == (6000,) and c.dtype == np.float64, (ex, name, c.shape, c.dtype)
            out[ex]["methods"][name] = {"final": float(c[-1]), "min": float(c.min()), "argmin": int(c.argmin()),
                                        "mean_last100": float(c[-100:].mean()),
                                        "trace": [float(c[i]) for i in TRACE_ITERS]}
    with open(os.path.join(REF, "experiment_four_focal_spots.ipynb")) as fh:
        nb = json.load(fh)
    text = "".join("".join(o.get("text", "")) for o in nb["cells"][8].get("outputs", []))
    pts = [(int(a), float(b)) for a, b in re.findall(r"The iteration : (\d+), Loss: ([0-9.e+-]+)", text)]
    out["notebook_v3_printed_trace"] = {"cell": 8, "points": pts}
    with open(os.path.join(HERE, "qat_curves.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print({k: (v["final"], v["min"]) for k, v in out["methods"].items()}, len(pts), file=sys.stderr)


if __name__ == "__main__":
    main()
