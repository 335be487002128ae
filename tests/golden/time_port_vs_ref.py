"""SURVEY.md §8(d) check of the CPU baseline: the oracle's ASM forward (the "port" that bench.py's
``cpu_baseline`` times on the GPU box) against the reference itself, on the cfg2 geometry, in THIS
container (the reference does not travel to the GPU box).

Both run the same plane: a 4096^2 Gaussian beam (w0 50 mm, 300 GHz, dx 0.25 mm) padded to
P = 8192 with the exact band limit, at z = 20 / 70 / 120 mm, torch-CPU fp32 on 8 threads, median of
``--reps`` calls each.  The reference path is ``Props/ASM_Prop.py:314-378`` (``ASM_prop.forward``)
imported from /root/reference through ``_refimport`` (build container only); the port is
``oracle.thz_oracle.asm_forward``.  Checks: outputs equal (rel-L2 <= 1e-6) and timing within ±15 %.
Writes profiles/r02_port_vs_reference_cpu.json.

usage: python tests/golden/time_port_vs_ref.py [--reps 3]
"""
import argparse
import contextlib
import io
import json
import os
import platform
import statistics
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from _refimport import import_reference  # noqa: E402

import bench  # noqa: E402  (cfg2 constants and the CPU Gaussian input)
from oracle import thz_oracle as orc  # noqa: E402


def timed(fn, reps):
    ts, out = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_port_vs_reference_cpu.json"))
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    ref = import_reference()
    x = bench.gaussian(bench.N_FIELD, bench.DX, bench.WAIST, "cpu")
    lam_f = bench.C0 / bench.FREQ
    lam = torch.tensor([lam_f], dtype=torch.float32)
    sp = torch.tensor([bench.DX, bench.DX], dtype=torch.float32)
    field = ref.ElectricField(data=x.clone(), wavelengths=lam_f, spacing=[bench.DX, bench.DX], device="cpu")
    rows = []
    orc.asm_forward(x[..., :512, :512], lam, sp, 0.02, 1)  # warm the FFT plans
    for z in (20e-3, 70e-3, 120e-3):
        prop = ref.ASM.ASM_prop(z_distance=z, padding_scale=1, bandlimit_kernel=True, bandlimit_type="exact",
                                device="cpu")

        def run_ref():
            with contextlib.redirect_stdout(io.StringIO()):
                return prop.forward(field).data

        t_ref, ts_ref, y_ref = timed(run_ref, args.reps)
        t_port, ts_port, y_port = timed(lambda: orc.asm_forward(x, lam, sp, z, 1), args.reps)
        a, b = y_port.numpy().astype(np.complex128), y_ref.numpy().astype(np.complex128)
        rel = float(np.linalg.norm(a - b) / np.linalg.norm(b))
        rows.append({"z_m": z, "reference_s": t_ref, "port_s": t_port, "port_over_reference": t_port / t_ref,
                     "reference_runs_s": ts_ref, "port_runs_s": ts_port, "rel_l2_port_vs_reference": rel})
        print(f"z={z * 1e3:.0f} mm reference {t_ref:.2f} s port {t_port:.2f} s ratio {t_port / t_ref:.3f} "
              f"rel-L2 {rel:.2e}", flush=True)
    ratio = statistics.median(r["port_over_reference"] for r in rows)
    ok = abs(ratio - 1.0) <= 0.15 and all(r["rel_l2_port_vs_reference"] <= 1e-6 for r in rows)
    res = {"check": "SURVEY.md §8(d): the port's timing within ±15 % of the reference, outputs equal",
           "workload": "cfg2 plane: 4096^2 Gaussian beam -> P = 8192, exact band limit, 300 GHz, dx 0.25 mm",
           "threads": args.threads, "cpu": platform.processor() or bench.cpu_model(), "cpu_model": bench.cpu_model(),
           "median_port_over_reference": ratio, "ok": ok, "planes": rows}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({"median_port_over_reference": ratio, "ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
