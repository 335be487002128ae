#!/usr/bin/env python3
"""The bench line's HIP-event kernel averages against rocprofv3's durations of the same dispatches.

rocprofv3's --stats average covers every dispatch of the run, the bench's warm-up launches included;
bench.py's HIP events cover only the timed steps.  This script reads the kernel trace of
scripts/profile_asm.sh's trace pass and the bench line that pass printed, drops the warm-up
dispatches, and writes both averages side by side:

    python3 scripts/trace_vs_events.py gpurun_out/<tag>/prof profiles/<name>.json
"""
import csv
import json
import os
import sys

KERNELS = {"asm_rows_fwd": "asm_rows_fwd<8192", "asm_cols": "asm_cols<8192>", "asm_rows_inv": "asm_rows_inv_mid<8192>"}


def main():
    prof, out = sys.argv[1], sys.argv[2]
    line = None
    with open(os.path.join(prof, "trace.log")) as fh:
        for text in fh:
            if text.startswith('{"metric'):
                line = json.loads(text)
    rows = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    res = {"source": prof, "warmup": line["warmup"], "steps": line["steps"], "kernels": {}}
    for key, pat in KERNELS.items():
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if pat in r["Kernel_Name"]]
        timed = ds[line["warmup"]:]
        ev = line["kernels"][key]["avg_ms"]
        tr = sum(timed) / len(timed)
        res["kernels"][key] = {"hip_events_avg_ms": ev, "rocprof_timed_avg_ms": round(tr, 4),
                               "rocprof_all_avg_ms": round(sum(ds) / len(ds), 4), "dispatches": len(ds),
                               "rel_diff_timed": round(tr / ev - 1, 4)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["kernels"]))


if __name__ == "__main__":
    main()
