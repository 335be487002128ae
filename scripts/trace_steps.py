#!/usr/bin/env python3
"""Per-step kernel sequence of a rocprofv3 kernel trace (kernel_trace.csv): the last ``n`` kernels
before the end of the trace, i.e. the last replayed step(s), with each kernel's duration and the gap
since the previous kernel ended.

    python3 scripts/trace_steps.py <dir with */kernel_trace.csv> [kernels_per_step]
"""
import csv
import glob
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    for p in ("void ", "at::native::"):
        n = n.replace(p, "")
    return n[:90]


def main():
    d = sys.argv[1]
    rows = load(d)
    # a step = the kernels between two consecutive launches of the step's first kernel: find the
    # period from the last repeated name sequence
    names = [short(r["Kernel_Name"]) for r in rows]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else None
    if n is None:  # the shortest period p with the last p names repeating the p before them
        n = next((p for p in range(1, len(names) // 2 + 1) if names[-p:] == names[-2 * p:-p]), len(names))
    seg = rows[-n:]
    t0 = int(seg[0]["Start_Timestamp"])
    prev = None
    busy = 0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += e - s
        print(f"{(s - t0) / 1e3:9.2f} us  +{gap:6.2f}  {(e - s) / 1e3:8.2f} us  {short(r['Kernel_Name'])}")
        prev = e
    span = (int(seg[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"{n} kernels, span {span:.2f} us, busy {busy / 1e3:.2f} us, gaps {span - busy / 1e3:.2f} us")


if __name__ == "__main__":
    main()
