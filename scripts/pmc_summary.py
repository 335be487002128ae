#!/usr/bin/env python3
"""Summarise a scripts/profile_asm.sh run into profiles/ (committed evidence).

Writes, for round tag R:
  profiles/R_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary (copied)
  profiles/R_pmc_summary.json   -- per-kernel averages of every PMC counter collected
  profiles/pmc_traffic.json     -- HBM bytes per launch per kernel, read by bench.py

HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  MI355X_MICROARCH.md §HBM: FETCH_SIZE
reads half the bytes of a wide streaming read on gfx950; calibrated here on our own 8-B/lane
accesses: asm_rows_inv gathers exactly 16 x 134.6 MB of U per launch (z_chunk 16) and
FETCH_SIZE read 1.09 GB (0.50x); asm_cols reads the 134.6 MB T once and read 76.6 MB
(0.57x).  WRITE_SIZE matched the known 2.15 GB of contiguous stores of both kernels within
1 %, so it is used as is ("Measurement").
"""
import collections
import csv
import json
import os
import shutil
import sys


def per_kernel(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "thz::" not in k:
            continue
        k = k.split("(")[0].replace("void thz::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    summ = {}
    for sub in ("fetch", "write", "sq", "sq2"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            for k, d in per_kernel(p).items():
                summ.setdefault(k, {}).update(d)
    import datetime
    traffic = {"_meta": {"profile": f"profiles/{tag}_pmc_summary.json", "date": datetime.date.today().isoformat(),
                         "note": "per-launch HBM bytes of the bench's cfg2 kernels, keyed by bench.py's timer names"}}
    # kernel name -> the KernelTimer name bench.py reports it under (the middle-crop row pass is
    # timed as asm_rows_inv)
    alias = {"asm_rows_inv_mid": "asm_rows_inv"}
    for k, d in summ.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            b = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
            d["hbm_bytes_per_launch"] = b
            base = k.split("<")[0]
            traffic[alias.get(base, base)] = int(b)
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
