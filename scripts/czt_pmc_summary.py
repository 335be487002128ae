#!/usr/bin/env python3
"""Summarise scripts/r03_czt.sh output into profiles/: <tag>_czt_kernel_stats.csv (rocprofv3
--stats) and <tag>_czt_pmc_summary.json (per-kernel averages of every counter; hbm_bytes =
(2 FETCH_SIZE + WRITE_SIZE) * 1024, the gfx950 correction of scripts/pmc_summary.py).
usage: czt_pmc_summary.py <dir> <tag>"""
import glob
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import per_kernel  # noqa: E402


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_czt_kernel_stats.csv"))
    acc = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
        for k, d in per_kernel(f).items():
            acc.setdefault(k, {}).update(d)
    for d in acc.values():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        if d.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_per_lds_inst"] = d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_INSTS_LDS"]
    with open(os.path.join(prof, f"{tag}_czt_pmc_summary.json"), "w") as f:
        json.dump(acc, f, indent=1)
    print(json.dumps({k: round(v.get("hbm_bytes", 0) / 1e6, 1) for k, v in acc.items()}))


if __name__ == "__main__":
    main()
