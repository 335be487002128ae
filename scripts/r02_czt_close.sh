#!/bin/bash
# cfg3 CZT evidence at the round-2 close: kernel trace + stats, then the PMC groups of
# scripts/r02_czt_pmc.sh (one pass each); summarise on the CPU with scripts/czt_pmc_summary.py
set -o pipefail
mkdir -p gpurun_out/czt_close
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/czt_close/trace -o run --output-format csv -- python3 scripts/czt_prof.py 10 > gpurun_out/czt_close/trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/czt_close/trace.log; exit 1; }
bash scripts/r02_czt_pmc.sh gpurun_out/czt_close/pmc
