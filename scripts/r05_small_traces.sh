#!/bin/bash
# Kernel traces of the small graph-replayed training steps (scripts/small_prof.py): per workload a
# plain timing run, then a rocprofv3 kernel trace of the same run.
# usage: scripts/r05_small_traces.sh <outdir> [workloads...]
set -o pipefail
out=${1:-gpurun_out/r05_small}; shift || true
W=${*:-donn32 donn256 qat dual edof}
export TMPDIR=/tmp
mkdir -p "$out"
for w in $W; do
  timeout -k 10 180 python3 -u scripts/small_prof.py $w 200 > "$out/$w.time" 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/$w" -o run --output-format csv -- python3 scripts/small_prof.py $w 20 > "$out/$w.log" 2>&1 || exit $?
  cat "$out/$w.time"
done
