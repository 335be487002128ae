#!/bin/bash
# QAT / DONN / loss parity subset, then the cfg4 / cfg5 timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "${1:-loss_fusion or optics or donn or doe or dropin}" > gpurun_out/small_tests.log 2>&1 || { tail -40 gpurun_out/small_tests.log; exit 1; }
tail -2 gpurun_out/small_tests.log
for rep in 1 2; do
  timeout -k 10 200 python scripts/small_bench.py > gpurun_out/small_$rep.log 2>&1 || { tail -20 gpurun_out/small_$rep.log; exit 1; }
  echo $(tail -1 gpurun_out/small_$rep.log)
done
