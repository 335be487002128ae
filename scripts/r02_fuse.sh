#!/bin/bash
# fused-loss parity subset, then cfg4 / cfg5 timings of the default library (A) vs libthzdoe_exp1.so (B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread -k "${1:-loss_fusion or doe or optics or donn or dropin}" > gpurun_out/fuse_tests.log 2>&1 || { tail -40 gpurun_out/fuse_tests.log; exit 1; }
tail -3 gpurun_out/fuse_tests.log
for rep in 1 2; do for v in A B; do
  if [ $v = B ]; then export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp1.so; else unset THZDOE_LIB; fi
  timeout -k 10 200 python scripts/small_bench.py > gpurun_out/small_$v$rep.log 2>&1 || { tail -20 gpurun_out/small_$v$rep.log; exit 1; }
  echo $v $(tail -1 gpurun_out/small_$v$rep.log)
done; done
