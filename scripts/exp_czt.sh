#!/bin/bash
# CZT A/B over library variants (default + libthzdoe_exp<N>.so): parity subset + cfg3 timing each.
set -u
mkdir -p gpurun_out
for v in 0 "$@"; do
  if [ $v = 0 ]; then L=quantizationawarethzdoe_amd/libthzdoe.so; else L=quantizationawarethzdoe_amd/libthzdoe_exp$v.so; fi
  THZDOE_LIB=$PWD/$L timeout -k 10 300 python -m pytest tests/test_czt_gpu.py -q -x -m gpu > gpurun_out/expczt_t$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/expczt_t$v.log; exit 1; }
  for rep in 1 2; do
    THZDOE_LIB=$PWD/$L timeout -k 10 200 python scripts/czt_prof.py 20 > gpurun_out/expczt_$v.$rep.log 2>&1 || { echo "time $v failed"; exit 1; }
    echo "$v: $(tail -1 gpurun_out/expczt_t$v.log) $(grep workload gpurun_out/expczt_$v.$rep.log | sed 's/.*ms_per_call/ms_per_call/')"
  done
done
