#!/bin/bash
# A/B of the 300-point column pass's waves-per-SIMD bound (MX_WPE 8 -> spills, 6 -> none) on the
# small graph-replayed steps: shipped library vs quantizationawarethzdoe_amd/libthzdoe_wpe6.so
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wpe
B=$PWD/quantizationawarethzdoe_amd/libthzdoe_wpe6.so
for i in 1 2; do
  for w in donn32 donn256 qat dual edof; do
    timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
    THZDOE_LIB=$B timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/b$i /" || exit $?
  done
done 2>&1 | tee gpurun_out/wpe/ab.log
