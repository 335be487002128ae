#!/bin/bash
# A/B: the 300-point column pass with its tables loaded before the forward transform (THZ_MX_EARLY=1)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/early
mkdir -p $O
B=$PWD/quantizationawarethzdoe_amd/libthzdoe_early.so
for i in 1 2; do
  for w in donn32 donn256 qat dual; do
    timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
    THZDOE_LIB=$B timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/b$i /" || exit $?
  done
done 2>&1 | tee $O/ab.log
