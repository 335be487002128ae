#!/bin/bash
# A/B of the resident-loop 300-point column pass (THZ_MX_LOOP=2 builds: WPE 5 and 6) on the batch-256
# DONN step, then the DONN / QAT tests on the WPE-5 build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/loop
mkdir -p $O
L5=$PWD/quantizationawarethzdoe_amd/libthzdoe_loop5.so
L6=$PWD/quantizationawarethzdoe_amd/libthzdoe_loop6.so
for i in 1 2; do
  timeout -k 10 120 python3 -u scripts/small_prof.py donn256 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
  THZDOE_LIB=$L5 timeout -k 10 120 python3 -u scripts/small_prof.py donn256 300 2>/dev/null | grep "ms per step" | sed "s/^/l5_$i /" || exit $?
  THZDOE_LIB=$L6 timeout -k 10 120 python3 -u scripts/small_prof.py donn256 300 2>/dev/null | grep "ms per step" | sed "s/^/l6_$i /" || exit $?
done 2>&1 | tee $O/ab.log
THZDOE_LIB=$L5 timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py > $O/tests_l5.log 2>&1
tail -3 $O/tests_l5.log
