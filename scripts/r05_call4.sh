#!/bin/bash
# the gradient-slot / DONN static-input changes: trainer + collective tests, then the small steps
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05c4
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_collective_capture_gpu.py \
  tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_qat_multi_gpu.py tests/test_doe_fused_bwd_gpu.py \
  tests/test_e2e_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|one-rank RCCL" $O/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in donn32 donn256 qat; do timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" || exit $?; done
