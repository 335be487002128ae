#!/bin/bash
# A/B of the column-pair 300-point column pass (THZ_MX_PAIR=1 build, libthzdoe_pair.so) on the small
# graph-replayed steps, then the P = 300 GPU tests on the pair build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/pair
mkdir -p $O
B=$PWD/quantizationawarethzdoe_amd/libthzdoe_pair.so
for i in 1 2; do
  for w in donn32 donn256 qat dual; do
    timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
    THZDOE_LIB=$B timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/b$i /" || exit $?
  done
done 2>&1 | tee $O/ab.log
THZDOE_LIB=$B timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_qat_multi_gpu.py tests/test_loss_fusion_gpu.py \
  tests/test_multiplane_loss_gpu.py tests/test_doe_fused_bwd_gpu.py tests/test_e2e_gpu.py tests/test_asm_gpu.py \
  tests/test_doe_gpu.py > $O/tests_b.log 2>&1
tail -3 $O/tests_b.log
