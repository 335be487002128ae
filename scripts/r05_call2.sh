#!/bin/bash
# round-5 GPU call: loss-gradient diagnostic, the DOE / trainer GPU tests, kernel traces of the small
# graph-replayed steps, then the 6,000-iteration QAT quality runs of the three systems.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05c2
timeout -k 10 120 python3 scripts/diag_loss_grad.py > gpurun_out/r05c2/diag.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_doe_fused_bwd_gpu.py \
  tests/test_doe_gpu.py tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_qat_multi_gpu.py \
  tests/test_loss_fusion_gpu.py tests/test_e2e_gpu.py > gpurun_out/r05c2/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05c2/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r05_small_traces.sh gpurun_out/r05_small || exit $?
for s in four_focal dual edof; do
  timeout -k 10 900 python3 -u scripts/qat_quality.py --system $s --seeds 3 --out gpurun_out/r05_qq_$s.json || exit $?
done
