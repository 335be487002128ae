#!/bin/bash
# DOE / loss / trainer GPU tests on the current library, then the MX_WPE A/B on the small steps
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05c3
timeout -k 10 900 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_doe_fused_bwd_gpu.py \
  tests/test_multiplane_loss_gpu.py tests/test_loss_fusion_gpu.py tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py \
  tests/test_qat_multi_gpu.py tests/test_e2e_gpu.py tests/test_doe_gpu.py tests/test_qat_quality_gpu.py \
  > gpurun_out/r05c3/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05c3/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r05_wpe.sh
