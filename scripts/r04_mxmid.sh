#!/bin/bash
# A/B of the 300-point column pass with compile-time windows (THZ_MX_MID=1) against the default:
# parity tests of the P = 300 paths with it on, DONN step kernel traces, full bench lines (cfg4/5).
set -o pipefail
o=gpurun_out/mxmid
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
THZ_MX_MID=1 bash $S 400 $o/tests.log python -u -m pytest tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_loss_fusion_gpu.py tests/test_e2e_gpu.py -x -q --timeout 240 --timeout-method thread &&
THZ_MX_MID=1 bash $S 300 $o/donn_mid.log rocprofv3 --kernel-trace --stats -d $o/donn_mid -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
bash $S 300 $o/donn_def.log rocprofv3 --kernel-trace --stats -d $o/donn_def -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
THZ_MX_MID=1 bash $S 300 $o/full_mid.log python bench.py --no-cpu-baseline --no-shares &&
bash $S 300 $o/full_def.log python bench.py --no-cpu-baseline --no-shares
