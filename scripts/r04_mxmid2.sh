#!/bin/bash
# A/B of the 300-point row passes with window constants (THZ_MX_MID=1: K1, K2, K3) against the
# column pass alone (2) and none (0): P = 300 parity tests, DONN traces, bench lines (cfg4 / cfg5).
set -o pipefail
o=gpurun_out/mxmid2
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 400 $o/tests.log python -u -m pytest tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_loss_fusion_gpu.py tests/test_e2e_gpu.py tests/test_doe_gpu.py -x -q --timeout 240 --timeout-method thread &&
bash $S 300 $o/donn_1.log rocprofv3 --kernel-trace --stats -d $o/donn_1 -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
THZ_MX_MID=2 bash $S 300 $o/donn_2.log rocprofv3 --kernel-trace --stats -d $o/donn_2 -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
bash $S 300 $o/full_1.log python bench.py --no-cpu-baseline --no-shares &&
THZ_MX_MID=2 bash $S 300 $o/full_2.log python bench.py --no-cpu-baseline --no-shares &&
bash $S 300 $o/full_1b.log python bench.py --no-cpu-baseline --no-shares &&
THZ_MX_MID=2 bash $S 300 $o/full_2b.log python bench.py --no-cpu-baseline --no-shares
