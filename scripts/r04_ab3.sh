#!/bin/bash
# Round-4 batch 3: LDS residency probe (workgroups per CU at the four-step K2's LDS size), the GPU
# tests touched by the default switches, and the cfg5 step with the 3 x 100 passes + aperture fold.
set -o pipefail
o=gpurun_out/ab3
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
R=scripts/diag/lds_residency
bash $S 60 $o/res.log bash -c "$R 0 512 && $R 65536 512 && $R 74248 512 && $R 78848 512 && $R 80000 512 && $R 81920 512 && $R 148992 1024" &&
bash $S 600 $o/tests.log python -u -m pytest tests/test_asm_gpu.py tests/test_donn_train_gpu.py tests/test_collective_capture_gpu.py tests/test_qat_quality_gpu.py -x -q --timeout 240 --timeout-method thread &&
bash $S 300 $o/full_def.log python bench.py --no-cpu-baseline --no-shares &&
THZ_K2_M3=1 bash $S 300 $o/full_m3.log python bench.py --no-cpu-baseline --no-shares
