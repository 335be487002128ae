#!/bin/bash
# A/B of the compile-time middle-crop K2 / K3 (asm_cols_mid, asm_rows_inv_mid) against the generic
# kernels on the cfg2 headline (two pairs), after their parity tests.
set -o pipefail
o=gpurun_out/mid
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
bash $S 400 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q --timeout 240 --timeout-method thread &&
bash $S 200 $o/mid_a.log python $B &&
THZ_K2_MID=0 THZ_K3_MID=0 bash $S 200 $o/gen_a.log python $B &&
bash $S 200 $o/mid_b.log python $B &&
THZ_K2_MID=0 THZ_K3_MID=0 bash $S 200 $o/gen_b.log python $B
