#!/bin/bash
# A/B of the four-step K2 (asm_cols_4s, default) against the three-stage asm_cols (THZ_K2_4S=0)
# on the cfg2 headline: ASM parity tests with the four-step kernel, then alternating bench lines.
set -o pipefail
o=gpurun_out/k24s
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
bash $S 400 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q --timeout 240 --timeout-method thread -k "four_step or cfg2 or full_size or paired" &&
THZ_K2_4S=1 bash $S 200 $o/bench_4s_a.log python $B &&
THZ_K2_4S=0 bash $S 200 $o/bench_3s_a.log python $B &&
THZ_K2_4S=1 bash $S 200 $o/bench_4s_b.log python $B &&
THZ_K2_4S=0 bash $S 200 $o/bench_3s_b.log python $B
[ $? -eq 0 ] && bash $S 400 $o/qat_quality.log python -u scripts/qat_quality.py --seeds 5 --out $o/qat_quality.json
