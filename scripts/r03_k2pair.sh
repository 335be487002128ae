#!/bin/bash
# A/B of the opt-in paired-column K2 (THZ_K2_PAIR=1) against the default one-column kernel
# (THZ_K2_PAIR=0) on the cfg2 headline: ASM parity tests with the pair on, then bench lines and
# WRITE_SIZE / FETCH_SIZE passes for both.
set -o pipefail
mkdir -p gpurun_out/k2pair
export TMPDIR=/tmp
S=scripts/gpu_step.sh
o=gpurun_out/k2pair
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 600 $o/tests.log python -u -m pytest tests/test_asm_gpu.py tests/test_rsc_gpu.py tests/test_e2e_gpu.py -x -q --timeout 240 --timeout-method thread &&
THZ_K2_PAIR=1 bash $S 300 $o/bench_pair.log python $B &&
THZ_K2_PAIR=0 bash $S 300 $o/bench_one.log python $B &&
THZ_K2_PAIR=1 bash $S 300 $o/write_pair.log rocprofv3 --pmc WRITE_SIZE -d $o/write_pair -o run --output-format csv -- python3 $P &&
THZ_K2_PAIR=0 bash $S 300 $o/write_one.log rocprofv3 --pmc WRITE_SIZE -d $o/write_one -o run --output-format csv -- python3 $P &&
THZ_K2_PAIR=1 bash $S 300 $o/fetch_pair.log rocprofv3 --pmc FETCH_SIZE -d $o/fetch_pair -o run --output-format csv -- python3 $P
