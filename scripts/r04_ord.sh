#!/bin/bash
# A/B of the K2 store order (THZ_K2_ORD=1: ascending rows) against the default, cfg2 headline, and
# its U writes.
set -o pipefail
o=gpurun_out/ord
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 300 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q -k "store_order" --timeout 240 --timeout-method thread &&
THZ_K2_ORD=1 bash $S 200 $o/ord_a.log python $B &&
bash $S 200 $o/def_a.log python $B &&
THZ_K2_ORD=1 bash $S 200 $o/ord_b.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_ORD=1 bash $S 120 $o/wr_ord.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_ord -o run --output-format csv -- python3 $P
