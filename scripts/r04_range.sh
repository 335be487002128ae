#!/bin/bash
# A/B of K2 with and without the restated thread-index range (THZ_K2_RANGE=0: the round-3 code
# path, 1316 vs 1241 VALU per thread per plane) and the middle-crop K2 (THZ_K2_MID=1), cfg2 headline.
set -o pipefail
o=gpurun_out/range
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
bash $S 200 $o/def_a.log python $B &&
THZ_K2_RANGE=0 bash $S 200 $o/nor_a.log python $B &&
THZ_K2_MID=1 bash $S 200 $o/mid_a.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_RANGE=0 bash $S 200 $o/nor_b.log python $B &&
THZ_K2_MID=1 bash $S 200 $o/mid_b.log python $B
