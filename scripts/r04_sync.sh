#!/bin/bash
# A/B of the K2 sibling pacing (THZ_K2_SYNC=1: the 4 column workgroups of a U block kept within
# one plane of each other so the L2 merges their sector writes) against the default, cfg2 headline;
# U write traffic of the paced kernel; the ASM parity tests with pacing on.
set -o pipefail
o=gpurun_out/sync
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 200 $o/def_a.log python $B &&
THZ_K2_SYNC=1 bash $S 200 $o/sync_a.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_SYNC=1 bash $S 200 $o/sync_b.log python $B &&
THZ_K2_SYNC=1 bash $S 120 $o/wr_sync.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_sync -o run --output-format csv -- python3 $P &&
bash $S 120 $o/wr_def.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_def -o run --output-format csv -- python3 $P &&
THZ_K2_SYNC=1 bash $S 400 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q --timeout 240 --timeout-method thread
