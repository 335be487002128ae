#!/bin/bash
# A/B: paired four-step K2 with both barriers per half except every 2nd plane (THZ_K2_4S=4) vs the
# barrier-A-only form (3) and the default, cfg2 headline; U writes of (4).
set -o pipefail
o=gpurun_out/hb2
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 300 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q -k "four_step_k2" --timeout 240 --timeout-method thread &&
THZ_K2_4S=4 bash $S 200 $o/hb2_a.log python $B &&
THZ_K2_4S=3 bash $S 200 $o/hb_a.log python $B &&
bash $S 200 $o/def_a.log python $B &&
THZ_K2_4S=4 bash $S 200 $o/hb2_b.log python $B &&
THZ_K2_4S=3 bash $S 200 $o/hb_b.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_4S=4 bash $S 120 $o/wr_hb2.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_hb2 -o run --output-format csv -- python3 $P
