#!/bin/bash
# A/B of the paired four-step K2 with per-half barriers (THZ_K2_4S=3: one workgroup barrier per
# plane instead of two, the other half runs on) against the paired (2) and default (0) kernels.
set -o pipefail
o=gpurun_out/hb
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 300 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q -k "four_step_k2" --timeout 240 --timeout-method thread &&
THZ_K2_4S=3 bash $S 200 $o/hb_a.log python $B &&
THZ_K2_4S=2 bash $S 200 $o/pair_a.log python $B &&
bash $S 200 $o/def_a.log python $B &&
THZ_K2_4S=3 bash $S 200 $o/hb_b.log python $B &&
THZ_K2_4S=2 bash $S 200 $o/pair_b.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_4S=3 bash $S 120 $o/wr_hb.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_hb -o run --output-format csv -- python3 $P
