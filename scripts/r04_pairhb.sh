#!/bin/bash
# A/B: the three-stage paired K2 with per-half barriers (THZ_K2_PAIR=2) vs the paired (1) and the
# default one-column kernel, cfg2 headline; its U writes; the pair parity test.
set -o pipefail
o=gpurun_out/pairhb
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
bash $S 300 $o/tests.log python -u -m pytest tests/test_asm_gpu.py -x -q -k "paired_column" --timeout 240 --timeout-method thread &&
THZ_K2_PAIR=2 bash $S 200 $o/hb_a.log python $B &&
THZ_K2_PAIR=1 bash $S 200 $o/pair_a.log python $B &&
bash $S 200 $o/def_a.log python $B &&
THZ_K2_PAIR=2 bash $S 200 $o/hb_b.log python $B &&
THZ_K2_PAIR=1 bash $S 200 $o/pair_b.log python $B &&
bash $S 200 $o/def_b.log python $B &&
THZ_K2_PAIR=2 bash $S 120 $o/wr_hb.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_hb -o run --output-format csv -- python3 $P &&
bash $S 1000 $o/gpu_tests.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider &&
bash $S 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
