#!/bin/bash
# Round-4 last check on the shipped defaults: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
o=gpurun_out/final2
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 1000 $o/gpu_tests.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider &&
bash $S 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
bash $S 400 $o/bench.log python bench.py
