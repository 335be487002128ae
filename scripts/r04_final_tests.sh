#!/bin/bash
# Round-4 close, part 1: the whole -m gpu suite and smoke() on the shipped defaults.
set -o pipefail
o=gpurun_out/r04t
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 1000 $o/gpu_tests.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider &&
bash $S 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
