#!/bin/bash
# CZT rows pass with the mirrored RS factors shared: parity tests, cfg3 timing (3 runs), kernel trace.
set -o pipefail
o=gpurun_out/cztm
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 400 $o/tests.log python -u -m pytest tests -x -q -m gpu -k "czt or CZT" --timeout 240 --timeout-method thread &&
bash $S 120 $o/time1.log python3 scripts/czt_prof.py 20 &&
bash $S 120 $o/time2.log python3 scripts/czt_prof.py 20 &&
bash $S 120 $o/time3.log python3 scripts/czt_prof.py 20 &&
bash $S 200 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python3 scripts/czt_prof.py 5
