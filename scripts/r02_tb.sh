#!/bin/bash
# -m gpu suite + smoke + bench line (no profiler passes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 900 gpurun_out/tests.log python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread &&
bash $S 200 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" &&
bash $S 400 gpurun_out/bench.log python bench.py --steps 20 --warmup 5
