#!/bin/bash
# CZT overlap-add check: parity tests, cfg3 timing, kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 600 gpurun_out/czt_tests.log python -u -m pytest tests/test_czt_gpu.py tests/test_abi.py -x -v -m gpu --timeout 240 --timeout-method thread &&
bash $S 200 gpurun_out/czt_time.log python scripts/czt_prof.py 20 &&
bash $S 300 gpurun_out/czt_trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/czt_prof -o run --output-format csv -- python3 scripts/czt_prof.py 10 &&
bash $S 600 gpurun_out/czt_pmc.log bash scripts/r02_czt_pmc.sh gpurun_out/czt_pmc
