#!/bin/bash
# GPU iteration loop: ASM/CZT/RSC parity tests, then the bench without the CPU baseline.
# usage: scripts/quick_check.sh <tag> [pytest -k expr]
set -u
tag=${1:-q}; k=${2:-}
mkdir -p gpurun_out
if [ -n "$k" ]; then
  bash scripts/gpu_step.sh 400 gpurun_out/${tag}_tests.log python -m pytest tests -q -x -m gpu -k "$k" || exit $?
else
  bash scripts/gpu_step.sh 400 gpurun_out/${tag}_tests.log python -m pytest tests -q -x -m gpu || exit $?
fi
grep -q " passed" gpurun_out/${tag}_tests.log && ! grep -q " failed" gpurun_out/${tag}_tests.log || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
bash scripts/gpu_step.sh 300 gpurun_out/${tag}_bench.log python bench.py --no-cpu-baseline
