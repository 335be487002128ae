#!/bin/bash
# Randomized property sweep only (THZ_PROP_EXAMPLES draws per test) plus an optional pytest -k
# selection of the regular GPU tests.  usage: scripts/r03_sweep_only.sh <tag> <n> [k-expr]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03w}; n=${2:-400}; kexpr=${3:-}
THZ_PROP_EXAMPLES=$n THZ_PROP_RANDOM=1 bash scripts/gpu_step.sh 1000 gpurun_out/${tag}_sweep.log \
  python -u -m pytest tests/test_properties_gpu.py -v -m gpu --hypothesis-show-statistics --timeout 900 --timeout-method thread
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$kexpr" ]; then
  bash scripts/gpu_step.sh 300 gpurun_out/${tag}_k.log python -u -m pytest tests -x -v -m gpu -k "$kexpr" \
    --timeout 240 --timeout-method thread
fi
