#!/bin/bash
# GPU test subset: python -u -m pytest on the given paths (default: the whole -m gpu suite).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 900 gpurun_out/tests_sub.log python -u -m pytest ${@:-tests} -x -v -m gpu --timeout 240 --timeout-method thread
