#!/bin/bash
# the tests added since the last full run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "${1:-max_planes or p16384 or train_history}" > gpurun_out/newtests.log 2>&1 || { tail -40 gpurun_out/newtests.log; exit 1; }
tail -5 gpurun_out/newtests.log
