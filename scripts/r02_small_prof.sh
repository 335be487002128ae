#!/bin/bash
# kernel traces of the eager cfg4 QAT step and cfg5 DONN step (per-kernel durations)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o q -- python3 scripts/qat_prof.py > gpurun_out/qprof.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o d -- python3 scripts/donn_prof.py 5 > gpurun_out/dprof.log 2>&1
