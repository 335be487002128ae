#!/bin/bash
# kernel trace of the eager cfg5 DONN step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof2 -o d -- python3 scripts/donn_prof.py 5 > gpurun_out/dprof2.log 2>&1
