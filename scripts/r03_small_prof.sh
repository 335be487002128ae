#!/bin/bash
# cfg5 DONN (batch 256) and cfg4 QAT kernel traces: which kernels the small-grid steps spend on.
set -o pipefail
mkdir -p gpurun_out/small
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/small/donn -o run --output-format csv -- python3 scripts/donn_prof.py 10 > gpurun_out/small/donn.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/small/qat -o run --output-format csv -- python3 scripts/qat_prof.py > gpurun_out/small/qat.log 2>&1
