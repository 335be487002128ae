#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dgprof -o d --output-format csv -- python3 scripts/donn_graph_prof.py 20 > gpurun_out/dgprof.log 2>&1
