#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/qgprof -o q --output-format csv -- python3 scripts/qat_graph_prof.py 100 > gpurun_out/qgprof.log 2>&1
