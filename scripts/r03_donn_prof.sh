#!/bin/bash
# cfg5 DONN step kernel trace (20 eager chained steps, batch 256) -> profiles/r03_donn_kernel_stats.csv
export TMPDIR=/tmp
mkdir -p gpurun_out/donnprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/donnprof/trace -o run --output-format csv -- python3 scripts/donn_prof.py 20 > gpurun_out/donnprof/trace.log 2>&1
