#!/bin/bash
# Round-2 close: -m gpu suite, smoke, bench line, rocprofv3 trace + PMC passes, then the
# cpu_baseline over all 64 planes of the cfg2 sweep (host cores of the GPU box)
set -o pipefail
bash scripts/r02_gpu_run.sh &&
timeout -k 10 600 python bench.py --cpu-only --cpu-planes 64 --cpu-budget 1e9 > gpurun_out/cpu64.json 2> gpurun_out/cpu64.log
