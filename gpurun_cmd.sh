set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/quantizationawarethzdoe_amd
THZDOE_LIB=$L/libthzdoe_v2.so bash scripts/gpu_step.sh 600 gpurun_out/gpu_tests_v2.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "p300 or donn or rsc or asm" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof.log 2>&1 &&
THZDOE_LIB=$L/libthzdoe_v2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn_v2 -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof_v2.log 2>&1 &&
THZDOE_LIB=$L/libthzdoe_v3.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn_v3 -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof_v3.log 2>&1
