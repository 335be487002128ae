set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/quantizationawarethzdoe_amd
bash scripts/gpu_step.sh 900 gpurun_out/gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof.log 2>&1 &&
THZDOE_LIB=$L/libthzdoe_v2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn_v2 -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof_v2.log 2>&1
