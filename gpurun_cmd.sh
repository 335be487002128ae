set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof.log 2>&1 &&
THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn_base -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof_base.log 2>&1
