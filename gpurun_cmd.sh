set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 300 gpurun_out/gpu_tests_czt.log python -u -m pytest tests/test_czt_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_czt2 -o run --output-format csv -- python3 scripts/czt_prof.py 5 > gpurun_out/czt_prof2.log 2>&1
