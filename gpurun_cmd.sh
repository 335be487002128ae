set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 300 gpurun_out/gpu_tests_czt_def.log python -u -m pytest tests/test_czt_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread &&
THZ_CZT_MX=1 bash scripts/gpu_step.sh 300 gpurun_out/gpu_tests_czt_mx1.log python -u -m pytest tests/test_czt_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread &&
timeout -k 10 300 python3 scripts/czt_prof.py 10 > gpurun_out/czt_def.log 2>&1
