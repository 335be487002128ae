set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 900 gpurun_out/gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
