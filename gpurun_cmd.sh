set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 gpurun_out/gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
tail -1 gpurun_out/gpu_tests.log && REPS=3 bash scripts/exp_multi.sh default base
