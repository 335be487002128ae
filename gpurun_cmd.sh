set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh 600 gpurun_out/gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
tail -2 gpurun_out/gpu_tests.log &&
bash scripts/gpu_step.sh 600 gpurun_out/bench.log python bench.py &&
tail -1 gpurun_out/bench.log | cut -c1-300 &&
bash scripts/profile_asm.sh gpurun_out/prof_r01 &&
REPS=2 bash scripts/exp_multi.sh default base
