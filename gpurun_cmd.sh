set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh 240 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
bash scripts/gpu_step.sh 600 gpurun_out/gpu_tests.log python -m pytest tests -q -m gpu &&
bash scripts/gpu_step.sh 300 gpurun_out/bench.log python bench.py &&
bash scripts/profile_asm.sh gpurun_out/prof_r1b
