set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 900 gpurun_out/gpu_tests_all.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
bash scripts/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
bash scripts/gpu_step.sh 400 gpurun_out/bench_final.log python bench.py
