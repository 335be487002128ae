set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 600 gpurun_out/final_gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
bash scripts/gpu_step.sh 200 gpurun_out/final_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" &&
bash scripts/gpu_step.sh 300 gpurun_out/final_bench.log python bench.py
