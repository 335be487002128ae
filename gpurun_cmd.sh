set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh 400 gpurun_out/donn_tests.log python -u -m pytest tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py -x -v --timeout 120 --timeout-method thread &&
tail -3 gpurun_out/donn_tests.log &&
bash scripts/gpu_step.sh 400 gpurun_out/bench_sec.log python bench.py --no-cpu-baseline &&
tail -2 gpurun_out/bench_sec.log
