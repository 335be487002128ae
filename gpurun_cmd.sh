set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_step.sh 600 gpurun_out/gpu_tests.log python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
tail -2 gpurun_out/gpu_tests.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_donn -o run --output-format csv -- python3 scripts/donn_prof.py 5 > gpurun_out/donn_prof.log 2>&1 &&
bash scripts/gpu_step.sh 300 gpurun_out/bench_sec.log python bench.py --no-cpu-baseline &&
tail -1 gpurun_out/bench_sec.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['secondary']['cfg4_qat']['phases']), json.dumps(d['secondary']['cfg5_donn']['modes']))"
