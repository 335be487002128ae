set -u
# parity subset + headline bench (2 reps) of the current build
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -x -m gpu -k "${1:-asm or rsc}" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for rep in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/ab_$rep.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab_$rep.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"achieved": [0-9.]*' gpurun_out/ab_$rep.log | tr '\n' ' '; echo
done
