set -u
# parity subset + headline bench of the current build; $2 = extra env assignment for a B run
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -x -m gpu -k "${1:-asm or rsc}" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for rep in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/ab_$rep.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab_$rep.log; exit 1; }
python - gpurun_out/ab_$rep.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('A', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
PY
if [ -n "${2:-}" ]; then
env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/abB_$rep.log 2>&1 || { echo "bench B failed"; exit 1; }
python - gpurun_out/abB_$rep.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('B', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
PY
fi
done
