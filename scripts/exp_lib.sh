set -u
# A/B of the default library against quantizationawarethzdoe_amd/libthzdoe_exp$1.so: parity subset
# with the default library, then the full bench line (no CPU baseline) of both, twice
mkdir -p gpurun_out
L=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp$1.so
timeout -k 10 400 python -m pytest tests -q -x -m gpu -k "${2:-asm or czt}" > gpurun_out/lib_tests.log 2>&1 || { echo "default-lib tests failed"; tail -30 gpurun_out/lib_tests.log; exit 1; }
tail -1 gpurun_out/lib_tests.log
for rep in 1 2; do
for v in A B; do
if [ $v = A ]; then unset THZDOE_LIB; else export THZDOE_LIB=$L; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/lib_$v$rep.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/lib_$v$rep.log; exit 1; }
python - gpurun_out/lib_$v$rep.log $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
s=d.get('secondary',{})
print(sys.argv[2], d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, 'czt', s.get('cfg3_czt',{}).get('ms_per_call'), 'qat', {k:v['ms_per_it'] for k,v in s.get('cfg4_qat',{}).get('phases',{}).items()}, 'donn', {k:v['ms_per_step'] for k,v in s.get('cfg5_donn',{}).get('modes',{}).items()})
PY
done; done
unset THZDOE_LIB
