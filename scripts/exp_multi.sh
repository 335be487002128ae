set -u
# Interleaved A/B/C... of library builds: "default" = quantizationawarethzdoe_amd/libthzdoe.so, any
# other name X = quantizationawarethzdoe_amd/libthzdoe_X.so.  Headline bench only, $REPS rounds.
# usage: bash scripts/exp_multi.sh default exp1 exp2 ...
mkdir -p gpurun_out
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
for v in "$@"; do
if [ "$v" = default ]; then unset THZDOE_LIB; else export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_$v.so; fi
timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/multi_$v$rep.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/multi_$v$rep.log; exit 1; }
python - gpurun_out/multi_$v$rep.log $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, flush=True)
PY
done; done
unset THZDOE_LIB
