set -u
mkdir -p gpurun_out
for rep in 1 2; do
for v in 5 6; do
for skip in 0 1; do
if [ $skip = 1 ]; then export THZ_SKIP_K3=1; else unset THZ_SKIP_K3; fi
THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/k2_$v$skip.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/k2_$v$skip.log; exit 1; }
python - gpurun_out/k2_$v$skip.log "lib$v skipK3=$skip" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
PY
done; done; done
