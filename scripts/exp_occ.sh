set -u
mkdir -p gpurun_out
export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp3.so
for x in 0 20000 0 20000; do
THZ_K3_LDS_EXTRA=$x timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/occ_$x.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/occ_$x.log; exit 1; }
python - gpurun_out/occ_$x.log $x <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
PY
done
