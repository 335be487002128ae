#!/bin/bash
# headline bench at z_chunk 32 (default) vs 64, interleaved twice
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for zc in 32 64; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 --z-chunk $zc > gpurun_out/zc_$zc.$rep.log 2>&1 || { tail -20 gpurun_out/zc_$zc.$rep.log; exit 1; }
  python - gpurun_out/zc_$zc.$rep.log $zc <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})
PY
done; done
