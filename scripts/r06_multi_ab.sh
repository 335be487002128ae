#!/bin/bash
# Round-6 A/B over N environments on one box (cfg2 headline only), two interleaved passes.
# usage: scripts/r06_multi_ab.sh <tag> "<env 1>" "<env 2>" ...   (an env may be "X=0")
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
OUT=gpurun_out/$TAG
mkdir -p $OUT
for pass in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 240 python -u bench.py --headline-only --no-cpu-baseline --steps 20 --warmup 3 \
      > $OUT/bench_v${i}_p$pass.json 2> $OUT/bench_v${i}_p$pass.err || { echo "FAILED: $E"; exit 1; }
    python - $OUT/bench_v${i}_p$pass.json "$E" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], {n: round(v["avg_ms"], 3) for n, v in d["kernels"].items()}, d["output_check"]["ok"], flush=True)
PY
  done
done
