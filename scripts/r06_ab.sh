#!/bin/bash
# Round-6 A/B on one box: the same library under two environments (e.g. THZ_K2_RECURRENCE=0 vs 1),
# cfg2 headline only, interleaved pairs; optional GPU tests first.
# usage: scripts/r06_ab.sh <tag> "<env a>" "<env b>" [pytest targets]
set -o pipefail
TAG=$1; ENVA=$2; ENVB=$3; TESTS=$4
cd "$(dirname "$0")/.."
OUT=gpurun_out/$TAG
mkdir -p $OUT
summary() {
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(os.path.basename(f), "no line", e); continue
    k = d["kernels"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: round(v["avg_ms"], 3) for n, v in k.items()},
          d["output_check"]["ok"], d["output_check"].get("planes", [{}])[0] if isinstance(d["output_check"].get("planes"), list) else "")
PY
}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $OUT/tests.log 2>&1
  rc=$?
  tail -5 $OUT/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  env $ENVA timeout -k 10 240 python -u bench.py --headline-only --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_a$i.json 2> $OUT/bench_a$i.err &&
  env $ENVB timeout -k 10 240 python -u bench.py --headline-only --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_b$i.json 2> $OUT/bench_b$i.err || { summary; exit 1; }
done
summary
