#!/bin/bash
# Round-5 A/B on one box: the shipped library vs an experimental build (THZDOE_LIB), cfg2 headline
# only, interleaved pairs; then the GPU tests on the shipped library and the ASM tests on the other.
# usage: scripts/r05_ab.sh <tag> <lib_b.so> [tests]
set -o pipefail
TAG=$1; LIBB=$2; TESTS=${3:-tests/test_asm_gpu.py}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$(dirname "$0")/.."
B=quantizationawarethzdoe_amd/$LIBB
summary() {
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(os.path.basename(f), "no line", e); continue
    k = d["kernels"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: round(v["avg_ms"], 3) for n, v in k.items()}, d["output_check"]["ok"])
PY
}
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --headline-only --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_a$i.json 2> $OUT/bench_a$i.err &&
  THZDOE_LIB=$PWD/$B timeout -k 10 240 python -u bench.py --headline-only --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_b$i.json 2> $OUT/bench_b$i.err || { summary; exit 1; }
done
summary
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests_a.log 2>&1
ra=$?
tail -3 $OUT/tests_a.log
[ $ra -eq 0 ] || [ $ra -eq 1 ] || exit $ra
THZDOE_LIB=$PWD/$B timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_asm_gpu.py > $OUT/tests_b.log 2>&1
tail -3 $OUT/tests_b.log
