#!/bin/bash
# Round-6 close-out on one box, in two parts (each its own gpurun call):
#   A: the whole -m gpu suite, smoke(), the default bench line
#   B: the bench's rocprofv3 kernel trace + PMC passes (cfg2), the cfg3 CZT trace + PMC passes, kernel
#      traces of the small graph-replayed steps, and the 6,000-iteration QAT quality runs
#   C: the cfg3 CZT trace + PMC passes only
# usage: scripts/r06_close.sh A|B|C <tag>
set -o pipefail
cd "$(dirname "$0")/.."
PART=$1; O=gpurun_out/${2:-r06close}
mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" = A ]; then
  timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -2 $O/smoke.log
  timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
  tail -c 400 $O/bench.json
else
  [ "$PART" = C ] || bash scripts/profile_asm.sh $O/prof || exit $?
  mkdir -p $O/czt
  C="python3 scripts/czt_prof.py 10"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/czt/trace -o run --output-format csv -- $C > $O/czt/trace.log 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/czt/pmc_fetch -o run --output-format csv -- $C > $O/czt/fetch.log 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/czt/pmc_write -o run --output-format csv -- $C > $O/czt/write.log 2>&1 || exit $?
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/czt/pmc_sq -o run --output-format csv -- $C > $O/czt/sq.log 2>&1 || exit $?
  [ "$PART" = C ] && exit 0
  bash scripts/r05_small_traces.sh $O/small donn32 donn256 qat dual edof || exit $?
  for s in four_focal dual edof; do
    timeout -k 10 400 python3 -u scripts/qat_quality.py --system $s --seeds 3 --out $O/qat_quality_$s.json > $O/qat_quality_$s.log 2>&1 || exit $?
    tail -5 $O/qat_quality_$s.log
  done
fi
