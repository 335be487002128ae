#!/bin/bash
# CZT cfg3 timing (scripts/czt_prof.py, 30 calls) over several library builds, two interleaved passes,
# then the CZT tests on the first experimental build.
# usage: scripts/czt_multi_ab.sh <tag> <lib_1.so> [lib_2.so ...]   ("-" = the shipped library)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/$1; shift
mkdir -p $O
for i in 1 2; do
  for L in "$@"; do
    if [ "$L" = "-" ]; then unset THZDOE_LIB; else export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/$L; fi
    timeout -k 10 120 python3 -u scripts/czt_prof.py 30 2>/dev/null | sed "s/^/$L p$i /" || exit $?
  done
done 2>&1 | tee $O/ab.log || exit $?
unset THZDOE_LIB
for L in "$@"; do
  [ "$L" = "-" ] && continue
  THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/$L timeout -k 10 400 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_czt_gpu.py > $O/tests_$L.log 2>&1
  echo "$L: $(tail -1 $O/tests_$L.log)"
done
