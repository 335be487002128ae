#!/bin/bash
# A/B of the CZT passes on cfg3 (scripts/czt_prof.py, 30 calls): the shipped library (a) against an
# experimental build (b, THZDOE_LIB), interleaved pairs, then the CZT tests on b.
# usage: scripts/czt_ab.sh <tag> <lib_b.so>
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/$1
B=$PWD/quantizationawarethzdoe_amd/$2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python3 -u scripts/czt_prof.py 30 2>/dev/null | sed "s/^/a$i /" || exit $?
  THZDOE_LIB=$B timeout -k 10 120 python3 -u scripts/czt_prof.py 30 2>/dev/null | sed "s/^/b$i /" || exit $?
done 2>&1 | tee $O/ab.log || exit $?
THZDOE_LIB=$B timeout -k 10 400 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_czt_gpu.py > $O/tests_b.log 2>&1
tail -3 $O/tests_b.log
