#!/bin/bash
# A/B of the small graph-replayed training steps (scripts/small_prof.py) on one box: the shipped
# library (a) against an experimental build (b, THZDOE_LIB), interleaved pairs a1 b1 a2 b2.
# usage: scripts/small_ab.sh <tag> <lib_b.so> [workloads...]   (default: donn32 donn256 qat dual)
# Build b with: make -C quantizationawarethzdoe_amd/csrc OUT=../libthzdoe_ab.so BUILD=build_ab DEFS=-D...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; B=$PWD/quantizationawarethzdoe_amd/$2; shift 2
W=${*:-donn32 donn256 qat dual}
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for w in $W; do
    timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
    THZDOE_LIB=$B timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/b$i /" || exit $?
  done
done 2>&1 | tee $O/ab.log
