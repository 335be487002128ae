#!/bin/bash
# A/B of a Python-side trainer change: the small graph-replayed steps (scripts/small_prof.py) from
# a snapshot of the previous package under ab_old/ (a) against the working tree (b), interleaved.
# usage: scripts/state_ab.sh <tag> [workloads...]
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/$1; shift
W=${*:-qat dual edof donn32}
mkdir -p $O
for i in 1 2; do
  for w in $W; do
    timeout -k 10 120 python3 -u ab_old/scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/a$i /" || exit $?
    timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | sed "s/^/b$i /" || exit $?
  done
done 2>&1 | tee $O/ab.log
