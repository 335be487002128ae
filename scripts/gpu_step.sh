#!/bin/bash
# Run one GPU step under its own time limit and pass its exit status on, so a `&&` chain
# stops at the first failing step (a red test suite included).
# usage: gpu_step.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" | tee -a "$log"
exit $rc
