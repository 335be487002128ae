#!/bin/bash
# Run one GPU step under its own time limit; stop the whole script on a crash-like exit.
# usage: gpu_step.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" | tee -a "$log"
case $rc in
  124|137|134|139|132|135) echo "[gpu_step] crash/timeout -- stopping"; exit $rc;;
esac
exit 0
