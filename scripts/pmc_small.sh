#!/bin/bash
# PMC passes (one counter group per run) over the graph-replayed small steps of scripts/small_prof.py
# usage: scripts/pmc_small.sh <outdir> <workload>
set -u
out=$1; w=$2
export TMPDIR=/tmp
mkdir -p "$out"
P="python3 scripts/small_prof.py $w 20"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU -d "$out/sq" -o run --output-format csv -- $P > "$out/sq.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$out/sq2" -o run --output-format csv -- $P > "$out/sq2.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- $P > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- $P > "$out/write.log" 2>&1 || exit $?
echo "pmc done"
