#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes for the bench workload (run on the GPU box).
# usage: scripts/profile_asm.sh <outdir> [extra bench args]
set -u
out=${1:-gpurun_out/prof}; shift || true
export TMPDIR=/tmp
mkdir -p "$out"
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only $*"
# the trace pass runs the bench's own default step counts so its averages match bench.py's
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --headline-only $* > "$out/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 $B > "$out/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 $B > "$out/write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$out/sq" -o run --output-format csv -- python3 $B > "$out/sq.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM -d "$out/sq2" -o run --output-format csv -- python3 $B > "$out/sq2.log" 2>&1 || exit $?
echo "profile done"
