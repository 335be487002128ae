#!/bin/bash
# SQ counters of the eager cfg5 DONN step (per-kernel), two passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/dpmc1 -o run --output-format csv -- python3 scripts/donn_prof.py 3 > gpurun_out/dpmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM -d gpurun_out/dpmc2 -o run --output-format csv -- python3 scripts/donn_prof.py 3 > gpurun_out/dpmc2.log 2>&1
