#!/bin/bash
# Wave-state breakdown of the bench kernels (one PMC pass per counter group).
set -u
out=${1:-gpurun_out/sq}; shift || true
export TMPDIR=/tmp
mkdir -p "$out"
B=${PROG:-"bench.py --steps 1 --warmup 1 --no-cpu-baseline --headline-only $*"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$out/g$i" -o run --output-format csv -- python3 $B > "$out/g$i.log" 2>&1 || { echo "group $i failed"; tail -5 "$out/g$i.log"; exit 1; }
done
echo "profile done"
