#!/bin/bash
# CZT kernel counters (one PMC pass per group) on the cfg3 workload.
set -u
out=${1:-gpurun_out/czt_pmc}
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d "$out/g$i" -o run --output-format csv -- python3 scripts/czt_prof.py 3 > "$out/g$i.log" 2>&1 || { echo "group $i failed"; tail -5 "$out/g$i.log"; exit 1; }
done
echo "profile done"
