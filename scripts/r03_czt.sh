#!/bin/bash
# cfg3 CZT: parity tests, timing, kernel trace and the LDS / traffic counters (one PMC pass each).
# usage: scripts/r03_czt.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/czt}
export TMPDIR=/tmp
mkdir -p "$out"
S=scripts/gpu_step.sh
bash $S 400 $out/tests.log python -u -m pytest tests -x -q -m gpu -k "czt" --timeout 240 --timeout-method thread &&
bash $S 200 $out/time.log python3 scripts/czt_prof.py 20 &&
bash $S 200 $out/trace.log rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 scripts/czt_prof.py 5 &&
bash $S 120 $out/pmc_lds.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAVES -d $out/pmc_lds -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $out/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $out/pmc_write.log rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run --output-format csv -- python3 scripts/czt_prof.py 3
