#!/bin/bash
# Round-4 close in one call, on the shipped defaults: (1) the whole -m gpu suite and smoke();
# (2) cfg2 kernel trace + PMC passes, cfg3 CZT trace + PMC, cfg5 DONN trace; (3) the default bench
# line with the CPU baseline leg.  Each GPU step under its own time limit (gpu_step.sh).  (The
# middle-crop A/B that first ran in this script: gpurun_out/close/ab.txt)
set -o pipefail
o=gpurun_out/close3
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
bash $S 1000 $o/gpu_tests.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider &&
bash $S 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
bash $S 900 $o/prof.log bash scripts/profile_asm.sh $o/prof &&
bash $S 200 $o/czt_trace.log rocprofv3 --kernel-trace --stats -d $o/czt/trace -o run --output-format csv -- python3 scripts/czt_prof.py 5 &&
bash $S 120 $o/czt_lds.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAVES -d $o/czt/pmc_lds -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $o/czt_fetch.log rocprofv3 --pmc FETCH_SIZE -d $o/czt/pmc_fetch -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $o/czt_write.log rocprofv3 --pmc WRITE_SIZE -d $o/czt/pmc_write -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 300 $o/donn.log rocprofv3 --kernel-trace --stats -d $o/donn -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
bash $S 400 $o/bench.log python bench.py
