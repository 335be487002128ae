#!/bin/bash
# Round-4 evidence: cfg2 kernel trace + PMC passes (profiles/r04_*), cfg3 CZT trace + PMC, cfg5 DONN
# kernel trace.  Each GPU step under its own time limit, chained with && (scripts/gpu_step.sh).
set -o pipefail
export TMPDIR=/tmp
S=scripts/gpu_step.sh
mkdir -p gpurun_out/r04ev
bash $S 1100 gpurun_out/r04ev/prof.log bash scripts/profile_asm.sh gpurun_out/r04ev/prof &&
bash $S 600 gpurun_out/r04ev/czt.log bash scripts/r03_czt.sh gpurun_out/r04ev/czt &&
bash $S 300 gpurun_out/r04ev/donn.log rocprofv3 --kernel-trace --stats -d gpurun_out/r04ev/donn -o run --output-format csv -- python3 scripts/donn_prof.py 20
