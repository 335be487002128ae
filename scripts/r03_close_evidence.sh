#!/bin/bash
# Round-3 close evidence (after the K3 / K1 table-load change): N = 2 rehearsal on one GPU (gloo), cfg2 rocprofv3 kernel trace + PMC passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r02_rehearse_n2.sh &&
bash scripts/gpu_step.sh 1100 gpurun_out/r03f_prof.log bash scripts/profile_asm.sh gpurun_out/r03f_prof
