#!/bin/bash
# per-kernel graph-replay floor under runtime environments, then the DONN batch-32 step under the same
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/floor
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python3 -u scripts/launch_floor.py 102 50 > gpurun_out/floor/$tag.log 2>&1 && \
  env "$@" timeout -k 10 120 python3 -u scripts/small_prof.py donn32 300 >> gpurun_out/floor/$tag.log 2>&1; grep -v amdgpu.ids gpurun_out/floor/$tag.log | grep "us/kernel\|ms per step"; }
run default
run devkarg HIP_FORCE_DEV_KERNARG=1
run nodevkarg HIP_FORCE_DEV_KERNARG=0
run optflush0 AMD_OPT_FLUSH=0
run optflush1 AMD_OPT_FLUSH=1
run gpc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run gpc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run sysscope0 ROC_SYSTEM_SCOPE_SIGNAL=0
exit 0
