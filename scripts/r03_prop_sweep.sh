#!/bin/bash
# A wide, randomly seeded hypothesis sweep of the GPU property tests (THZ_PROP_EXAMPLES draws per
# test), then the round-3 GPU check.  A failing sweep (rc 1) still runs the check; a time limit,
# abort or crash (any other non-zero rc) ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03s}; n=${2:-300}
THZ_PROP_EXAMPLES=$n THZ_PROP_RANDOM=1 bash scripts/gpu_step.sh 900 gpurun_out/${tag}_sweep.log \
  python -u -m pytest tests/test_properties_gpu.py -x -v -m gpu --timeout 600 --timeout-method thread
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/r03_gpu.sh $tag
