#!/bin/bash
# The level-parallel Gumbel quantizer forward: quantizer / layer / trainer tests, then step timings.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/qlv
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_doe_gpu.py \
  tests/test_doe_fused_bwd_gpu.py tests/test_device_rng_gpu.py tests/test_optics_qat_gpu.py tests/test_qat_multi_gpu.py \
  tests/test_e2e_gpu.py tests/test_properties_gpu.py tests/test_qat_quality_gpu.py tests/test_integration_doc_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/host_probe.py 300 2>&1 | grep "us/step" | tee $O/probe.log
for w in dual edof; do timeout -k 10 120 python3 -u scripts/small_prof.py $w 300 2>/dev/null | grep "ms per step" | tee -a $O/probe.log || exit $?; done
