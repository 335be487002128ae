#!/bin/bash
# optics / DOE parity subset, then bench_aux.py with the default library (A) and libthzdoe_exp1.so (B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread -k "optics or doe or donn or dropin or loss_fusion" > gpurun_out/aux_tests.log 2>&1 || { tail -30 gpurun_out/aux_tests.log; exit 1; }
tail -1 gpurun_out/aux_tests.log
timeout -k 10 300 python scripts/bench_aux.py > gpurun_out/auxA.json 2>&1 &&
THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp1.so timeout -k 10 300 python scripts/bench_aux.py > gpurun_out/auxB.json 2>&1 &&
grep kernel gpurun_out/auxA.json | sed 's/^/A /' && grep kernel gpurun_out/auxB.json | sed 's/^/B /'
