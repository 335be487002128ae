#!/bin/bash
# parity subset with the default library, then bench A (default) vs B (libthzdoe_exp1.so), twice
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread -k "${1:-asm or czt or rsc}" > gpurun_out/abf_tests.log 2>&1 || { tail -30 gpurun_out/abf_tests.log; exit 1; }
tail -1 gpurun_out/abf_tests.log
bash scripts/exp_lib.sh 1
