#!/bin/bash
# Round-3 GPU check: -m gpu suite (optionally a -k filter), smoke, bench line.
# usage: scripts/r03_gpu.sh <tag> [pytest -k expression]
set -o pipefail
tag=${1:-r03}; kexpr=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
if [ -n "$kexpr" ]; then K=(-k "$kexpr"); else K=(); fi
bash $S 1000 gpurun_out/${tag}_tests.log python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread "${K[@]}" &&
bash $S 200 gpurun_out/${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" &&
bash $S 500 gpurun_out/${tag}_bench.log python bench.py --steps 20 --warmup 5
