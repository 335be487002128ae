#!/bin/bash
# Rehearse the N = 2 bench path on a one-GPU box: two ranks on cuda:0 over gloo (the driver's
# scaling runs use one GPU per rank over RCCL).  Exercises the launcher, z / lambda / batch
# sharding, barrier + max-time reduce, the output check gather and the trainers' world > 1
# all-reduce split on real kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp THZ_BENCH_SAME_DEVICE=1 THZ_BENCH_BACKEND=gloo
timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse_n2.log 2>&1
rc=$?
echo "[rehearse] rc=$rc"
tail -3 gpurun_out/rehearse_n2.log | cut -c1-600
exit $rc
