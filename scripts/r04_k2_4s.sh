#!/bin/bash
# A/B of the four-step K2 (asm_cols_4s, default) against the three-stage asm_cols (THZ_K2_4S=0)
# on the cfg2 headline, the CZT columns-pass rewrite (parity tests + the full bench line's cfg3),
# and the QAT quality runs.
set -o pipefail
o=gpurun_out/k24s
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
THZ_K2_4S=1 bash $S 200 $o/bench_4s_a.log python $B &&
THZ_K2_4S=0 bash $S 200 $o/bench_3s_a.log python $B &&
THZ_K3_4S=1 bash $S 200 $o/bench_k3_4s_a.log python $B &&
bash $S 600 $o/tests.log python -u -m pytest tests/test_asm_gpu.py tests/test_czt_gpu.py tests/test_loss_fusion_gpu.py tests/test_donn_train_gpu.py tests/test_optics_qat_gpu.py tests/test_e2e_gpu.py tests/test_doe_gpu.py tests/test_collective_capture_gpu.py -x -q --timeout 240 --timeout-method thread &&
THZ_K2_4S=2 bash $S 200 $o/bench_4s2_a.log python $B &&
THZ_K2_4S=1 bash $S 200 $o/bench_4s_b.log python $B &&
THZ_K2_4S=0 bash $S 200 $o/bench_3s_b.log python $B &&
THZ_K2_4S=2 bash $S 200 $o/bench_4s2_b.log python $B &&
THZ_K3_4S=1 bash $S 200 $o/bench_k3_4s_b.log python $B &&
bash $S 400 $o/bench_full.log python bench.py --no-cpu-baseline &&
bash $S 400 $o/qat_quality.log python -u scripts/qat_quality.py --seeds 5 --out $o/qat_quality.json
