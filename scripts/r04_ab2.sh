#!/bin/bash
# Round-4 A/B batch 2: QAT quality after the Exp(1) fix (v3, naive Gumbel), cfg5 with and without
# the 3 x 100 passes (THZ_K2_M3), the paired four-step K2, and SQ counters of the two K2 kernels.
set -o pipefail
o=gpurun_out/ab2
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
P="bench.py --steps 2 --warmup 1 --no-cpu-baseline --headline-only"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
bash $S 300 $o/qat.log python -u scripts/qat_quality.py --seeds 5 --methods Ours,GS --out $o/qat_quality.json &&
THZ_K2_M3=1 bash $S 300 $o/donn_m3.log rocprofv3 --kernel-trace --stats -d $o/donn_m3 -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
THZ_K2_M3=0 bash $S 300 $o/donn_mx.log rocprofv3 --kernel-trace --stats -d $o/donn_mx -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
THZ_K2_M3=1 THZ_K2_4S=0 bash $S 300 $o/full_m3.log python bench.py --no-cpu-baseline --no-shares &&
THZ_K2_M3=0 THZ_K2_4S=0 bash $S 300 $o/full_mx.log python bench.py --no-cpu-baseline --no-shares &&
THZ_K2_4S=2 bash $S 200 $o/bench_4s2.log python $B &&
THZ_K2_4S=0 bash $S 200 $o/bench_3s.log python $B &&
THZ_K2_4S=1 bash $S 120 $o/sq1_4s.log rocprofv3 --pmc $SQ1 -d $o/sq1_4s -o run --output-format csv -- python3 $P &&
THZ_K2_4S=1 bash $S 120 $o/sq2_4s.log rocprofv3 --pmc $SQ2 -d $o/sq2_4s -o run --output-format csv -- python3 $P &&
THZ_K2_4S=0 bash $S 120 $o/sq1_3s.log rocprofv3 --pmc $SQ1 -d $o/sq1_3s -o run --output-format csv -- python3 $P &&
THZ_K2_4S=0 bash $S 120 $o/sq2_3s.log rocprofv3 --pmc $SQ2 -d $o/sq2_3s -o run --output-format csv -- python3 $P &&
THZ_K2_4S=2 bash $S 120 $o/wr_4s2.log rocprofv3 --pmc WRITE_SIZE -d $o/wr_4s2 -o run --output-format csv -- python3 $P
