#!/bin/bash
# parity subset + bench A/B (default vs libthzdoe_exp1.so) + one SQ LDS PMC pass of each library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread -k "${1:-asm or czt or rsc or fft or helper}" > gpurun_out/lds_tests.log 2>&1 || { tail -30 gpurun_out/lds_tests.log; exit 1; }
tail -1 gpurun_out/lds_tests.log
bash scripts/exp_lib.sh 1 || exit 1
for v in A B; do
  if [ $v = A ]; then unset THZDOE_LIB; else export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp1.so; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES -d gpurun_out/lds_$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --headline-only > gpurun_out/lds_pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/lds_pmc_$v.log; exit 1; }
done
unset THZDOE_LIB
python3 - <<'PY'
import csv, glob, collections
for v in 'AB':
    f = glob.glob(f'gpurun_out/lds_{v}/**/*counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0]
        if 'asm_' not in k: continue
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, m in acc.items():
        print(v, k[:40], 'conf/lds %.3f' % (m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_INSTS_LDS'], 1)),
              'lds_wait %.3f' % (m['SQ_WAIT_INST_LDS'] / max(m['SQ_WAVE_CYCLES'], 1)),
              'valu/wave %.0f' % (m['SQ_INSTS_VALU'] / max(m['SQ_WAVES'], 1)))
PY
