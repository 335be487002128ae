#!/bin/bash
# Round-4 close in one call: (1) A/B of the compile-time middle-crop K2 / K3 against the generic
# kernels on the cfg2 headline (two pairs); the faster form is used for the rest of the call
# (THZ_K2_MID / THZ_K3_MID exported, recorded in ab.txt); (2) the whole -m gpu suite and smoke();
# (3) cfg2 kernel trace + PMC passes, cfg3 CZT trace + PMC, cfg5 DONN trace; (4) the default
# bench line with the CPU baseline leg.  Each GPU step under its own time limit (gpu_step.sh).
set -o pipefail
o=gpurun_out/close
mkdir -p $o
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --headline-only"
THZ_K2_MID=1 THZ_K3_MID=1 bash $S 200 $o/mid_a.log python $B &&
THZ_K2_MID=0 THZ_K3_MID=0 bash $S 200 $o/gen_a.log python $B &&
THZ_K2_MID=1 THZ_K3_MID=1 bash $S 200 $o/mid_b.log python $B &&
THZ_K2_MID=0 THZ_K3_MID=0 bash $S 200 $o/gen_b.log python $B || exit $?
python3 - "$o" > $o/ab.txt <<'PY'
import json, sys
o = sys.argv[1]
def v(f):
    for l in open(f"{o}/{f}.log"):
        if l.startswith("{"):
            return json.loads(l)["value"]
mid = (v("mid_a") + v("mid_b")) / 2
gen = (v("gen_a") + v("gen_b")) / 2
print(f"mid {mid:.1f} gen {gen:.1f} -> {'mid' if mid >= gen else 'generic'}")
PY
cat $o/ab.txt
if grep -q "generic" $o/ab.txt; then export THZ_K2_MID=0 THZ_K3_MID=0; else export THZ_K2_MID=1 THZ_K3_MID=1; fi
bash $S 1000 $o/gpu_tests.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider &&
bash $S 200 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
bash $S 900 $o/prof.log bash scripts/profile_asm.sh $o/prof &&
bash $S 200 $o/czt_trace.log rocprofv3 --kernel-trace --stats -d $o/czt/trace -o run --output-format csv -- python3 scripts/czt_prof.py 5 &&
bash $S 120 $o/czt_lds.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAVES -d $o/czt/pmc_lds -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $o/czt_fetch.log rocprofv3 --pmc FETCH_SIZE -d $o/czt/pmc_fetch -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 120 $o/czt_write.log rocprofv3 --pmc WRITE_SIZE -d $o/czt/pmc_write -o run --output-format csv -- python3 scripts/czt_prof.py 3 &&
bash $S 300 $o/donn.log rocprofv3 --kernel-trace --stats -d $o/donn -o run --output-format csv -- python3 scripts/donn_prof.py 20 &&
bash $S 400 $o/bench.log python bench.py
