set -u
# A/B: default library vs the THZ_PV=8 variant (ASM parity with the variant, then headline bench of both)
mkdir -p gpurun_out
L8=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp8.so
THZDOE_LIB=$L8 timeout -k 10 400 python -m pytest tests -q -x -m gpu -k "asm or rsc or czt" > gpurun_out/pv8_tests.log 2>&1 || { echo "pv8 tests failed"; tail -30 gpurun_out/pv8_tests.log; exit 1; }
for rep in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/pv16_$rep.log 2>&1 || { echo "pv16 failed"; exit 1; }
THZDOE_LIB=$L8 timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 > gpurun_out/pv8_$rep.log 2>&1 || { echo "pv8 failed"; exit 1; }
done
echo done
