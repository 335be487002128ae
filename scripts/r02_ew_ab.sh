set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -x -m gpu -k "optics or lens or aperture or donn or qat" > gpurun_out/ew_tests.log 2>&1 || { tail -20 gpurun_out/ew_tests.log; exit 1; }
tail -1 gpurun_out/ew_tests.log
for rep in 1 2; do for v in A B; do
  if [ $v = A ]; then unset THZDOE_LIB; else export THZDOE_LIB=$PWD/quantizationawarethzdoe_amd/libthzdoe_exp1.so; fi
  timeout -k 10 200 python scripts/bench_aux.py > gpurun_out/ew_$v$rep.log 2>&1 || { tail -5 gpurun_out/ew_$v$rep.log; exit 1; }
  echo "$v$rep"; grep -E "thin_lens|aperture" gpurun_out/ew_$v$rep.log | cut -c1-200
done; done
