set -u
mkdir -p gpurun_out
for v in 0 2 8; do
  if [ $v = 0 ]; then L=quantizationawarethzdoe_amd/libthzdoe.so; else L=quantizationawarethzdoe_amd/libthzdoe_exp$v.so; fi
  THZDOE_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/exp$v.log 2>&1 || { echo "exp $v failed rc=$?"; exit 1; }
done
echo done
