set -u
mkdir -p gpurun_out
for zc in 16 32 64; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --headline-only --steps 10 --z-chunk $zc > gpurun_out/zc$zc.log 2>&1 || { echo "zc $zc failed"; exit 1; }
done
echo done
