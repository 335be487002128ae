set -u
# kernel trace of the full bench line (headline + cfg3 CZT + cfg4 QAT), no CPU baseline
export TMPDIR=/tmp
out=${1:-gpurun_out/pfull}; mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $out/bench.log 2>&1 || exit $?
echo ok
