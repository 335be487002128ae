#!/bin/bash
# round-5 full check on one box: the whole -m gpu suite, smoke(), the default bench line, the bench's
# rocprofv3 kernel trace + PMC passes, and kernel traces of the small graph-replayed steps.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r05full}
mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -c 600 $O/bench.json
bash scripts/profile_asm.sh gpurun_out/${2:-r05_prof2} || exit $?
bash scripts/r05_small_traces.sh gpurun_out/${3:-r05_small2} || exit $?
