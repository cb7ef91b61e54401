#!/bin/bash
# The round's final evidence on one gpurun box (development tool): GPU tests,
# smoke, the default bench line, and a rocprofv3 kernel-trace summary of the
# bench's config-3 step.  Every GPU step under its own time limit; the first
# failure ends the script.   dev/scripts/gpu_final.sh TAG
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $O/bench.log; exit $rc; }
grep '"metric"' $O/bench.log > $O/bench.json; head -c 600 $O/bench.json; echo
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python3 $R/bench.py --profile-only --steps 40 --warmup 5 > $R/$O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; find $R/$O/prof -name "*kernel_stats.csv" | head -2
exit $rc
