#!/bin/bash
# rocprofv3 copy + kernel trace of bench.py's host-memory leg, per call
# (development): dev/scripts/host_outlier.sh TAG
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$ROOT/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace -d $O/trace -o run -- \
  python3 $ROOT/dev/scripts/host_outlier_trace.py $O/calls.json > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; grep '^{' $O/trace.log
[ $rc -eq 0 ] && python3 $ROOT/dev/scripts/host_outlier_summary.py $O
