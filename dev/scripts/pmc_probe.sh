#!/bin/bash
# Collect SQ counter groups (one rocprofv3 --pmc pass each) for bench.py --profile-only.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-pmc}; shift
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/g$i" -o run -- \
     python3 "$ROOT/bench.py" --steps 3 --warmup 1 --profile-only > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i ($group) rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/g$i.log"; exit $rc;; esac
done
