#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/fault/timeout ends the
# script (no further GPU work).  Usage: dev/scripts/gpu_check.sh TAG [STEPS...]
# steps: test smoke bench prof pmc (default: test smoke bench prof)
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-test smoke bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"

fatal() {  # exit codes that mean the GPU step crashed or hung
  case $1 in 124|134|137|139|143) return 0;; esac; return 1; }

run() {  # run NAME LIMIT CMD...
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  local t0=$(date +%s)
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/steps.log"
  tail -n 25 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return $rc
}

for s in $STEPS; do
  case $s in
    test)  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
    bench) run bench 600 python bench.py && grep '^{' "$OUT/bench.log" > "$OUT/bench.json" ;;
    prof)  ( cd /tmp && export TMPDIR=/tmp && run rocprof 600 rocprofv3 --kernel-trace --stats \
               --output-format csv -d "$OUT/prof" -o run -- \
               python3 "$ROOT/bench.py" --steps 10 --warmup 2 --profile-only ) ;;
    pmc)   for ctr in FETCH_SIZE WRITE_SIZE; do
             ( cd /tmp && export TMPDIR=/tmp && run pmc_$ctr 600 rocprofv3 --pmc $ctr \
                 --output-format csv -d "$OUT/pmc_$ctr" -o run -- \
                 python3 "$ROOT/bench.py" --steps 5 --warmup 1 --profile-only ) || exit $?
           done ;;
  esac
done
echo "done: $STEPS"
