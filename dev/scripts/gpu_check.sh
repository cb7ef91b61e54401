#!/bin/bash
# One GPU check on a gpurun box: selected GPU tests, then (only if they pass)
# a short bench run.  Every GPU step under its own time limit; the first
# failure ends the script.
#   dev/scripts/gpu_check.sh <out-dir> "<pytest -k expression or ALL>" [bench args...]
out=gpurun_out/$1; shift
sel=$1; shift
mkdir -p "$out"
if [ "$sel" = "ALL" ]; then k=(); else k=(-k "$sel"); fi
if [ "$sel" != "NONE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${k[@]}" > "$out/pytest.log" 2>&1
  rc=$?
  tail -3 "$out/pytest.log"
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
fi
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u bench.py "$@" > "$out/bench.log" 2>&1
  rc=$?
  echo "bench rc=$rc"
  tail -c 600 "$out/bench.log"
  exit $rc
fi
