#!/bin/bash
# GPU check of the whole-section pipelines (decoder and encoder sides, the
# QIF driver) and one bench run.  Usage: dev/scripts/gpu_sections.sh TAG
set -u
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$ROOT/gpurun_out/$TAG; mkdir -p "$O"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_qpack.py tests/test_gpu_qif.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/tests_qpack.log" 2>&1; rc=$?
tail -1 "$O/tests_qpack.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || exit $?
grep "^{" "$O/bench.log" > "$O/bench.json"
