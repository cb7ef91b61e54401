#!/bin/bash
# Decoder development run: GPU tests of the decoder, then variant timings
# (config 3 A and U, config 5 Zipf A).  Every step has its own limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-dec}; KINDS=${2:-wring11x16r2,peek11lda}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
fatal() { case $1 in 124|134|137|139|143) return 0;; esac; return 1; }
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 15 "$OUT/$name.log"; if fatal $rc; then echo "FATAL $name"; exit $rc; fi; return $rc; }
run tests 300 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "not variants and not length_passes" || exit 1
# (any failure ends the session: a faulting variant must not run again)
run varA 120 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 10 || exit 1
run varZ 180 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 3 --zipf || exit 1
run varU 120 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 5 --alphabet U || exit 1
