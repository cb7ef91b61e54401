#!/bin/bash
# Development session on the GPU box: decoder variants of the development
# build (make dev) through the parity tests, then timed on config 3 (alphabets
# A and U) and config 5 lengths.  Usage: dev/scripts/gpu_dev.sh TAG KINDS
set -u
TAG=$1; KINDS=$2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$ROOT"
export QHUFF_LIB=$ROOT/nghttp3_amd/lib/libqhuff_dev.so
step() {  # step NAME LIMIT CMD...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "$OUT/$name.log"
  case $rc in 0) return 0;; *) exit $rc;; esac
}
DEVK=$(echo "$KINDS" | tr ',' '\n' | grep -v -x -e peek11s -e wring11x16r2 | paste -sd, -)
QH_TEST_DEV_DECODERS=$DEVK step tests 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "decoder_variants or zipf or full_size" -p no:cacheprovider --timeout 120 --timeout-method thread
step timeA 200 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 10
step timeU 200 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 5 --alphabet U
step timeZ 300 python dev/scripts/dec_variants.py --kinds "$KINDS" --reps 3 --zipf --n 2097152
