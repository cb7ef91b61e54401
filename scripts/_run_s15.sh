#!/bin/bash
set -u
bash scripts/gpu_check.sh s15 test || exit $?
for a in A U; do
  timeout -k 10 120 python -u scripts/dec_variants.py --kinds peek11,peek12,peek10 --alphabet $a --reps 10 2>&1 | grep '^{'
done
