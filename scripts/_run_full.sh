#!/bin/bash
# full GPU test suite, then the default decoder's timing
set -o pipefail
O=gpurun_out/${TAG:-full}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 240 python -u scripts/dec_variants.py --reps 10 > $O/A.log 2>&1 || { tail -5 $O/A.log; exit 1; }
cat $O/A.log
