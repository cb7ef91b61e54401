#!/bin/bash
# decoder occupancy variants: parity first, then timing (A and U alphabets)
set -o pipefail
O=gpurun_out/${TAG:-v1}; mkdir -p $O
K=${K:-peek11,peek11s,peek11d,peek11sd,peek11_2w5sd}
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "decoder_variants" > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 240 python -u scripts/dec_variants.py --kinds $K --reps 10 > $O/A.log 2>&1 || { tail -5 $O/A.log; exit 1; }
cat $O/A.log
timeout -k 10 240 python -u scripts/dec_variants.py --kinds $K --reps 5 --alphabet U > $O/U.log 2>&1 || { tail -5 $O/U.log; exit 1; }
cat $O/U.log
