#!/bin/bash
# blocks-per-CU sweep for the codes kernel and the decoder (timing only)
set -o pipefail
O=gpurun_out/${TAG:-bpc}; mkdir -p $O
for e in 2 3 4; do
  QHUFF_ENC_BPC=$e timeout -k 10 200 python -u bench.py --no-configs > $O/enc$e.log 2>&1 || { tail -5 $O/enc$e.log; exit 1; }
  echo "enc_bpc=$e $(grep '^{' $O/enc$e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], {k:v['avg_us'] for k,v in d['extra']['kernels'].items()})")"
done
for b in 2 3; do
  QHUFF_BPC=$b timeout -k 10 200 python -u scripts/dec_variants.py --kinds peek11ld --reps 10 > $O/dec$b.log 2>&1 || { tail -5 $O/dec$b.log; exit 1; }
  echo "dec_bpc=$b $(grep kind $O/dec$b.log)"
done
