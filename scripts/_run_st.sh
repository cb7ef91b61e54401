#!/bin/bash
set -o pipefail
O=gpurun_out/${TAG:-st1}; mkdir -p $O
for k in ${K:-peek11 peek11d}; do
  QHUFF_DECODER=$k QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=dec_peek REPS=3 \
    timeout -k 10 120 python -u scripts/stamp_run.py > $O/$k.log 2>&1 || { tail -5 $O/$k.log; exit 1; }
  echo "== $k"; cat $O/$k.log
done
