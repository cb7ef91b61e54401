#!/bin/bash
set -o pipefail
O=gpurun_out/${TAG:-st2}; mkdir -p $O
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lens REPS=3 \
  timeout -k 10 120 python -u scripts/stamp_run.py > $O/lens.log 2>&1 || { tail -5 $O/lens.log; exit 1; }
cat $O/lens.log
QHUFF_DEBUG=32 QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lanes REPS=3 \
  timeout -k 10 120 python -u scripts/stamp_run.py > $O/lanes.log 2>&1 || { tail -5 $O/lanes.log; exit 1; }
cat $O/lanes.log
