#!/bin/bash
for k in ${KERNELS:-enc_lens}; do
REPS=1 QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=$k timeout -k 10 200 python -u scripts/stamp_run.py
done
