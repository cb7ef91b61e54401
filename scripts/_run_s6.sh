#!/bin/bash
set -u
bash scripts/gpu_check.sh s6 test || exit $?
bash scripts/_run_pk3.sh || exit $?
QHUFF_DEBUG=32 QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lanes timeout -k 10 200 python -u scripts/stamp_run.py
