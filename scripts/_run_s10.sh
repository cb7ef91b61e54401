#!/bin/bash
set -u
bash scripts/gpu_check.sh s10 test || exit $?
bash scripts/_run_s9.sh || exit $?
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lens timeout -k 10 200 python -u scripts/stamp_run.py
