#!/bin/bash
# GPU tests, bench kernel times and stream-lens stamps (development helper)
set -u
bash scripts/gpu_check.sh s4 test || exit $?
bash scripts/_run_pk3.sh || exit $?
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=enc_lens timeout -k 10 200 python -u scripts/stamp_run.py
