#!/bin/bash
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=${KERNELS:-enc_lanes} timeout -k 10 200 python -u scripts/stamp_run.py
