#!/bin/bash
# Codes-pass ablations (config 3).
set -u
OUT=gpurun_out/${1:-r04la}; mkdir -p $OUT
step() { local n=$1; shift; timeout -k 10 120 "$@" >> $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
step lens python dev/scripts/lens_time.py &&
for v in la12 la14 la4; do QHUFF_LIB=nghttp3_amd/lib/libqhuff_$v.so step lens python dev/scripts/lens_time.py || exit 1; done &&
QHUFF_ENC_BPC=2 step lens python dev/scripts/lens_time.py && QHUFF_ENC_BPC=3 step lens python dev/scripts/lens_time.py
grep -v amdgpu.ids $OUT/lens.log
