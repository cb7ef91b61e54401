#!/bin/bash
# Dense-pack ablations (config 3, dense device decode).
set -u
OUT=gpurun_out/${1:-r04dp}; mkdir -p $OUT
step() { local n=$1; shift; timeout -k 10 120 "$@" >> $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
step dense python dev/scripts/dense_times.py &&
for v in dp1 dp2 dp4; do echo "== $v" >> $OUT/dense.log; QHUFF_LIB=nghttp3_amd/lib/libqhuff_$v.so step dense python dev/scripts/dense_times.py || exit 1; done
grep -v amdgpu.ids $OUT/dense.log
