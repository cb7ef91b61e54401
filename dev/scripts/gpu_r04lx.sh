#!/bin/bash
# Length pass: product timing and the encoder GPU tests.
set -u
OUT=gpurun_out/${1:-r04lx}; mkdir -p $OUT
step() { local n=$1; shift; timeout -k 10 300 "$@" >> $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
QHUFF_VERBOSE=1 step lens python dev/scripts/lens_time.py &&
step pytest python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
step lens python dev/scripts/lens_time.py
grep -v amdgpu.ids $OUT/lens.log; tail -5 $OUT/pytest.log
