#!/bin/bash
# Round-end evidence: parity tests, smoke, bench, rocprofv3 kernel stats,
# FETCH/WRITE passes, then the bench again with the fresh traffic numbers.
set -u
bash scripts/gpu_check.sh r01g test smoke prof pmc || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r01g > gpurun_out/r01g/traffic.log 2>&1 || exit $?
cp profiles/pmc_traffic.json gpurun_out/r01g/pmc_traffic.json
bash scripts/gpu_check.sh r01g bench || exit $?
