#!/bin/bash
# Round-end evidence: parity tests, smoke, bench, rocprofv3 kernel stats,
# FETCH/WRITE passes, then the bench again with the fresh traffic numbers.
set -u
bash scripts/gpu_check.sh r01f test smoke prof pmc || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r01f > gpurun_out/r01f/traffic.log 2>&1 || exit $?
cp profiles/pmc_traffic.json gpurun_out/r01f/pmc_traffic.json
bash scripts/gpu_check.sh r01f bench || exit $?
