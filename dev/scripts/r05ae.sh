set -o pipefail
mkdir -p gpurun_out/r05ae
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "cu_masked" > gpurun_out/r05ae/t.log 2>&1; rc=$?; tail -15 gpurun_out/r05ae/t.log; exit $rc
