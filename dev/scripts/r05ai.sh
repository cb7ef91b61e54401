set -o pipefail
mkdir -p gpurun_out/r05ai
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or host_path or decode_host" > gpurun_out/r05ai/t.log 2>&1; rc=$?; tail -3 gpurun_out/r05ai/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u dev/scripts/dense_times.py > gpurun_out/r05ai/d.log 2>&1 || exit 1
grep dense gpurun_out/r05ai/d.log
