set -o pipefail
mkdir -p gpurun_out/r05ak
timeout -k 10 600 python -u -m pytest tests/test_gpu_qpack.py tests/test_gpu_qif.py tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "section or config4 or qpack or token or check or qif" > gpurun_out/r05ak/t.log 2>&1; rc=$?; tail -2 gpurun_out/r05ak/t.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 120 python dev/scripts/frame_time.py > gpurun_out/r05ak/f$i.txt 2>&1 || exit 1; tail -1 gpurun_out/r05ak/f$i.txt | cut -c1-300; done
