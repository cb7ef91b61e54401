set -o pipefail
mkdir -p gpurun_out/r05aj
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "enc or count or full_size or c5 or round" > gpurun_out/r05aj/t.log 2>&1; rc=$?; tail -2 gpurun_out/r05aj/t.log; [ $rc -eq 0 ] || exit 1
for e in 0 1 0 1; do
if [ $e = 1 ]; then export QHUFF_LENS_WIN64=1; else unset QHUFF_LENS_WIN64; fi
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet A > gpurun_out/r05aj/e$e.log 2>&1 || exit 1
echo "win64=$e $(grep encoder gpurun_out/r05aj/e$e.log | cut -c60-200)"
done
unset QHUFF_LENS_WIN64
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet U > gpurun_out/r05aj/eU.log 2>&1 || exit 1
echo "U $(grep encoder gpurun_out/r05aj/eU.log | cut -c60-200)"
