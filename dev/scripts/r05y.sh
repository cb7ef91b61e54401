set -o pipefail
mkdir -p gpurun_out/r05y
export QHUFF_SEG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "encoder_variants or full_size or c5 or encode" > gpurun_out/r05y/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/r05y/pytest.log
[ $rc -eq 0 ] || exit 1
for a in A U; do
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows,fused --alphabet $a > gpurun_out/r05y/e$a.log 2>&1 || exit 1
grep encoder gpurun_out/r05y/e$a.log | cut -c1-330
done
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows,fused --zipf > gpurun_out/r05y/ez.log 2>&1 || exit 1
grep encoder gpurun_out/r05y/ez.log | cut -c1-330
