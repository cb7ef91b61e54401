set -o pipefail
mkdir -p gpurun_out/r05j
export QH_TEST_DEV_DECODERS=peek11snake,pair13w16s2
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "test_decoder_variants or test_long_code_mode or test_full_size_config or test_window_decoder_plan" > gpurun_out/r05j/t.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r05j/t.log; exit 1; }
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,peek11snake,peek11s,peek11snake --reps 10 > gpurun_out/r05j/decA.log 2>&1 || exit 1
timeout -k 10 300 python -u dev/scripts/dec_variants.py --alphabet U --kinds peek11s,peek11snake,sorted11 --reps 5 > gpurun_out/r05j/decU.log 2>&1 || exit 1
timeout -k 10 300 python -u dev/scripts/dec_variants.py --zipf --n 2097152 --kinds peek11s,peek11snake,sorted11 --reps 3 > gpurun_out/r05j/decZ.log 2>&1
cat gpurun_out/r05j/decA.log gpurun_out/r05j/decU.log gpurun_out/r05j/decZ.log; grep -E "passed|failed" gpurun_out/r05j/t.log | tail -2
