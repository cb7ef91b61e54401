set -o pipefail
mkdir -p gpurun_out/r05b
export QH_TEST_DEV_DECODERS=pair13w16s2,pair13w12s4,pair12w16s2,pair12w12s4
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "test_decoder_variants or test_long_code_mode" > gpurun_out/r05b/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05b/t.log; exit 1; }
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,pair13w16s2,pair13w12s4,pair12w16s2,pair12w12s4 --reps 10 > gpurun_out/r05b/decA.log 2>&1
timeout -k 10 300 python -u dev/scripts/dec_variants.py --alphabet U --kinds peek11s,pair13w16s2,pair13w12s4,pair12w16s2,pair12w12s4 --reps 5 > gpurun_out/r05b/decU.log 2>&1
cat gpurun_out/r05b/decA.log gpurun_out/r05b/decU.log
