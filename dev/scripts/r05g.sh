set -o pipefail
mkdir -p gpurun_out/r05g
export QH_TEST_DEV_DECODERS=pair13w16s2,pair13w12s4,pair13w16s2k4,pair13w12s4k4
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "test_decoder_variants or test_long_code_mode" > gpurun_out/r05g/t.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r05g/t.log; exit 1; }
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,pair13w16s2,pair13w12s4,pair13w16s2k4,pair13w12s4k4 --reps 10 > gpurun_out/r05g/decA.log 2>&1 || exit 1
for k in pair13w16s2 pair13w12s4k4; do
  QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=$k timeout -k 10 120 python -u dev/scripts/stamp_pairs.py >> gpurun_out/r05g/st.log 2>&1 || exit 1
done
timeout -k 10 300 python -u dev/scripts/dec_variants.py --alphabet U --kinds peek11s,sorted11,pair13w16s2,pair13w12s4 --reps 5 > gpurun_out/r05g/decU.log 2>&1
timeout -k 10 300 python -u dev/scripts/dec_variants.py --zipf --n 2097152 --kinds peek11s,sorted11,pair13w16s2,pair13w12s4 --reps 3 > gpurun_out/r05g/decZ.log 2>&1
cat gpurun_out/r05g/decA.log gpurun_out/r05g/st.log gpurun_out/r05g/decU.log gpurun_out/r05g/decZ.log
