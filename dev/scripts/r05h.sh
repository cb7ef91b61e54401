set -o pipefail
mkdir -p gpurun_out/r05h
export QH_TEST_DEV_DECODERS=pair13w16s2,pair13w16s2k2,pair13w12s4,pair13w12s4k2
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "test_decoder_variants or test_long_code_mode" > gpurun_out/r05h/t.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r05h/t.log; exit 1; }
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,pair13w16s2,pair13w16s2k2,pair13w12s4,pair13w12s4k2,pair13w16s2_ns --reps 10 > gpurun_out/r05h/decA.log 2>&1 || exit 1
for k in pair13w16s2 pair13w16s2k2; do
  QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=$k timeout -k 10 120 python -u dev/scripts/stamp_pairs.py >> gpurun_out/r05h/st.log 2>&1 || exit 1
done
cat gpurun_out/r05h/decA.log gpurun_out/r05h/st.log
