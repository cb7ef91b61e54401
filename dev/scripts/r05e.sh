set -o pipefail
mkdir -p gpurun_out/r05e
K=pair13w16s2,pair13w16s4p32,pair13w16s2p32t12,pair13w12s4,pair13w12s4p32t12
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,$K --reps 10 > gpurun_out/r05e/decA.log 2>&1 || exit 1
for k in pair13w16s4p32 pair13w12s4; do
  QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=$k timeout -k 10 120 python -u dev/scripts/stamp_pairs.py >> gpurun_out/r05e/st.log 2>&1 || exit 1
done
cat gpurun_out/r05e/decA.log gpurun_out/r05e/st.log
