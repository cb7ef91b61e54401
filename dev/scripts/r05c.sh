set -o pipefail
mkdir -p gpurun_out/r05c
for k in pair13w16s2 pair13w12s4; do
  QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=$k timeout -k 10 120 python -u dev/scripts/stamp_pairs.py >> gpurun_out/r05c/st.log 2>&1 || exit 1
done
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=pair13w16s2 ALPH=U timeout -k 10 120 python -u dev/scripts/stamp_pairs.py >> gpurun_out/r05c/st.log 2>&1
cat gpurun_out/r05c/st.log
