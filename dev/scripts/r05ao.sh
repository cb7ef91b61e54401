set -o pipefail
mkdir -p gpurun_out/r05ao
for L in libqhuff libqhuff_ew0s32768 libqhuff_ew0s28672 libqhuff libqhuff_ew0s32768; do
QHUFF_VERBOSE=1 QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet A > gpurun_out/r05ao/$L.log 2>&1 || { tail -3 gpurun_out/r05ao/$L.log; exit 1; }
echo "$L $(grep -h 'lds=' gpurun_out/r05ao/$L.log | grep -v 'lds=39984\|lds=156' | sort -u | head -2 | tr '\n' ' ') $(grep encoder gpurun_out/r05ao/$L.log | cut -c60-230)"
done
QHUFF_LIB=nghttp3_amd/lib/libqhuff_ew0s32768.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet U > gpurun_out/r05ao/U.log 2>&1 || exit 1
echo "U s32768 $(grep encoder gpurun_out/r05ao/U.log | cut -c60-230)"
