set -o pipefail
mkdir -p gpurun_out/r05af
for L in libqhuff libqhuff_ew5s22528 libqhuff_ew6s16384 libqhuff_ew4s20480 libqhuff; do
QHUFF_VERBOSE=1 QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet A > gpurun_out/r05af/$L.log 2>&1 || { tail -3 gpurun_out/r05af/$L.log; exit 1; }
echo "$L $(grep -h 'blocks/CU' gpurun_out/r05af/$L.log | sort -u | head -1) $(grep encoder gpurun_out/r05af/$L.log | cut -c60-230)"
done
