set -o pipefail
mkdir -p gpurun_out/r05ap
for A in A U Z; do
for L in libqhuff libqhuff_ew0s32768 libqhuff_ew0s45056 libqhuff_ew0s65536; do
Z=""; AL=$A; if [ $A = Z ]; then Z=--zipf; AL=A; fi
QHUFF_VERBOSE=1 QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet $AL $Z > gpurun_out/r05ap/$A$L.log 2>&1 || { tail -3 gpurun_out/r05ap/$A$L.log; exit 1; }
echo "$A $L $(grep -h 'lds=' gpurun_out/r05ap/$A$L.log | grep -v 'lds=39984\|lds=156' | sort -u | head -1 | cut -c16-80) $(grep encoder gpurun_out/r05ap/$A$L.log | grep -o '"qh_k_enc_lanes": [0-9.]*\|"sha": "[0-9a-f]*"' | tr '\n' ' ')"
done; done
