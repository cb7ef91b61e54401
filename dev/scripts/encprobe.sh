# usage: bash dev/scripts/encprobe.sh OUTDIR "lib1 lib2 ..." "A U Z"
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for A in $3; do
for L in $2; do
Z=""; AL=$A; if [ $A = Z ]; then Z=--zipf; AL=A; fi
QHUFF_VERBOSE=1 QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet $AL $Z > $O/$A$L.log 2>&1 || { tail -3 $O/$A$L.log; exit 1; }
echo "$A $L $(grep -h 'lds=' $O/$A$L.log | grep -v 'lds=39984\|lds=156' | sort -u | head -1 | cut -c16-80) $(grep encoder $O/$A$L.log | grep -o '"qh_k_enc_lens_stream": [0-9.]*\|"qh_k_enc_lanes": [0-9.]*\|"sha": "[0-9a-f]*"' | tr '\n' ' ')"
done; done
