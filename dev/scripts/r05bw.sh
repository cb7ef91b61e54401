set -o pipefail
bash dev/scripts/benchvar.sh r05bw "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vring.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vring.so"
