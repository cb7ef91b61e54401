set -o pipefail
mkdir -p gpurun_out/r05ay
for L in libqhuff libqhuff_lx2 libqhuff_lx4 libqhuff_lx8 libqhuff_lx12 libqhuff_lx14 libqhuff; do
QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/lens_time.py > gpurun_out/r05ay/$L.log 2>&1 || { tail -3 gpurun_out/r05ay/$L.log; exit 1; }
tail -1 gpurun_out/r05ay/$L.log
done
