set -o pipefail
mkdir -p gpurun_out/r05az
for L in libqhuff libqhuff_vspn libqhuff libqhuff_vspn; do
QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/lens_time.py > gpurun_out/r05az/$L.log 2>&1 || { tail -3 gpurun_out/r05az/$L.log; exit 1; }
tail -1 gpurun_out/r05az/$L.log
done
