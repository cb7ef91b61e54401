set -o pipefail
mkdir -p gpurun_out/r05x
for L in libqhuff libqhuff_frc32 libqhuff_frc16 libqhuff; do
QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python dev/scripts/frame_time.py > gpurun_out/r05x/$L.txt 2>&1 || { tail -5 gpurun_out/r05x/$L.txt; exit 1; }
echo "$L $(tail -1 gpurun_out/r05x/$L.txt)"
done
