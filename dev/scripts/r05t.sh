set -o pipefail
mkdir -p gpurun_out/r05t
for d in 0 16 8; do
QHUFF_DEBUG=$d QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=dec_peek timeout -k 10 120 python dev/scripts/stamp_run.py > gpurun_out/r05t/s$d.txt 2>&1 || { tail -5 gpurun_out/r05t/s$d.txt; exit 1; }
echo "dbg=$d"; cat gpurun_out/r05t/s$d.txt | grep -v amdgpu.ids
done
