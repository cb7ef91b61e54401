set -o pipefail
mkdir -p gpurun_out/r05ac
QHUFF_SEG=1 QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so KERNELS=encs timeout -k 10 120 python dev/scripts/stamp_run.py > gpurun_out/r05ac/s.txt 2>&1; grep -v amdgpu gpurun_out/r05ac/s.txt
