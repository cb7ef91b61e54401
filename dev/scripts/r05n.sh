set -o pipefail
mkdir -p gpurun_out/r05n
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u dev/scripts/block_times.py dec > gpurun_out/r05n/bt.log 2>&1
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u dev/scripts/block_times.py dec >> gpurun_out/r05n/bt.log 2>&1
cat gpurun_out/r05n/bt.log
