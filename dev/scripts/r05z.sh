set -o pipefail
mkdir -p gpurun_out/r05z
SEG_DUMP=gpurun_out/r05z timeout -k 10 200 python -u dev/scripts/seg_check.py > gpurun_out/r05z/check.log 2>&1; cat gpurun_out/r05z/check.log | grep -v amdgpu.ids
