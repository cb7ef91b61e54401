set -o pipefail
mkdir -p gpurun_out/r05ab
timeout -k 10 200 python -u dev/scripts/seg_check.py > gpurun_out/r05ab/check.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r05ab/check.log | tail -3; [ $rc -eq 0 ] || exit 1
export QHUFF_SEG=1
for d in 0 256 512 2048; do
QHUFF_DEBUG=$d timeout -k 10 120 python -u dev/scripts/enc_variants.py --only fused --alphabet A > gpurun_out/r05ab/e$d.log 2>&1 || exit 1
echo "abl=$((d>>8)) $(grep encoder gpurun_out/r05ab/e$d.log | cut -c60-200)"
done
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only fused --alphabet U > gpurun_out/r05ab/eU.log 2>&1 || exit 1
echo "U $(grep encoder gpurun_out/r05ab/eU.log | cut -c60-200)"
