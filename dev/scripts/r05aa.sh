set -o pipefail
mkdir -p gpurun_out/r05aa
export QHUFF_SEG=1
for d in 0 256 512 1024 2048 1280 3072; do
QHUFF_DEBUG=$d timeout -k 10 120 python -u dev/scripts/enc_variants.py --only fused --alphabet A > gpurun_out/r05aa/e$d.log 2>&1 || exit 1
echo "abl=$((d>>8)) $(grep encoder gpurun_out/r05aa/e$d.log | cut -c60-200)"
done
