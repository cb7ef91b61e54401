set -o pipefail
mkdir -p gpurun_out/r05r
for d in 16; do
QHUFF_DEBUG=$d bash dev/scripts/pmc_dec.sh r05r/d$d "peek11s" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/r05r/d$d.txt 2>&1 || { cat gpurun_out/r05r/d$d.txt; exit 1; }
QHUFF_DEBUG=$d timeout -k 10 120 python dev/scripts/dec_variants.py --kinds peek11s > gpurun_out/r05r/t$d.txt 2>&1 || exit 1
echo "dbg=$d"; grep peek gpurun_out/r05r/d$d.txt; tail -1 gpurun_out/r05r/t$d.txt | cut -c1-400
done
