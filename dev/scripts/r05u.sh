set -o pipefail
mkdir -p gpurun_out/r05u
for d in 0 16; do for a in A U; do
QHUFF_DEBUG=$d timeout -k 10 120 python dev/scripts/dec_variants.py --alphabet $a --kinds peek11s,peek11s_e,peek11s > gpurun_out/r05u/t$d$a.txt 2>&1 || exit 1
echo "dbg=$d"; grep kind gpurun_out/r05u/t$d$a.txt | cut -c1-250
done; done
