set -o pipefail
mkdir -p gpurun_out/r05w
for a in A U; do
timeout -k 10 120 python dev/scripts/dec_variants.py --alphabet $a --kinds peek11s,peek11sn,peek11s,peek11sn > gpurun_out/r05w/t$a.txt 2>&1 || { tail -5 gpurun_out/r05w/t$a.txt; exit 1; }
grep kind gpurun_out/r05w/t$a.txt | cut -c1-250
done
timeout -k 10 120 python dev/scripts/dec_variants.py --zipf --kinds peek11s,peek11sn > gpurun_out/r05w/tz.txt 2>&1 || { tail -5 gpurun_out/r05w/tz.txt; exit 1; }
grep kind gpurun_out/r05w/tz.txt | cut -c1-250
