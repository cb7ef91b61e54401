set -o pipefail
mkdir -p gpurun_out/r05q
bash dev/scripts/pmc_dec.sh r05q/a "peek11s,peek11s_256,wring11x16r2" "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/r05q/a.txt 2>&1 || { cat gpurun_out/r05q/a.txt; exit 1; }
QHUFF_DEBUG=8 bash dev/scripts/pmc_dec.sh r05q/b "peek11s" "FETCH_SIZE" > gpurun_out/r05q/b.txt 2>&1 || { cat gpurun_out/r05q/b.txt; exit 1; }
cat gpurun_out/r05q/a.txt gpurun_out/r05q/b.txt
