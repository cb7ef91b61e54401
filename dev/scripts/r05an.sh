set -o pipefail
mkdir -p gpurun_out/r05an
for b in 0 8 12 16 0; do
if [ $b = 0 ]; then unset QHUFF_BPC; else export QHUFF_BPC=$b; fi
timeout -k 10 120 python dev/scripts/dec_variants.py --alphabet A --kinds peek11s > gpurun_out/r05an/d$b.txt 2>&1 || { tail -3 gpurun_out/r05an/d$b.txt; exit 1; }
echo "dec bpc=$b $(grep kind gpurun_out/r05an/d$b.txt | cut -c60-220)"
done
unset QHUFF_BPC
for b in 0 8 12 0; do
if [ $b = 0 ]; then unset QHUFF_ENC_BPC; else export QHUFF_ENC_BPC=$b; fi
timeout -k 10 120 python -u dev/scripts/enc_variants.py --only windows --alphabet A > gpurun_out/r05an/e$b.log 2>&1 || exit 1
echo "enc bpc=$b $(grep encoder gpurun_out/r05an/e$b.log | cut -c60-220)"
done
