set -o pipefail
mkdir -p gpurun_out/r05ah
for a in U A; do for sl in 1.5 1.2 2.0 100; do
QHUFF_PLAN_SKEW_LONG=$sl timeout -k 10 120 python dev/scripts/dec_variants.py --alphabet $a --kinds peek11s,sorted11 > gpurun_out/r05ah/t$a$sl.txt 2>&1 || { tail -3 gpurun_out/r05ah/t$a$sl.txt; exit 1; }
echo "$a long=$sl $(grep kind gpurun_out/r05ah/t$a$sl.txt | cut -c1-200 | tr '\n' ' ')"
done; done
for sk in 3.0 2.0 100; do
QHUFF_PLAN_SKEW=$sk timeout -k 10 120 python dev/scripts/dec_variants.py --zipf --kinds peek11s,sorted11 > gpurun_out/r05ah/z$sk.txt 2>&1 || exit 1
echo "zipf skew=$sk $(grep kind gpurun_out/r05ah/z$sk.txt | cut -c1-200 | tr '\n' ' ')"
done
