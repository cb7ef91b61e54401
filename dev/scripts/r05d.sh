set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,pair13w16s2,pair13w16s2_nw,pair13w16s2_nr,pair13w16s2_nwr,pair13w16s2_b,pair13w12s4,pair13w12s4_nw --reps 10 > gpurun_out/r05d/decA.log 2>&1
cat gpurun_out/r05d/decA.log
