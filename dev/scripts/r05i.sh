set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s,pair13w16s2,pair13w16s2sel,pair13w16s2k2,pair13w12s4,pair13w16s2_ns --reps 10 > gpurun_out/r05i/decA.log 2>&1 || exit 1
QHUFF_DEBUG=8 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 > gpurun_out/r05i/decA_nostore.log 2>&1 || exit 1
cat gpurun_out/r05i/decA.log gpurun_out/r05i/decA_nostore.log
