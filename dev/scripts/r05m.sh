set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 > gpurun_out/r05m/a.log 2>&1 || exit 1
QHUFF_DEBUG=32 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05m/a.log 2>&1 || exit 1
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05m/a.log 2>&1 || exit 1
QHUFF_DEBUG=32 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05m/a.log 2>&1 || exit 1
cat gpurun_out/r05m/a.log | grep kind
