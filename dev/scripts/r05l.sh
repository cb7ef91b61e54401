set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 > gpurun_out/r05l/a.log 2>&1 || exit 1
QHUFF_DEBUG=16 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05l/a.log 2>&1 || exit 1
QHUFF_DEBUG=8 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05l/a.log 2>&1 || exit 1
QHUFF_DEBUG=24 timeout -k 10 300 python -u dev/scripts/dec_variants.py --kinds peek11s --reps 10 >> gpurun_out/r05l/a.log 2>&1 || exit 1
cat gpurun_out/r05l/a.log | grep kind
