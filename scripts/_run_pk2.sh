set -o pipefail
mkdir -p gpurun_out/pk2
for cfg in "0 0" "1 0" "0 2" "1 2" "0 1" "1 1"; do
  set -- $cfg
  QHUFF_DEBUG=$1 QHUFF_BPC=$2 timeout -k 10 120 python -u scripts/dec_variants.py --kinds peek11 --reps 5 > gpurun_out/pk2/d$1_b$2.log 2>&1 || exit $?
  echo "debug=$1 bpc=$2 $(grep '^{' gpurun_out/pk2/d$1_b$2.log)"
done
