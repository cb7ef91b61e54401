for d in 0 0 1 3; do QHUFF_DEBUG=$d QHUFF_DECODER=run timeout -k 10 120 python -u scripts/dec_variants.py --kinds run --reps 5 2>&1 | grep -E "^\{" | sed "s/^/dbg=$d /" | cut -c1-160; done
for b in 1 2; do QHUFF_BPC=$b QHUFF_DEBUG=3 QHUFF_DECODER=run timeout -k 10 120 python -u scripts/dec_variants.py --kinds run --reps 5 2>&1 | grep -E "^\{" | sed "s/^/dbg=3 bpc=$b /" | cut -c1-160; done
