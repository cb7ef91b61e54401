#!/bin/bash
for b in 2 3 4 5 6; do
  echo "== QHUFF_BPC=$b"
  QHUFF_BPC=$b timeout -k 10 120 python -u scripts/dec_variants.py --kinds peek11 --reps 10 2>&1 | grep '^{'
done
