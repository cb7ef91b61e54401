#!/bin/bash
# SQ PMC groups over the fused encoder alone (dev/scripts/enc_variants.py --only
# fused), one rocprofv3 --pmc pass per group.  Usage: dev/scripts/pmc_encf.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-pmcencf}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/g$i" -o run -- \
     python3 "$ROOT/dev/scripts/enc_variants.py" --only fused --reps 2 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 "$ROOT/dev/scripts/pmc_summary.py" "$OUT" | grep -E 'qhk' | sed 's/  /\n   /g' > "$OUT/summary.txt"
cat "$OUT/summary.txt"
