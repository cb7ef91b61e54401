#!/bin/bash
# rocprofv3 PMC passes over decoder variants (development tool): one pass
# per counter group given, each under its own time limit.
#   dev/scripts/pmc_dec.sh TAG KINDS "GROUP1" ["GROUP2" ...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=$1; KINDS=$2; shift 2
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/g$i" -o run -- \
     python3 "$ROOT/dev/scripts/dec_variants.py" --kinds "$KINDS" --reps 2 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 "$ROOT/dev/scripts/pmc_summary.py" "$OUT" | grep -E 'dec_'
