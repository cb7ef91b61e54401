#!/bin/bash
# SQ + memory-path PMC groups over bench.py --profile-only (one rocprofv3
# --pmc pass per group, each under its own limit).  Usage: dev/scripts/pmc_enc.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${1:-pmcenc}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for group in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_BUSY_avr TCC_EA0_RDREQ_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/g$i" -o run -- \
     python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile-only > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 "$ROOT/dev/scripts/pmc_summary.py" "$OUT" | grep -E 'qhk' | sed 's/  /\n   /g' > "$OUT/summary.txt"
cat "$OUT/summary.txt"
