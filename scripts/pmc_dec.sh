#!/bin/bash
# PMC counter groups for the decoder variants (one rocprofv3 --pmc pass per
# group, each under its own time limit).  Usage: scripts/pmc_dec.sh TAG KINDS [GROUPSET]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmcdec}; KINDS=${2:-peek11}; SET=${3:-sq}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "$SET" = sq ]; then
  GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
elif [ "$SET" = full ]; then
  GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_BUSY_avr TCC_EA0_RDREQ_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum")
else
  GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum")
fi
i=0
for group in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/$SET$i" -o run -- \
     python3 "$ROOT/scripts/dec_variants.py" --kinds "$KINDS" --reps 2 > "$OUT/$SET$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$SET$i.log"; exit $rc; fi
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" | grep -E 'qhk::' > "$OUT/summary_$SET.txt"; cat "$OUT/summary_$SET.txt"
