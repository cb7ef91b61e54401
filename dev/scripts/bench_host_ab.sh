#!/bin/bash
# The whole bench (no CPU baseline) per library, host-path leg printed
# (development): dev/scripts/bench_host_ab.sh OUT LIB1 LIB2 ...  (LIB: path or base)
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1))
  EV=""; [ "$L" != base ] && EV="QHUFF_LIB=$(realpath $L)"
  env $EV timeout -k 10 600 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/b$i.log 2>&1 || { tail -5 $O/b$i.log; exit 1; }
  grep '"metric"' $O/b$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); h=d['extra']['host_path']
print('$L', d['value'], h['probe']['both_ms'], 'pinned', h['pinned']['ms'], h['pinned']['ms_each'], 'pageable', h['pageable']['ms'], h['pageable']['ms_each'])"
done
