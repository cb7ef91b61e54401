#!/bin/bash
# A/B libraries on one box: bench (config 3 kernels, same-run counters, the
# encode / decode / cold legs) per library, each under its own time limit.
#   dev/scripts/ab_lib.sh OUTDIR LIB1 LIB2 ...   (LIB: path or "base")
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for L in "$@"; do
  i=$((i+1))
  EV=""; [ "$L" != base ] && EV="QHUFF_LIB=$(realpath $L)"
  env $EV timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-path --c5-strings 0 --c4-blocks 0 > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1])
k=d['extra']['kernels']; r=d['roofline']; e=d['extra']
print('$L', d['value'], d['ms_per_step'], {n: v['avg_us'] for n,v in k.items()}, r.get('traffic'),
      {x: e.get(x) for x in ('encode_GiBps','decode_GiBps','decode_dense_GiBps','encode_cold_GiBps','decode_cold_GiBps')})"
done
