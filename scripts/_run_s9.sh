#!/bin/bash
for d in 0 4; do
  echo "== QHUFF_DEBUG=$d"
  QHUFF_DEBUG=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --steps 5 --warmup 2 > gpurun_out/b_$d.log 2>&1
  grep '^{' gpurun_out/b_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value']); [print(k, v['avg_us']) for k, v in d['extra']['kernels'].items() if 'enc' in k]"
done
