#!/bin/bash
set -u
bash scripts/gpu_check.sh s16 test || exit $?
for a in A U; do
  timeout -k 10 120 python -u scripts/dec_variants.py --kinds peek11 --alphabet $a --reps 10 2>&1 | grep '^{'
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/b16.log 2>&1
grep '^{' gpurun_out/b16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'dec', d['extra']['decode_GiBps']); print(d['extra']['configs']); [print(k, v['avg_us']) for k, v in d['extra']['kernels'].items()]"
