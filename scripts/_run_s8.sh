#!/bin/bash
set -u
bash scripts/gpu_check.sh s8 test || exit $?
QHUFF_VERBOSE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --steps 5 --warmup 2 > gpurun_out/b1.log 2>&1
grep qhuff gpurun_out/b1.log | sort | uniq
grep '^{' gpurun_out/b1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'dec', d['extra']['decode_GiBps'], 'enc', d['extra']['encode_GiBps']); [print(k, v['avg_us']) for k, v in d['extra']['kernels'].items()]"
