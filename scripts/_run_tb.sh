#!/bin/bash
# full GPU tests, then one bench line (no extra configs)
set -o pipefail
O=gpurun_out/${TAG:-tb}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python -u bench.py --no-configs > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['extra']['kernels'].items()})"
