timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/b1.log 2>&1 || exit $?
grep '^{' gpurun_out/b1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'dec', d['extra']['decode_GiBps'], 'enc', d['extra']['encode_GiBps']); [print(k, v['avg_us']) for k, v in d['extra']['kernels'].items()]"
