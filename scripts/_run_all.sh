set -o pipefail
mkdir -p gpurun_out/all
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/all/test.log 2>&1
rc=$?; tail -4 gpurun_out/all/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/all/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/all/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'dec', d['extra']['decode_GiBps'], 'enc', d['extra']['encode_GiBps']); [print(k, v['avg_us']) for k, v in d['extra']['kernels'].items()]"
for k in peek11 run; do QHUFF_DECODER=$k timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path > gpurun_out/all/bench_$k.log 2>&1 || exit $?; grep '^{' gpurun_out/all/bench_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$k value', d['value'], 'dec', d['extra']['decode_GiBps'], 'enc', d['extra']['encode_GiBps'])"; done
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so QHUFF_DECODER=run timeout -k 10 120 python -u scripts/stamp_run3.py
