set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or host" > gpurun_out/r05bt_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bt_pytest.log; [ $rc -eq 0 ] || exit 1
mkdir -p gpurun_out/r05bt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-pmc --no-configs > gpurun_out/r05bt/b1.json 2> gpurun_out/r05bt/b1.err || { tail -5 gpurun_out/r05bt/b1.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05bt/b1.json').read().strip().splitlines()[-1]); e=d['extra']
print(d['value'], d['bit_exact'], e['decode_dense_GiBps'], e['decode_dense_bit_exact'], e['decode_GiBps'], e['host_path']['pinned']['decode_GiBps_incl_h2d_d2h'])"
