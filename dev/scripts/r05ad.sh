set -o pipefail
mkdir -p gpurun_out/r05ad
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ad/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r05ad/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05ad/smoke.log 2>&1 || { tail -5 gpurun_out/r05ad/smoke.log; exit 1; }
tail -1 gpurun_out/r05ad/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r05ad/bench.json 2> gpurun_out/r05ad/bench.err || { tail -20 gpurun_out/r05ad/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05ad/bench.json').read().strip().splitlines()[-1])
print(d['value'],d['ms_per_step'],d['roofline']['avg_us'],d['roofline']['traffic_over_algo'])"
