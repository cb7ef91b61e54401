set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r05k/pytest_gpu.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r05k/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r05k/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r05k/bench.json 2> gpurun_out/r05k/bench.err || { tail -20 gpurun_out/r05k/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r05k/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_us'],d['extra']['kernels'])"
