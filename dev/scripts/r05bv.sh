set -o pipefail
mkdir -p gpurun_out/r05bv
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05bv/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r05bv/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05bv/smoke.log 2>&1 || { tail -5 gpurun_out/r05bv/smoke.log; exit 1; }
tail -1 gpurun_out/r05bv/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r05bv/bench.json 2> gpurun_out/r05bv/bench.err || { tail -20 gpurun_out/r05bv/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05bv/bench.json').read().strip().splitlines()[-1])
print(d['value'],d['ms_per_step'],d['roofline']['avg_us'],d['roofline']['traffic_over_algo'])"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05bv/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --profile-only > $GRAFT_REPO_ROOT/gpurun_out/r05bv/prof.log 2>&1 ) || exit 1
head -8 gpurun_out/r05bv/prof/run_kernel_stats.csv | cut -c1-200
