set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 600 python -u bench.py > gpurun_out/r05o/bench.json 2> gpurun_out/r05o/bench.err || { tail -30 gpurun_out/r05o/bench.err; exit 1; }
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05o/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --profile-only > $GRAFT_REPO_ROOT/gpurun_out/r05o/prof.log 2>&1 ) || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r05o/bench.json').read().strip().splitlines()[-1])
print(d['value'],d['ms_per_step'],json.dumps(d['roofline']));print(json.dumps(d['extra']['counters']))"
find gpurun_out/r05o/prof -name '*kernel_stats.csv' | head -2
