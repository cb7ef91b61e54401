set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u dev/scripts/host_path_trace.py > $O/hp.log 2>&1 || { tail -5 $O/hp.log; exit 1; }
cat $O/hp.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 dev/scripts/host_path_trace.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
timeout -k 10 120 python -u dev/scripts/frame_time.py > $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }
cat $O/frame.log
timeout -k 10 120 python -u dev/scripts/frame_stamps.py > $O/frame_stamps.log 2>&1 || { tail -5 $O/frame_stamps.log; exit 1; }
cat $O/frame_stamps.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print(d['value'], d['ms_per_step']); print(json.dumps(e['host_path'])[:600]); print(json.dumps(e['config4_qpack_blocks'].get('kernel_avg_us_rank0')), e['config4_qpack_blocks'].get('gpu_pipeline_ms'))"
