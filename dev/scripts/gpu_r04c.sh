set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qpack.py tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "long or sections or config4 or netbsd" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error|assert" $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u dev/scripts/long_latency.py sections > $O/lat_sections.log 2>&1 || { tail -5 $O/lat_sections.log; exit 1; }
cat $O/lat_sections.log
timeout -k 10 600 python -u dev/scripts/long_latency.py > $O/lat.log 2>&1 || { tail -5 $O/lat.log; exit 1; }
cat $O/lat.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'], d['cpu_baseline']['tall']['round_trip_min_med_max']); print(json.dumps(d['extra'].get('config4_qpack_blocks'))[:600])"
