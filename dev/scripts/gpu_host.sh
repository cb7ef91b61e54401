set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03h3}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "host" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new old new old; do
  if [ $v = new ]; then export QHUFF_HOST_MAPPED_ENDS=1; else unset QHUFF_HOST_MAPPED_ENDS; fi
  timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --steps 5 > $O/bench_$v.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_$v.log') if l.startswith('{')][0]); print('$v', json.dumps(d['extra']['host_path']))"
done
