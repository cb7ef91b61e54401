set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_qpack.py -x -q --timeout 120 --timeout-method thread -k "dense or host" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u dev/scripts/dense_times.py > $O/dense.log 2>&1 || { tail -3 $O/dense.log; exit 1; }; cat $O/dense.log | grep dense
timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --steps 10 > $O/bench.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][0]); e=d['extra']; print(d['value'], e['decode_GiBps'], e['decode_dense_GiBps'], e['decode_dense_bit_exact'], json.dumps(e['host_path']))"
