set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u dev/scripts/dense_times.py > $O/dense.log 2>&1 || { tail -5 $O/dense.log; exit 1; }
cat $O/dense.log
timeout -k 10 120 python -u dev/scripts/host_path_trace.py > $O/hp.log 2>&1 || { tail -5 $O/hp.log; exit 1; }
cat $O/hp.log
