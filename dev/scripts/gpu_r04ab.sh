set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qpack.py tests/test_gpu_qif.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 120 python -u dev/scripts/frame_time.py >> $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }; done
grep pipeline $O/frame.log
