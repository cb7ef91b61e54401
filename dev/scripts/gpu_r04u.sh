set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qpack.py tests/test_gpu_qif.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
exit $rc
