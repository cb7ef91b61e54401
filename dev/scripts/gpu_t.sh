set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; grep -E "FAIL|Error|assert" $O/pytest.log | head -20
exit $rc
