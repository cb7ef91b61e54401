set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03lg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "long_strings" > $O/pytest_long.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest_long.log | head -20; exit 1; }
tail -1 $O/pytest_long.log
QHUFF_LONG_MIN=64 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "sorted" > $O/pytest_sorted64.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest_sorted64.log | head -20; exit 1; }
tail -1 $O/pytest_sorted64.log
timeout -k 10 400 python -u dev/scripts/long_latency.py > $O/lat.log 2>&1 || { tail -3 $O/lat.log; exit 1; }; grep case $O/lat.log
