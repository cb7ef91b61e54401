set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03lg2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "long_strings or decoder_variants or full_size_config or dense" > $O/pytest_long.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest_long.log | head -20; exit 1; }
tail -1 $O/pytest_long.log
timeout -k 10 400 python -u dev/scripts/long_latency.py > $O/lat.log 2>&1 || { tail -3 $O/lat.log; exit 1; }; grep case $O/lat.log | cut -c1-200
timeout -k 10 120 python -u dev/scripts/dec_kinds.py --only windows > $O/dec_c3.log 2>&1 || exit 1; grep decoder $O/dec_c3.log | cut -c1-250
