set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u dev/scripts/dec_choice.py peek11s,sorted11 > $O/dec.log 2>&1 || { tail -5 $O/dec.log; exit 1; }
grep case $O/dec.log
timeout -k 10 120 python -u dev/scripts/frame_time.py > $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }
cat $O/frame.log
