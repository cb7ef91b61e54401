set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u dev/scripts/enc_choice.py windows,fused,auto > $O/enc.log 2>&1 || { tail -5 $O/enc.log; exit 1; }
grep case $O/enc.log
