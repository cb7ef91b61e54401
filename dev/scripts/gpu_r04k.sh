set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
for L in libqhuff.so libqhuff.so; do
  QHUFF_LIB=nghttp3_amd/lib/$L timeout -k 10 120 python -u dev/scripts/frame_time.py >> $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }
done
grep pipeline $O/frame.log
timeout -k 10 120 python -u dev/scripts/host_path_trace.py > $O/hp.log 2>&1 || { tail -5 $O/hp.log; exit 1; }
cat $O/hp.log
