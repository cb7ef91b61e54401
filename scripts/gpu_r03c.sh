set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "sorted" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/dec_kinds.py --only windows,sorted > $O/dec_c3.log 2>&1; cat $O/dec_c3.log
timeout -k 10 200 python -u scripts/dec_kinds.py --zipf --only sorted > $O/dec_c5.log 2>&1; cat $O/dec_c5.log
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u scripts/stamp_encf.py > $O/stamps.log 2>&1; cat $O/stamps.log
