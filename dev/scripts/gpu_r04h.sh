set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u dev/scripts/host_path_trace.py > $O/hp.log 2>&1 || { tail -5 $O/hp.log; exit 1; }
cat $O/hp.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 dev/scripts/host_path_trace.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
tail -2 $O/trace.log
find $O/trace -name "*.csv" | head
QHUFF_LIB=nghttp3_amd/lib/libqhuff_frns.so timeout -k 10 120 python -u dev/scripts/frame_time.py > $O/frame_frns.log 2>&1 || { tail -5 $O/frame_frns.log; exit 1; }
timeout -k 10 120 python -u dev/scripts/frame_time.py > $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }
cat $O/frame.log $O/frame_frns.log
timeout -k 10 120 python -u dev/scripts/frame_stamps.py > $O/frame_stamps.log 2>&1 || { tail -5 $O/frame_stamps.log; exit 1; }
cat $O/frame_stamps.log
timeout -k 10 200 python -u dev/scripts/enc_choice.py windows,fused > $O/enc.log 2>&1 || { tail -5 $O/enc.log; exit 1; }
QHUFF_LIB=nghttp3_amd/lib/libqhuff_ew3.so timeout -k 10 200 python -u dev/scripts/enc_choice.py windows,fused > $O/enc3.log 2>&1 || { tail -5 $O/enc3.log; exit 1; }
cat $O/enc.log $O/enc3.log
