set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u dev/scripts/sections_trace.py > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
cat $O/st.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $O/trace -o run -- python3 dev/scripts/sections_trace.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 dev/scripts/sections_trace.py $O/trace > $O/timeline.txt 2>&1; cat $O/timeline.txt
