set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03x}; mkdir -p $O profiles/r03
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
fi
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 300 python -u dev/scripts/decoder_steps.py ${TAG:-r03x} > $O/steps.log 2>&1 || { tail -5 $O/steps.log; exit 1; }
cp $O/decoder_steps.json profiles/r03/
timeout -k 10 120 ./dev/ubench/lds_chain > $O/lds_chain.txt 2>&1 || exit 1
tail -1 $O/lds_chain.txt > profiles/r03/lds_chain.json; cp profiles/r03/lds_chain.json $O/
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep metric $O/bench.log > $O/bench.json; head -c 1500 $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --profile-only --no-configs --no-cpu-baseline --no-host-path > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -2
