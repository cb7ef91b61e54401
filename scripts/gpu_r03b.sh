set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "encoder_variants or full_size_config or decoder_variants or config5" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "PASS|FAIL|ERROR" $O/pytest.log | tail -30 | cut -c1-150
if [ $rc -ne 0 ]; then exit $rc; fi
for cpl in 2 4; do
QHUFF_EF_CPL=$cpl timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/enc_A_$cpl.log 2>&1 || exit $?
echo "cpl=$cpl $(grep fused $O/enc_A_$cpl.log)"
done
timeout -k 10 120 python -u scripts/dec_kinds.py > $O/dec_c3.log 2>&1; cat $O/dec_c3.log
timeout -k 10 200 python -u scripts/dec_kinds.py --zipf > $O/dec_c5.log 2>&1; cat $O/dec_c5.log
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u scripts/stamp_encf.py > $O/stamps.log 2>&1; cat $O/stamps.log
