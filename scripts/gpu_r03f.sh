set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "encoder_variants or c3_A-fused or c2_U-fused or config5" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAIL|Error|assert" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/enc_variants.py --only windows,fused > $O/enc_A.log 2>&1; cat $O/enc_A.log
timeout -k 10 120 python -u scripts/enc_variants.py --only windows,fused --alphabet U > $O/enc_U.log 2>&1; cat $O/enc_U.log
timeout -k 10 200 python -u scripts/enc_variants.py --zipf --n 2097152 --only waves,fused > $O/enc_Z.log 2>&1; cat $O/enc_Z.log
