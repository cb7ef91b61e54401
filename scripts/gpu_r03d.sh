set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "encoder_variants or c3_A-fused or c2_U-fused" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cpl in 1 2 4; do
QHUFF_EF_CPL=$cpl timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/enc_A_$cpl.log 2>&1 || exit $?
echo "cpl=$cpl $(grep fused $O/enc_A_$cpl.log)"
done
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u scripts/stamp_encf.py > $O/stamps.log 2>&1; cat $O/stamps.log
