set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "encoder_variants or full_size_config" > gpurun_out/r03a/pytest_enc.log 2>&1
rc=$?; tail -3 gpurun_out/r03a/pytest_enc.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cpl in 1 2 4; do
QHUFF_EF_CPL=$cpl timeout -k 10 120 python -u scripts/enc_variants.py --only fused > gpurun_out/r03a/enc_A_$cpl.log 2>&1 || exit $?
echo "cpl=$cpl $(grep fused gpurun_out/r03a/enc_A_$cpl.log)"
done
QHUFF_EF_CPL=2 timeout -k 10 120 python -u scripts/enc_variants.py --only fused --alphabet U > gpurun_out/r03a/enc_U.log 2>&1 && cat gpurun_out/r03a/enc_U.log || exit $?
QHUFF_EF_CPL=2 timeout -k 10 120 python -u scripts/enc_variants.py --zipf --n 2097152 --only fused > gpurun_out/r03a/enc_Z.log 2>&1 && cat gpurun_out/r03a/enc_Z.log || exit $?
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u scripts/stamp_encf.py > gpurun_out/r03a/stamps.log 2>&1; cat gpurun_out/r03a/stamps.log
