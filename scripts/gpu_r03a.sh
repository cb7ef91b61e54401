set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "encoder_variants or full_size_config" > gpurun_out/r03a/pytest_enc.log 2>&1
rc=$?; tail -3 gpurun_out/r03a/pytest_enc.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/enc_variants.py --only windows,fused > gpurun_out/r03a/enc_A.log 2>&1 && cat gpurun_out/r03a/enc_A.log || exit $?
timeout -k 10 120 python -u scripts/enc_variants.py --only windows,fused --alphabet U > gpurun_out/r03a/enc_U.log 2>&1 && cat gpurun_out/r03a/enc_U.log || exit $?
timeout -k 10 120 python -u scripts/enc_variants.py --zipf --n 2097152 --only waves,fused > gpurun_out/r03a/enc_Z.log 2>&1 && cat gpurun_out/r03a/enc_Z.log
