set -o pipefail
mkdir -p gpurun_out/pk1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "decoder_variants and (run or fsm)" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pk1/test.log 2>&1
rc=$?; tail -15 gpurun_out/pk1/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/dec_variants.py --kinds run,fsm,peek11 > gpurun_out/pk1/var_A.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/dec_variants.py --alphabet U --kinds run,fsm > gpurun_out/pk1/var_U.log 2>&1
rc=$?; cat gpurun_out/pk1/var_A.log gpurun_out/pk1/var_U.log | grep '^{'; exit $rc
