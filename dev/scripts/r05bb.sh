set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dec or plan or sect or zipf or digest" > gpurun_out/r05bb_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bb_pytest.log; [ $rc -eq 0 ] || exit 1
bash dev/scripts/benchvar.sh r05bb "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_voldplan.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_voldplan.so"
