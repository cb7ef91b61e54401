set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dec or plan or sect or zipf or digest or kat or corpus" > gpurun_out/r05bd_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bd_pytest.log; [ $rc -eq 0 ] || exit 1
bash dev/scripts/benchvar.sh r05bd "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vnopre.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vnopre.so"
