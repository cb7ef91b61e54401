set -o pipefail
mkdir -p gpurun_out/r05bh
for L in libqhuff libqhuff_vlw0 libqhuff libqhuff_vlw0; do
QHUFF_LIB=nghttp3_amd/lib/$L.so timeout -k 10 120 python -u dev/scripts/lens_time.py > gpurun_out/r05bh/$L.log 2>&1 || { tail -3 gpurun_out/r05bh/$L.log; exit 1; }
tail -1 gpurun_out/r05bh/$L.log
done
ALPH=U QHUFF_LIB=nghttp3_amd/lib/libqhuff.so timeout -k 10 120 python -u dev/scripts/lens_time.py | tail -1
ALPH=U QHUFF_LIB=nghttp3_amd/lib/libqhuff_vlw0.so timeout -k 10 120 python -u dev/scripts/lens_time.py | tail -1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "enc or count or digest or kat or corpus or sect" > gpurun_out/r05bh_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bh_pytest.log; exit $rc
