set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dec or digest or kat or corpus or zipf or long or err or sect" > gpurun_out/r05bm_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bm_pytest.log; [ $rc -eq 0 ] || exit 1
bash dev/scripts/benchvar.sh r05bm "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vldnt.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vldsc1.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vldnt.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vldsc1.so"
for i in 1 2 3 4 5 6; do python -c "
import json;d=json.loads(open('gpurun_out/r05bm/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
