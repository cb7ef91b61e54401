set -o pipefail
QHUFF_DECODER=peek11p timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dec or digest or kat or corpus or zipf or long or err" > gpurun_out/r05bj_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05bj_pytest.log; [ $rc -eq 0 ] || exit 1
bash dev/scripts/benchvar.sh r05bj "base QHUFF_DECODER=peek11p,QHUFF_VERBOSE=1 base QHUFF_DECODER=peek11p"
for i in 1 2 3 4; do python -c "
import json;d=json.loads(open('gpurun_out/r05bj/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
