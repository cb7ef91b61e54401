set -o pipefail
bash dev/scripts/benchvar.sh r05bo "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vb2.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vb3.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vb2.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vb3.so"
for i in 1 2 3 4 5 6; do python -c "
import json;d=json.loads(open('gpurun_out/r05bo/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
