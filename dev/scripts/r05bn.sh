set -o pipefail
bash dev/scripts/benchvar.sh r05bn "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsrcnt.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsrcnt.so"
for i in 1 2 3 4; do python -c "
import json;d=json.loads(open('gpurun_out/r05bn/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
