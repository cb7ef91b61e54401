set -o pipefail
bash dev/scripts/benchvar.sh r05bu "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vlnt.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vlnt.so"
for i in 1 2 3 4; do python -c "
import json;d=json.loads(open('gpurun_out/r05bu/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
