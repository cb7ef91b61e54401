set -o pipefail
bash dev/scripts/benchvar.sh r05bl "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vntsc1.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsc0sc1.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vntsc1.so QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsc0sc1.so"
for i in 1 2 3 4 5 6; do python -c "
import json;d=json.loads(open('gpurun_out/r05bl/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
