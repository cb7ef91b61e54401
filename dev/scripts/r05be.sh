set -o pipefail
bash dev/scripts/benchvar.sh r05bf "base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vp2.so,QHUFF_DECODER=peek11s2,QHUFF_VERBOSE=1 base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vp2.so,QHUFF_DECODER=peek11s2"
for i in 1 2 3 4; do python -c "
import json;d=json.loads(open('gpurun_out/r05bf/b$i.json').read().strip().splitlines()[-1]); print($i, d['bit_exact'])"; done
grep -h "numRegs\|peek11s2" gpurun_out/r05bf/b2.err | sort -u | head
