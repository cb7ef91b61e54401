set -o pipefail
mkdir -p gpurun_out/r05bq
i=0
for E in base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsc1only.so base QHUFF_LIB=nghttp3_amd/lib/libqhuff_vsc1only.so; do
i=$((i+1)); EV=""; [ "$E" != base ] && EV=$E
env $EV timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-path --no-pmc --c5-strings 4194304 > gpurun_out/r05bq/b$i.json 2> gpurun_out/r05bq/b$i.err || { tail -5 gpurun_out/r05bq/b$i.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05bq/b$i.json').read().strip().splitlines()[-1]); q=d['extra']['config4_qpack_blocks']
print('$E', d['value'], q['gpu_pipeline_ms'], q['kernel_avg_us_rank0'], q['bit_exact'], d['extra']['decode_GiBps'])"
done
