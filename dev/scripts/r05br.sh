set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dec or sect or digest or corpus or kat or long or err or frame" > gpurun_out/r05br_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05br_pytest.log; [ $rc -eq 0 ] || exit 1
mkdir -p gpurun_out/r05br
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-path --no-pmc --c5-strings 4194304 > gpurun_out/r05br/b1.json 2> gpurun_out/r05br/b1.err || { tail -5 gpurun_out/r05br/b1.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r05br/b1.json').read().strip().splitlines()[-1]); q=d['extra']['config4_qpack_blocks']
print(d['value'], d['bit_exact'], q['gpu_pipeline_ms'], q['kernel_avg_us_rank0'], q['bit_exact'], d['extra']['decode_GiBps'], {n: v['avg_us'] for n,v in d['extra']['kernels'].items()})"
