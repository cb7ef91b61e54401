set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qpack.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --no-host-path > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']; c4=e['config4_qpack_blocks']
print(d['value'], c4['encoder_gpu_ms'], c4['encoder_bit_exact'], c4['encoder_kernel_us_per_call_rank0'], c4['gpu_pipeline_ms'])"
