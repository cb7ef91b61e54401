set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|^E " $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u dev/scripts/enc_choice.py windows,fused,auto > $O/enc.log 2>&1 || { tail -5 $O/enc.log; exit 1; }
grep case $O/enc.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-host-path > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep "^{" $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print(d['value'], d['ms_per_step'], json.dumps(e['config3_alphabet_U']), json.dumps({k: v for k, v in e['config5_zipf'].items() if 'GiBps' in k}), e['config4_qpack_blocks']['encoder_gpu_ms'])"
