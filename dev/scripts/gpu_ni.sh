set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ni; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 120 python -u dev/scripts/dec_kinds.py --only windows > $O/dec_c3_$i.log 2>&1 || exit 1; grep decoder $O/dec_c3_$i.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --steps 20 > $O/bench.log 2>&1 || { tail -3 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][0]); e=d['extra']; print(d['value'], d['ms_per_step'], e['decode_GiBps'], e['config4_qpack_blocks']['gpu_pipeline_ms'], json.dumps(e['config4_qpack_blocks']['kernel_avg_us_rank0']))"
