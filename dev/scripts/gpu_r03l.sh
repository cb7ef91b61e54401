set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "dense or host" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K=lsorted11,sorted11,peek11s
for a in A U; do
timeout -k 10 200 python -u dev/scripts/dec_variants.py --kinds $K --alphabet $a > $O/dec_$a.log 2>&1 || { tail -5 $O/dec_$a.log; exit 1; }; grep kind $O/dec_$a.log | cut -c1-330
done
timeout -k 10 200 python -u dev/scripts/dec_variants.py --kinds $K --zipf --n 2097152 > $O/dec_Z.log 2>&1 || exit 1; grep kind $O/dec_Z.log | cut -c1-330
timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --no-host-path --steps 10 > $O/bench.log 2>&1 || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][0]); e=d['extra']; print(d['value'], e['decode_GiBps'], e['decode_dense_GiBps'], e['decode_dense_bit_exact'])"
