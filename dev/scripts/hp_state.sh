set -o pipefail
O=gpurun_out/r06aj; mkdir -p $O
for args in "--c5-strings 0 --c4-blocks 0" "" ; do
  timeout -k 10 600 python -u bench.py --no-cpu-baseline $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '"metric"' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); h=d['extra']['host_path']
print('$args', d['value'], h['probe']['both_ms'], 'pinned', h['pinned']['ms'], h['pinned']['ms_each'], 'pageable', h['pageable']['ms'])"
done
timeout -k 10 150 python -u dev/scripts/host_probe.py 2>&1 | grep '^{' | cut -c1-300
