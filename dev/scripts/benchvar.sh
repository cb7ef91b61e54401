# usage: bash dev/scripts/benchvar.sh OUTDIR "ENV1 ENV2 ..." (ENV: VAR=val,VAR2=val or "base")
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
i=0
for E in $2; do
i=$((i+1))
EV=""; [ "$E" != base ] && EV=$(echo $E | tr ',' ' ')
env $EV timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-path --no-pmc --no-configs > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
python -c "
import json,sys;d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1])
k=d['extra']['kernels']; print('$E', d['value'], d['ms_per_step'], {n: v['avg_us'] for n,v in k.items()})"
done
