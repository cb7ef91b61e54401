#!/bin/bash
# Round-4 final evidence on one box: GPU tests, smoke, two bench runs,
# rocprofv3 kernel stats, FETCH/WRITE PMC passes, the encoder choice and the
# config-4 pipelines' kernel/copy timeline.  Every GPU step has its own time
# limit; a failing step ends the script (gpu_check.sh stops on crashes).
set -u
TAG=${1:-r04final}
OUT=gpurun_out/$TAG
bash dev/scripts/gpu_check.sh $TAG test smoke bench prof pmc || exit $?
timeout -k 10 300 python bench.py > $OUT/bench2.log 2>&1 || exit $?
grep '^{' $OUT/bench2.log > $OUT/bench2.json
timeout -k 10 300 python -u dev/scripts/enc_choice.py windows,fused,auto > $OUT/enc.log 2>&1 || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace \
    --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sec -o run -- python3 $GRAFT_REPO_ROOT/dev/scripts/sections_trace.py ) \
    > $OUT/sec.log 2>&1 || exit $?
python3 dev/scripts/sections_trace.py $OUT/sec > $OUT/sections_timeline.txt 2>&1
echo done
