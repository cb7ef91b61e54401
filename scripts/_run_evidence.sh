#!/bin/bash
# Round evidence (TAG = $1): parity tests, smoke, bench, rocprofv3 kernel stats of
# the main bench (profile-only) and of the full bench (framing/check/token
# kernels of the config-4 leg).
set -u
TAG=${1:-r01j}
bash scripts/gpu_check.sh ${TAG} test smoke bench prof || exit $?
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$ROOT/gpurun_out/${TAG}/prof_full" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline \
  > "$ROOT/gpurun_out/${TAG}/rocprof_full.log" 2>&1
echo "prof_full rc=$?"
