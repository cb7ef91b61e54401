set -o pipefail
mkdir -p gpurun_out/r05ag
bash dev/scripts/r05af.sh || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05ag/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --profile-only > $GRAFT_REPO_ROOT/gpurun_out/r05ag/prof.log 2>&1 ) || exit 1
head -8 gpurun_out/r05ag/prof/run_kernel_stats.csv | cut -c1-200
