set -o pipefail
mkdir -p gpurun_out/r05ba
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05ba/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --profile-only --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05ba/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05ba/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --profile-only --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05ba/p2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
ls gpurun_out/r05ba/p1 gpurun_out/r05ba/p2
