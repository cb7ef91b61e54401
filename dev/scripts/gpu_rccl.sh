set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03rccl; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u bench.py --gpus 2 --one-device --dist-backend nccl --strings 65536 --steps 3 --warmup 1 --c5-strings 200000 --c4-blocks 2000 --no-cpu-baseline --no-host-path > $O/bench2.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "metric|Error|error|Duplicate" $O/bench2.log | head -8 | cut -c1-400
exit 0
