set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
for d in 128 384 640 1152 1920; do
QHUFF_DEBUG=$d QHUFF_EF_CPL=2 timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/enc_$d.log 2>&1 || exit $?
echo "dbg=$d $(grep fused $O/enc_$d.log | cut -c1-200)"
done
