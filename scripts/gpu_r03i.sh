set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 120 python -u scripts/debug_encf.py > $O/dbg.log 2>&1; tail -2 $O/dbg.log
timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/enc_A.log 2>&1; cat $O/enc_A.log
timeout -k 10 120 python -u scripts/enc_variants.py --only fused --alphabet U > $O/enc_U.log 2>&1; cat $O/enc_U.log
timeout -k 10 200 python -u scripts/enc_variants.py --zipf --n 2097152 --only fused > $O/enc_Z.log 2>&1; cat $O/enc_Z.log
QHUFF_LIB=nghttp3_amd/lib/libqhuff_stamps.so timeout -k 10 120 python -u scripts/stamp_encw.py > $O/stamp.log 2>&1; cat $O/stamp.log
