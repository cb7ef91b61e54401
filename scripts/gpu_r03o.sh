set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 120 python -u scripts/debug_encf.py > $O/dbg.log 2>&1; tail -2 $O/dbg.log
timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/enc_A.log 2>&1; grep encoder $O/enc_A.log
timeout -k 10 120 python -u scripts/enc_variants.py --only fused --alphabet U > $O/enc_U.log 2>&1; grep encoder $O/enc_U.log
timeout -k 10 200 python -u scripts/enc_variants.py --zipf --n 2097152 --only fused > $O/enc_Z.log 2>&1; grep encoder $O/enc_Z.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py -k "encoder or fused or c3_A or c2_U or config5" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
