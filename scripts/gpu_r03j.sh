set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
for m in 0 1 3 7 15 16 48 64 127; do
  echo "abl $m"
  QHUFF_LIB=nghttp3_amd/lib/libqhuff_abl$m.so timeout -k 10 120 python -u scripts/enc_variants.py --only fused > $O/abl$m.log 2>&1 || { tail -3 $O/abl$m.log; exit 1; }
  grep encoder $O/abl$m.log
done
