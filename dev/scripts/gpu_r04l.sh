set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l; mkdir -p $O
for L in libqhuff.so libqhuff_frx1.so libqhuff_frx4.so libqhuff_frx8.so libqhuff_frx12.so libqhuff.so; do
  QHUFF_LIB=nghttp3_amd/lib/$L timeout -k 10 120 python -u dev/scripts/frame_time.py >> $O/frame.log 2>&1 || { tail -5 $O/frame.log; exit 1; }
done
grep pipeline $O/frame.log
