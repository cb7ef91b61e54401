set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04m; mkdir -p $O
for L in libqhuff.so libqhuff_ps15.so libqhuff_ps22.so; do
  echo "== $L" >> $O/dec.log
  QHUFF_LIB=nghttp3_amd/lib/$L timeout -k 10 300 python -u dev/scripts/dec_choice.py peek11s,sorted11,lsorted11 >> $O/dec.log 2>&1 || { tail -5 $O/dec.log; exit 1; }
done
cat $O/dec.log
