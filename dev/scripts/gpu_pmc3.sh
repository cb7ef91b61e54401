set -u
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r03p2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/encf_$ctr -o run -- python3 $GRAFT_REPO_ROOT/dev/scripts/enc_variants.py --only fused --reps 2 > $O/encf_$ctr.log 2>&1 || { tail -3 $O/encf_$ctr.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $O/encfz_$ctr -o run -- python3 $GRAFT_REPO_ROOT/dev/scripts/enc_variants.py --only fused --zipf --n 2097152 --reps 2 > $O/encfz_$ctr.log 2>&1 || { tail -3 $O/encfz_$ctr.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/decs_$ctr -o run -- python3 $GRAFT_REPO_ROOT/dev/scripts/dec_kinds.py --only sorted --reps 2 > $O/decs_$ctr.log 2>&1 || { tail -3 $O/decs_$ctr.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $O/decsz_$ctr -o run -- python3 $GRAFT_REPO_ROOT/dev/scripts/dec_kinds.py --only sorted --zipf --reps 2 > $O/decsz_$ctr.log 2>&1 || { tail -3 $O/decsz_$ctr.log; exit 1; }
done
echo done
