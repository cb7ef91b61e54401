set -o pipefail
mkdir -p gpurun_out/r05s
R=$GRAFT_REPO_ROOT
timeout -k 10 60 dev/ubench/wr_half > gpurun_out/r05s/plain.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05s/f -o run -- $R/dev/ubench/wr_half > $R/gpurun_out/r05s/f.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r05s/w -o run -- $R/dev/ubench/wr_half > $R/gpurun_out/r05s/w.txt 2>&1 || exit 1
cd $R; cat gpurun_out/r05s/plain.txt; python3 dev/scripts/pmc_summary.py gpurun_out/r05s
