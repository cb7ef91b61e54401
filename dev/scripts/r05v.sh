set -o pipefail
mkdir -p gpurun_out/r05v
R=$GRAFT_REPO_ROOT
timeout -k 10 60 dev/ubench/rd_gran > gpurun_out/r05v/plain.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r05v/f -o run -- $R/dev/ubench/rd_gran > $R/gpurun_out/r05v/f.txt 2>&1 || exit 1
cd $R; cat gpurun_out/r05v/plain.txt; python3 dev/scripts/pmc_summary.py gpurun_out/r05v
