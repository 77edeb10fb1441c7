# rocprofv3 kernel summary of tools/prof_read.py (read/1 on config 5, Merkle build + diff).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rd -o run -- python3 $R/tools/prof_read.py > $R/gpurun_out/prof_rd.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_rd.log; exit 1; }
f=$(find $R/gpurun_out/prof_rd -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/read_merkle_kernel_stats.csv; cut -d, -f1-4 $f | cut -c1-170 | head -20
