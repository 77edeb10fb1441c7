# rocprofv3 kernel summary of tools/prof_read.py (read/1 on config 5's joined state, then a
# Merkle build + diff) -> gpurun_out/prof_read/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_read
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_read -o rd -- python3 $R/tools/prof_read.py > $R/gpurun_out/prof_read/run.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_read/run.log; exit 1; }
tail -2 $R/gpurun_out/prof_read/run.log
python3 $R/tools/kernel_timeline.py $R/gpurun_out/prof_read 0
