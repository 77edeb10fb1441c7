# rocprofv3 kernel summary + the last round's dispatch timeline of tools/prof_merkle.py
# -> gpurun_out/prof_merkle/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_merkle
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_merkle -o mk -- python3 $R/tools/prof_merkle.py $1 > $R/gpurun_out/prof_merkle/run.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_merkle/run.log; exit 1; }
tail -2 $R/gpurun_out/prof_merkle/run.log
python3 $R/tools/kernel_timeline.py $R/gpurun_out/prof_merkle 40
