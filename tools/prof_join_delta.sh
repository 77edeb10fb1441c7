# rocprofv3 kernel summary + the last dispatches of tools/prof_join_delta.py -> gpurun_out/prof_jd/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_jd
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_jd -o jd -- python3 $R/tools/prof_join_delta.py $1 > $R/gpurun_out/prof_jd/run.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_jd/run.log; exit 1; }
tail -1 $R/gpurun_out/prof_jd/run.log
python3 $R/tools/kernel_timeline.py $R/gpurun_out/prof_jd 24
