# rocprofv3 kernel summary + the last dispatches of the config-5 join loop (tools/prof_c5.py)
# -> gpurun_out/prof_c5/ ; extra arguments: environment for prof_c5.py is inherited
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_c5
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5 -- python3 $R/tools/prof_c5.py > $R/gpurun_out/prof_c5/run.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_c5/run.log; exit 1; }
tail -1 $R/gpurun_out/prof_c5/run.log
python3 $R/tools/kernel_timeline.py $R/gpurun_out/prof_c5 8
