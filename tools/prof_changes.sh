# GPU parity suite, then a rocprofv3 kernel summary of dg_join2 vs dg_join2_changes (config 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_chg -o run -- python3 $R/tools/prof_changes.py > $R/gpurun_out/prof_chg.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_chg.log; exit 1; }
grep "us/call" $R/gpurun_out/prof_chg.log
f=$(find $R/gpurun_out/prof_chg -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/changes_kernel_stats.csv; cut -d, -f1-4 $f | cut -c1-150 | head -10
