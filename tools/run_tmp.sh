set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_delta.py tests/test_gpu_binding.py tests/test_gpu_mutate.py > gpurun_out/t2.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
bash tools/c5_control.sh
