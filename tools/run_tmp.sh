set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_delta.py tests/test_gpu_binding.py tests/test_gpu_mutate.py tests/test_gpu_parity.py tests/test_gpu_splice.py tests/test_gpu_changes.py tests/test_gpu_concurrency.py > gpurun_out/t2.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_stamps.so DG_LIB_ANY_DIGEST=1 C5_CONFIG=2 C5_REPS=20 C5_STAMPS=gpurun_out/c2_stamps.npy timeout -k 10 120 python tools/prof_c5.py > gpurun_out/c2_stamps.log 2>&1 || { echo ST_FAIL; tail -5 gpurun_out/c2_stamps.log; exit 1; }
python tools/stamps_report.py gpurun_out/c2_stamps.npy >> gpurun_out/c2_stamps.log
