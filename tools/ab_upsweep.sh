# A/B: the chunk upsweep in one block barrier (default build) against ab/libdeltagpu_base.so
# (eleven barriers): the Merkle GPU tests on the default, then the config-4 round under
# rocprofv3, alternating (the build's and the update's chunk kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abu
timeout -k 10 900 python -u -m pytest $R/tests/test_gpu_merkle.py $R/tests/test_gpu_term_trees.py $R/tests/test_gpu_join_delta.py $R/tests/test_gpu_configs.py -q --timeout 600 --timeout-method thread -m gpu > $R/gpurun_out/abu/pytest.log 2>&1 || { echo TESTS_FAILED; tail -3 $R/gpurun_out/abu/pytest.log; grep -E "^(FAILED|ERROR)" $R/gpurun_out/abu/pytest.log | head; exit 1; }
tail -1 $R/gpurun_out/abu/pytest.log
DG_LIB_ANY_DIGEST=1 timeout -k 10 900 bash $R/tools/ab_prof.sh libdeltagpu_base.so tools/prof_merkle.sh 'chunk_kernel'
