# A/B: the Merkle diff with subtrees of 8192 buckets and 512-thread workgroups
# (ab/libdeltagpu_DG_DIFF_WIDE1.so) against the default (4096, 256): the Merkle GPU tests on
# the variant, then the config-4 round's diff kernels under rocprofv3, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
V=$R/delta_crdt_ex_amd/ab/libdeltagpu_DG_DIFF_WIDE1.so
mkdir -p $R/gpurun_out/abw
DG_LIB_PATH=$V timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_merkle.py -q --timeout 300 --timeout-method thread -m gpu > $R/gpurun_out/abw/pytest.log 2>&1 || { echo VAR_TESTS_FAILED; tail -3 $R/gpurun_out/abw/pytest.log; exit 1; }
tail -1 $R/gpurun_out/abw/pytest.log
timeout -k 10 900 bash $R/tools/ab_prof.sh libdeltagpu_DG_DIFF_WIDE1.so tools/prof_merkle.sh 'diff_(count|write)'
