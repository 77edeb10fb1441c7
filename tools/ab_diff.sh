# Diff-kernel variants: each checked by the Merkle diff tests, then timed (rocprofv3 kernel
# stats of tools/prof_merkle.py) alternating with the in-tree build:
#   bash tools/ab_diff.sh <variant .so under ab/>...
set -o pipefail
R=$GRAFT_REPO_ROOT
export DG_LIB_ANY_DIGEST=1
for v in "$@"; do
  DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $R/tests/test_gpu_merkle.py -k "diff" > $R/gpurun_out/abd_$v.log 2>&1 || { echo "TESTS FAIL $v"; tail -20 $R/gpurun_out/abd_$v.log; exit 1; }
  echo "$v: $(tail -1 $R/gpurun_out/abd_$v.log)"
done
bash $R/tools/ab_multi.sh tools/prof_merkle.sh "diff_count" "$@"
