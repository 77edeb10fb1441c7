# The diff's phase stamps with the CU and XCC of every subtree workgroup (a stamps build
# that records them, ab/libdeltagpu_stamps.so, built from a patched copy of the sources).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/stamps
DG_LIB_ANY_DIGEST=1 timeout -k 10 300 python3 $R/tools/diff_stamps.py > $R/gpurun_out/stamps/diff_where.txt 2>&1 || { echo DF_STAMPS_FAILED; tail -5 $R/gpurun_out/stamps/diff_where.txt; exit 1; }
cat $R/gpurun_out/stamps/diff_where.txt
