# Phase stamps of the fold and the Merkle diff at the final sources (a DG_STAMPS=1 build
# under ab/; the default library is not touched).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/stamps
timeout -k 10 300 python3 $R/tools/kfold_stamps.py > $R/gpurun_out/stamps/kfold_stamps.txt 2>&1 || { echo KF_STAMPS_FAILED; tail -5 $R/gpurun_out/stamps/kfold_stamps.txt; exit 1; }
cat $R/gpurun_out/stamps/kfold_stamps.txt
timeout -k 10 300 python3 $R/tools/diff_stamps.py > $R/gpurun_out/stamps/diff_stamps.txt 2>&1 || { echo DF_STAMPS_FAILED; tail -5 $R/gpurun_out/stamps/diff_stamps.txt; exit 1; }
cat $R/gpurun_out/stamps/diff_stamps.txt
