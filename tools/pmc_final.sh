set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 bash $R/tools/pmc_diff.sh > $R/gpurun_out/pmc_diff_final.txt 2>&1 || { echo PMC_DIFF_FAILED; tail -5 $R/gpurun_out/pmc_diff_final.txt; exit 1; }
grep -E "diff_count|diff_write|chunk_kernel" $R/gpurun_out/pmc_diff_final.txt
