# One GPU call for the end of a round, at the final sources: the GPU test suite and the
# bench line (tools/gpu_check.sh), the headline join's PMC traffic (tools/pmc_traffic.py ->
# gpurun_out/join2_pmc.json), then the kernel profiles the DESIGN numbers cite.  Every step
# has its own time limit; the first failure ends the call.
#   bash tools/final_check.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_check.sh || exit $?
timeout -k 10 400 python -u tools/pmc_traffic.py > gpurun_out/pmc_traffic.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/pmc_traffic.log; exit 1; }
echo "pmc traffic: $(grep hbm_bytes_per_launch gpurun_out/pmc_traffic.log)"
bash tools/prof_c5.sh > gpurun_out/final_c5.txt 2>&1 || { echo C5_PROF_FAILED; exit 1; }
bash tools/prof_merkle.sh > gpurun_out/final_round.txt 2>&1 || { echo ROUND_PROF_FAILED; exit 1; }
bash tools/prof_join_delta.sh > gpurun_out/final_jd.txt 2>&1 || { echo JD_PROF_FAILED; exit 1; }
bash tools/prof_kfold.sh > gpurun_out/final_kfold.txt 2>&1 || { echo KFOLD_PROF_FAILED; exit 1; }
echo FINAL_OK
