# A/B of two library builds on config 5 by rocprofv3 kernel time (tools/prof_c5.sh):
#   bash tools/ab_prof_c5.sh <variant .so>      (base: the default library)
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/$1; else unset DG_LIB_PATH; fi
  bash $R/tools/prof_c5.sh > $R/gpurun_out/abp_$v.txt 2>&1 || { echo FAIL; tail -5 $R/gpurun_out/abp_$v.txt; exit 1; }
  echo "$v: $(grep -E 'partition.*calls' $R/gpurun_out/abp_$v.txt | cut -c60-) | $(grep -E 'stream_kernel.*calls' $R/gpurun_out/abp_$v.txt | cut -c60-)"
done
