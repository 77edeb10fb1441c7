# A/B of two library builds by rocprofv3 kernel time: bash tools/ab_prof.sh <variant .so> <profile script> <kernel regex>
#   e.g. bash tools/ab_prof.sh libdeltagpu_X.so tools/prof_kfold.sh 'kfold_kernel|kfold_fill'
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$1; else unset DG_LIB_PATH; fi
  bash $R/$2 > $R/gpurun_out/abk_$v.txt 2>&1 || { echo FAIL; tail -5 $R/gpurun_out/abk_$v.txt; exit 1; }
  echo "$v: $(grep -E "$3" $R/gpurun_out/abk_$v.txt | grep calls | cut -c1-30,60- | tr '\n' ' ')"
done
