# A/B of an experiment build against the default one on the config-4 round profile:
#   bash tools/ab_variant.sh <variant .so name> <kernel regex>
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$1; else if [ -n "$3" ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$3; else unset DG_LIB_PATH; fi; fi
  bash $R/tools/prof_merkle.sh > $R/gpurun_out/ab_$v.txt 2>&1 || { echo FAIL; tail -5 $R/gpurun_out/ab_$v.txt; exit 1; }
  echo "$v: $(grep -E "$2" $R/gpurun_out/ab_$v.txt | head -1 | cut -c60-)"
done
