# A/B of two library builds on the config-5 join loop (tools/prof_c5.py), alternating:
#   bash tools/ab_c5.sh <variant .so> [<base .so>]   (base: the default library)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in base var base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/$1;
  elif [ -n "$2" ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/$2; else unset DG_LIB_PATH; fi
  timeout -k 10 200 python -u $R/tools/prof_c5.py > $R/gpurun_out/ab_c5_$v.txt 2>&1 || { echo FAIL; tail -5 $R/gpurun_out/ab_c5_$v.txt; exit 1; }
  echo "$v: $(tail -1 $R/gpurun_out/ab_c5_$v.txt)"
done
