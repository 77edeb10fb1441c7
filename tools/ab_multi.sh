# A/B of several library builds by rocprofv3 kernel time, alternating (base first):
#   bash tools/ab_multi.sh <profile script> <kernel regex> <variant .so under ab/>...
set -o pipefail
R=$GRAFT_REPO_ROOT
S=$1; K=$2; shift 2
for round in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset DG_LIB_PATH; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$v; fi
    bash $R/$S > $R/gpurun_out/abm.txt 2>&1 || { echo FAIL $v; tail -5 $R/gpurun_out/abm.txt; exit 1; }
    echo "$v: $(grep -E "$K" $R/gpurun_out/abm.txt | grep calls | cut -c1-40,73- | tr '\n' ' ')"
  done
done
