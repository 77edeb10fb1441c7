# rocprofv3 kernel averages of tools/prof_merkle.py for the default build and every
# experiment build (libdeltagpu_*.so): A/B of Merkle kernel variants.
set -o pipefail
R=$GRAFT_REPO_ROOT
for lib in $R/delta_crdt_ex_amd/libdeltagpu*.so; do
  case $lib in *stamps*) continue;; esac
  d=$R/gpurun_out/abm_$(basename $lib .so)
  mkdir -p $d
  (cd /tmp && export TMPDIR=/tmp && DG_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o mk -- python3 $R/tools/prof_merkle.py $1 > $d/run.log 2>&1) || { echo "$lib PROF_FAILED"; tail -5 $d/run.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $(basename $lib)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "merkle" in r["Name"]:
        print(f'  {r["Name"][22:70]:48s} calls={r["Calls"]:>4} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
done
