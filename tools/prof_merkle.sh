# rocprofv3 kernel summary of tools/prof_merkle.py -> gpurun_out/prof_merkle/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_merkle
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_merkle -o mk -- python3 $R/tools/prof_merkle.py $1 > $R/gpurun_out/prof_merkle/run.log 2>&1 || { echo PROF_FAILED; tail -5 $R/gpurun_out/prof_merkle/run.log; exit 1; }
tail -2 $R/gpurun_out/prof_merkle/run.log
f=$(find $R/gpurun_out/prof_merkle -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
