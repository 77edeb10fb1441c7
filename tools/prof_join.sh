# rocprofv3 kernel trace + stats of the bench's join loop -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-join}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/prof_$TAG/bench.log 2>&1 || exit 1
python - "$TAG" <<'PY'
import csv, sys, collections
tag = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/{tag}_kernel_stats.csv")))
for r in rows:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5} avg_us={float(r["AverageNs"])/1e3:8.2f}')
tr = list(csv.DictReader(open(f"gpurun_out/prof_{tag}/{tag}_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
j = [r for r in tr if "join2" in r["Kernel_Name"]]
if len(j) > 6:
    seq = j[-6:]
    t0 = int(seq[0]["Start_Timestamp"])
    for r in seq:
        print(f'  {r["Kernel_Name"][:40]:40s} start={(int(r["Start_Timestamp"])-t0)/1e3:8.2f} dur={(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3:7.2f}')
PY
