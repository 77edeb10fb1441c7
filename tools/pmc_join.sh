# PMC counters of the join kernels (separate rocprofv3 passes, no trace domains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc -o pass$i --output-format csv -- python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/pmc/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/pass$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc/pass*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "join2" not in k:
            continue
        import re
        m = re.search(r"(join2_\w+)", k)
        name = m.group(1) if m else k[:40]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        # per dispatch: counters are reported per dispatch (summed over instances)
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
