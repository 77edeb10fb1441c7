# HBM traffic of the Merkle round's kernels (the diff above all) at the config-4 shard:
# rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, one pass each (MI355X_MICROARCH.md: they
# do not fit one pass), over tools/prof_merkle.py -> gpurun_out/pmc_diff/{fetch,write}
# and a per-kernel summary (per dispatch, kB; FETCH_SIZE raw: x2 for wide streaming reads
# per the guide, uncalibrated for the diff's scattered 8-B/4-B loads)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_diff
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o p -- python3 $R/tools/prof_merkle.py > $O/$c.log 2>&1 || { echo PMC_FAILED $c; tail -5 $O/$c.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, os, sys, collections
o = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(o, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) / len(v) > 100:
            print(f"{c:10s} {k:70s} dispatches={len(v):3d} per_dispatch_kB={sum(v) / len(v):12.1f}")
PY
