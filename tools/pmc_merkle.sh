# SQ counters of the Merkle diff count kernel and the build kernel (tools/prof_merkle.py), one pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_merkle
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "merkle_(diff_count|chunk)" --output-format csv -d $R/gpurun_out/pmc_merkle -o pm -- python3 $R/tools/prof_merkle.py $1 > $R/gpurun_out/pmc_merkle/run.log 2>&1 || { echo PMC_FAILED; tail -5 $R/gpurun_out/pmc_merkle/run.log; exit 1; }
f=$(find $R/gpurun_out/pmc_merkle -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][22:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    calls = max(n[(k, c)] for c in d)
    print(k, {c: round(v / calls) for c, v in sorted(d.items())})
PY
