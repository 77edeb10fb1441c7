# SQ instruction / wait counters of the config-3 fold kernels (tools/prof_kfold.py), one
# pass -> gpurun_out/kfold_sq.txt (per dispatch, per wave)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_kfold_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
KF_REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --kernel-include-regex "kfold_kernel" --output-format csv -d $O -o pm -- python3 $R/tools/prof_kfold.py > $O/run.log 2>&1 || { echo PMC_FAILED; tail -5 $O/run.log; exit 1; }
python3 - $O <<'PY' | tee $R/gpurun_out/kfold_sq.txt
import csv, sys, glob, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = {c: v / n[c] for c, v in acc.items()}
w = d.get("SQ_WAVES", 1)
print("# kfold_kernel, config 3 (tools/prof_kfold.py), rocprofv3 --pmc, per dispatch and per wave")
for c in sorted(d):
    print(f"{c:24s} {d[c]:16.0f}  per wave {d[c] / w:10.1f}")
PY
