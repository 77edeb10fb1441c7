# PMC passes over the config-4 round's kernels (tools/prof_merkle.py): SQ counters, then
# FETCH_SIZE, then WRITE_SIZE (separate passes: rocprofv3 does not split counters).
# -> gpurun_out/pmc_round/  (FETCH_SIZE is in kB; on gfx950 double it for 16-B/lane
# streaming reads, MI355X_MICROARCH.md; 8-B scattered reads count their 64-B requests)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_round
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
RX="merkle_diff_count|splice_kernel|take_keys|merkle_update_kernel|merkle_chunk"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d $O/p$i -o pm -- python3 $R/tools/prof_merkle.py > $O/run$i.log 2>&1 || { echo PMC_FAILED $i; tail -5 $O/run$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][22:64]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / max(n[(k, c)], 1)) for c, v in sorted(d.items())})
PY
