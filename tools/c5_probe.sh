# Config-5 join investigation: wall rate, rocprofv3 kernel stats, stamps, SQ counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/c5/rate.log 2>&1 || { tail -20 gpurun_out/c5/rate.log; exit 1; }
cat gpurun_out/c5/rate.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -o c5 --output-format csv -- python -u tools/prof_c5.py > gpurun_out/c5/prof.log 2>&1 || { tail -20 gpurun_out/c5/prof.log; exit 1; }
python -c "
import csv
for r in csv.DictReader(open('gpurun_out/c5/c5_kernel_stats.csv')):
    print(f'{r[\"Name\"][:60]:60s} calls={r[\"Calls\"]:>5} avg_us={float(r[\"AverageNs\"])/1e3:9.2f}')
"
C5_STAMPS=gpurun_out/c5/stamps.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/libdeltagpu_stamps.so timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/c5/stamps.log 2>&1 || { tail -20 gpurun_out/c5/stamps.log; exit 1; }
python tools/stamps_report.py gpurun_out/c5/stamps.npy
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  C5_REPS=5 timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/c5/pmc -o pass$i --output-format csv -- python -u tools/prof_c5.py > gpurun_out/c5/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/c5/pmc$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/c5/pmc/pass*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(join2_\w+)", r["Kernel_Name"])
        if not m: continue
        agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
