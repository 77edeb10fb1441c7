# kfold_kernel on config 3: phase stamps (default build, then the half-bucket build if
# present), then SQ counters (three rocprofv3 --pmc passes, no trace domains).
# Usage (GPU box): bash tools/kfold_probe.sh  -> gpurun_out/kfold_sq_counters.txt
set -o pipefail
mkdir -p gpurun_out
for l in libdeltagpu_stamps.so libdeltagpu_stamps_DG_KFOLD_BLOCK512_DG_KFOLD_SCALE1_DG_KFOLD_NSUB256.so; do
  [ -e delta_crdt_ex_amd/$l ] || continue
  echo "== stamps $l"
  KF_STAMPS_LIB=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u tools/kfold_stamps.py > gpurun_out/kfst_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/kfst_$l.log; exit 1; }
  cat gpurun_out/kfst_$l.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  KF_REPS=3 timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/kfpmc -o pass$i --output-format csv -- python -u tools/prof_kfold.py > gpurun_out/kf_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/kf_pmc$i.log; exit 1; }
done
python - > gpurun_out/kfold_sq_counters.txt <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/kfpmc/**/pass*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(kfold_\w+)", r["Kernel_Name"])
        if m:
            agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("# rocprofv3 --pmc SQ counters per dispatch, config-3 fold (tools/prof_kfold.py), 3 passes")
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
cat gpurun_out/kfold_sq_counters.txt
