# Round-2 evidence -> gpurun_out/profiles_r2/ (copy to profiles/r2/ afterwards):
#   the GPU test log; rocprofv3 kernel summaries of the config-2 bench join loop, the
#   config-5 join loop, the config-3 fold and the config-4 Merkle round; the join's
#   FETCH_SIZE / WRITE_SIZE traffic (profiles/join2_pmc.json for the bench); config-5 SQ
#   counters; config-5 join stamps (needs libdeltagpu_stamps.so); one full bench line.
# Usage (on the GPU box):  bash tools/profile_round2.sh
set -o pipefail
OUT=gpurun_out/profiles_r2
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/ -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
# config-2 join loop
bash tools/prof_join.sh r2 > $OUT/prof_join.txt 2>&1 || { cat $OUT/prof_join.txt; exit 1; }
cp gpurun_out/prof_r2/r2_kernel_stats.csv $OUT/join2_kernel_stats.csv
head -4 $OUT/prof_join.txt
cd /tmp && export TMPDIR=/tmp && cd $R
# config-5 join loop
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python -u tools/prof_c5.py > $OUT/c5_run.log 2>&1 || { tail -20 $OUT/c5_run.log; exit 1; }
cp gpurun_out/prof_c5/c5_kernel_stats.csv $OUT/c5_kernel_stats.csv
tail -1 $OUT/c5_run.log
# config-3 fold
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kf -o kf --output-format csv -- python -u tools/prof_kfold.py > $OUT/kfold_run.log 2>&1 || { tail -20 $OUT/kfold_run.log; exit 1; }
cp gpurun_out/prof_kf/kf_kernel_stats.csv $OUT/kfold_kernel_stats.csv
# config-4 Merkle round
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mk -o mk --output-format csv -- python -u tools/prof_merkle.py > $OUT/merkle_run.log 2>&1 || { tail -20 $OUT/merkle_run.log; exit 1; }
cp gpurun_out/prof_mk/mk_kernel_stats.csv $OUT/merkle_kernel_stats.csv
# join traffic (two PMC passes), then the PMC summary the bench reads
timeout -k 10 400 python -u tools/pmc_traffic.py > $OUT/pmc_traffic.log 2>&1 || { tail -20 $OUT/pmc_traffic.log; exit 1; }
cp gpurun_out/join2_pmc.json $OUT/join2_pmc.json
mkdir -p profiles && cp $OUT/join2_pmc.json profiles/join2_pmc.json
# config-5 SQ counters (three passes, no trace domains)
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  C5_REPS=5 timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/c5pmc -o pass$i --output-format csv -- python -u tools/prof_c5.py > $OUT/c5_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/c5_pmc$i.log; exit 1; }
done
python - > $OUT/c5_sq_counters.txt <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/c5pmc/pass*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(join2_\w+)", r["Kernel_Name"])
        if m:
            agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("# rocprofv3 --pmc SQ counters per dispatch, config-5 join loop (tools/prof_c5.py), 3 passes")
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
# config-5 join stamps
if [ -e delta_crdt_ex_amd/ab/libdeltagpu_stamps.so ]; then
  C5_STAMPS=gpurun_out/c5_stamps.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/ab/libdeltagpu_stamps.so timeout -k 10 200 python -u tools/prof_c5.py > $OUT/c5_stamps_run.log 2>&1 || { tail -20 $OUT/c5_stamps_run.log; exit 1; }
  python tools/stamps_report.py gpurun_out/c5_stamps.npy > $OUT/c5_stamps.txt
fi
# config-2 join stamps (the bench's fused path)
if [ -e delta_crdt_ex_amd/ab/libdeltagpu_stamps.so ]; then
  C5_CONFIG=2 C5_STAMPS=gpurun_out/c2_stamps.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/ab/libdeltagpu_stamps.so timeout -k 10 200 python -u tools/prof_c5.py > $OUT/c2_stamps_run.log 2>&1 || { tail -20 $OUT/c2_stamps_run.log; exit 1; }
  python tools/stamps_report.py gpurun_out/c2_stamps.npy > $OUT/c2_stamps.txt
fi
# read/1 (segmented reduction) on config 5's joined state + a Merkle build/diff
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rd -o rd --output-format csv -- python -u tools/prof_read.py > $OUT/read_run.log 2>&1 || { tail -20 $OUT/read_run.log; exit 1; }
cp gpurun_out/prof_rd/rd_kernel_stats.csv $OUT/read_merkle_kernel_stats.csv
# the full default bench line (reads profiles/join2_pmc.json for `traffic`)
timeout -k 10 600 python -u bench.py > $OUT/bench_full.log 2>&1 || { tail -20 $OUT/bench_full.log; exit 1; }
tail -1 $OUT/bench_full.log
