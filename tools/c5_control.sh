# does the profiler's presence slow the persistent config-5 join, or does the
# bench's event clock disagree with the kernel trace?  One box, the same process shape:
# the bench's config-5 object (20 event-timed launches) without and under rocprofv3
# --kernel-trace, for the persistent single-pass join and for a control that does not
# wait on other workgroups (the two-pass kernels, DG_JOIN_MODE=2), alternating twice.
# -> gpurun_out/c5ctl/ (summary.txt)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5ctl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for mode in 1 2; do
    tag=m${mode}_r${round}
    DG_JOIN_MODE=$mode timeout -k 10 300 python3 $R/tools/bench_c5_line.py > $O/plain_$tag.log 2>&1 || { echo C5_PLAIN_FAIL; tail -5 $O/plain_$tag.log; exit 1; }
    DG_JOIN_MODE=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o c5 -- python3 $R/tools/bench_c5_line.py > $O/prof_$tag.log 2>&1 || { echo C5_PROF_FAIL; tail -5 $O/prof_$tag.log; exit 1; }
    python3 - "$O" "$tag" "$mode" <<'PY' >> $O/summary.txt
import csv, glob, json, sys
o, tag, mode = sys.argv[1:4]
def ev(path):
    for l in open(path):
        if l.startswith("{"):
            d = json.loads(l)
            return d["roofline"]["avg_launch_us"]
plain = ev(f"{o}/plain_{tag}.log")
prof = ev(f"{o}/prof_{tag}.log")
tr = glob.glob(f"{o}/prof_{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
# the timed launches: the last 20 joins (single pass: stream [+ partition]; two pass: partition + slot + compact)
names = ("join2_stream", "join2_partition") if mode == "1" else ("join2_partition", "join2_slot", "join2_compact")
js = [r for r in rows if any(n in r["Kernel_Name"] for n in names)]
per = len(set(r["Kernel_Name"] for r in js[-12:])) if mode == "1" else 3
sel = js[-40 * per:-20 * per]  # the 20 back-to-back launches the events time (the per-launch loop follows)
tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel) / 1e3 / 20
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / 20
print(f"{tag} mode={'single-pass' if mode == '1' else 'two-pass'} events_plain_us={plain:.1f} "
      f"events_under_profiler_us={prof:.1f} trace_kernel_sum_us={tot:.1f} trace_span_us={span:.1f} "
      f"profiler_cost={100 * (prof / plain - 1):+.1f}%")
PY
    rm -f $O/prof_$tag/*/*kernel_trace.csv $O/prof_$tag/*kernel_trace.csv
  done
done
cat $O/summary.txt
