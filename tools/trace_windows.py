"""The bench's config-5 windows in a rocprofv3 kernel trace of the bench itself
(rocprofv3 --kernel-trace -- python3 bench.py ...): config 5 is the bench's last
partitioned full-state join (join2_partition_kernel + join2_stream_kernel<true, false,
false, false>); its 20 back-to-back launches (what roofline.avg_launch_us times with HIP
events) are followed by the 20 of the per-launch loop.  Prints the trace's average per
launch (partition + stream, as the bench counts them) beside the bench line's own events,
from the same process.  Usage: trace_windows.py TRACE_DIR BENCH_LOG"""
import csv
import glob
import json
import sys

d, log = sys.argv[1], sys.argv[2]
tr = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
c5 = [r for r in rows if "join2_stream_kernel<true, false, false, false>" in r["Kernel_Name"]
      or "join2_partition_kernel" in r["Kernel_Name"]]
# a join is a partition launch and a stream launch: pair them, last 40 joins
joins = []
i = 0
while i + 1 < len(c5):
    if "partition" in c5[i]["Kernel_Name"] and "stream" in c5[i + 1]["Kernel_Name"]:
        joins.append((c5[i], c5[i + 1]))
        i += 2
    else:
        i += 1
b2b = joins[-40:-20]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
kern = sum(dur(p) + dur(s) for p, s in b2b) / len(b2b)
span = (int(b2b[-1][1]["End_Timestamp"]) - int(b2b[0][0]["Start_Timestamp"])) / 1e3 / len(b2b)
line = json.loads([x for x in open(log) if x.startswith('{"metric"')][-1])
ev = line["config5"]["roofline"]["avg_launch_us"]
alg = line["config5"]["roofline"]["alg_bytes_per_launch"]
print(f"config5 (the bench's own process): events {ev:.1f} us/launch (frac {alg / ev / 8e6:.4f}); "
      f"trace kernels {kern:.1f} us (frac {alg / kern / 8e6:.4f}), trace span {span:.1f} us per join")
