"""Per-kernel stats and the last N dispatches (start offset, duration, gap before) of a
rocprofv3 --kernel-trace --output-format csv directory.  Usage: kernel_timeline.py DIR [N]

    kernel_timeline.py DIR N REGEX   the average and median duration of the LAST N
                                     dispatches whose name matches REGEX: the timed window
                                     of a bench run (the summary's average also counts its
                                     settle and warm-up launches, at lower clocks)"""
import csv
import glob
import os
import re
import signal
import statistics
import sys

signal.signal(signal.SIGPIPE, signal.SIG_DFL)  # (piped into head: end quietly)

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if len(sys.argv) > 3:
    pat = re.compile(sys.argv[3])
    rows = sorted((r for r in csv.DictReader(open(trace[0])) if pat.search(r["Kernel_Name"])),
                  key=lambda r: int(r["Start_Timestamp"]))[-n:]
    d_us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    print(f"window: last {len(d_us)} of /{sys.argv[3]}/: avg_us={statistics.fmean(d_us):.2f} "
          f"median_us={statistics.median(d_us):.2f} min_us={min(d_us):.2f} max_us={max(d_us):.2f}")
    sys.exit(0)
if stats:
    for r in csv.DictReader(open(stats[0])):
        print(f'{r["Name"][:72]:72s} calls={r["Calls"]:>5} avg_us={float(r["AverageNs"]) / 1e3:9.2f}')
if trace:
    rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    prev = None
    print(f"--- last {len(rows)} dispatches (us: start, duration, gap after the previous end)")
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:8.1f}  {r["Kernel_Name"][:80]}')
        prev = e
