"""HBM traffic of the join (rocprofv3 FETCH_SIZE / WRITE_SIZE, one pass each) for the
bench workload; writes profiles/join2_pmc.json, which bench.py reports as
`roofline.traffic`.

    python tools/pmc_traffic.py            # on the GPU box (runs rocprofv3 twice)

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per L2 fabric
read request while wide streaming reads issue 128-B requests, so it reports ~1/2 of
the bytes read for 16-B/lane loads; other widths are uncalibrated.  Our loads are
8-B/lane (u64 columns) and 4-B/lane (node column), so we calibrate on a kernel with a
known byte count and the same load width: `bench.py --calibrate` runs
dg_store_check once over every input store after timing.  That kernel compares
neighbouring rows; row_cmp decides on the key column alone unless two keys are equal,
and the compiler sinks the other columns' loads behind that test, so on a config-2
store (one row per key) it reads exactly the key column from memory: 8 B/row,
8-B/lane coalesced loads (the neighbour's read is an L1/L2 hit).  The calibrated
factor comes out near the guide's 2.  WRITE_SIZE is taken as is (exact for streaming stores
per the guide).  FETCH_SIZE also counts Infinity-Cache hits (guide), so `traffic`
is bytes that left L2, an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "pmc_traffic")


def run(counter, tag, reuse=False):
    d = os.path.join(OUT, tag)
    os.makedirs(d, exist_ok=True)
    if reuse:
        return collect(d, json.load(open(os.path.join(d, "bench.json"))))
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", counter, "-d", d, "-o", tag,
           "--output-format", "csv", "--", sys.executable, "-u", "bench.py", "--steps", "16",
           "--warmup", "4", "--no-cpu-baseline", "--no-merkle", "--no-configs", "--calibrate"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, env=dict(os.environ, TMPDIR="/tmp"))
    if r.returncode != 0:
        raise SystemExit(f"rocprofv3 {counter} failed:\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    bench = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    json.dump(bench, open(os.path.join(d, "bench.json"), "w"))
    return collect(d, bench)


def collect(d, bench):
    vals = {}
    check = 0.0
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "store_check" in k:
                check += float(row["Counter_Value"])
                continue
            m = re.search(r"join2_(\w+?)_kernel", k)  # partition / stream / slot / compact
            if m:
                name = m.group(1)
                vals.setdefault(name, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, check, bench


def main():
    reuse = "--reuse" in sys.argv  # recompute from the CSVs of an earlier run
    fetch, check_kib, bench = run("FETCH_SIZE", "fetch", reuse)
    write, _, _ = run("WRITE_SIZE", "write", reuse)
    n_in = bench["config"]["rows_in_per_gpu"]
    n_out = bench["config"]["rows_out_per_gpu"]
    kib = 1024.0
    sys.path.insert(0, ROOT)
    from bench import kernel_source_digest
    res = {"rows_in": n_in, "rows_out": n_out, "kernel_sources": kernel_source_digest(),
           "fetch_kib": fetch, "write_kib": write}
    if check_kib > 0:
        known = 8.0 * bench["calib_rows"]  # key column only, see the module docstring
        factor = known / (check_kib * kib)
        res["fetch_correction"] = factor
        res["fetch_correction_source"] = ("dg_store_check over every input store: key column, "
                                          "8 B/row, 8-B/lane loads")
    else:
        factor = 2.0
        res["fetch_correction"] = factor
        res["fetch_correction_source"] = "MI355X_MICROARCH.md 16-B/lane factor (uncalibrated)"
    res["per_kernel_read_bytes"] = {k: v * kib * factor for k, v in fetch.items()}
    res["per_kernel_write_bytes"] = {k: v * kib for k, v in write.items()}
    tot_fetch = sum(fetch.values()) * kib * factor
    tot_write = sum(write.values()) * kib
    res["hbm_read_bytes_per_launch"] = tot_fetch
    res["hbm_write_bytes_per_launch"] = tot_write
    res["hbm_bytes_per_launch"] = tot_fetch + tot_write
    res["alg_bytes_per_launch"] = bench["roofline"]["alg_bytes_per_launch"]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "join2_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
