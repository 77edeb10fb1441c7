# HBM traffic of the config-3 one-pass fold per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE,
# one pass each, tools/prof_kfold.py); FETCH_SIZE scaled by the calibrated factor in
# profiles/join2_pmc.json (tools/pmc_traffic.py).  Output: gpurun_out/kfold_pmc.txt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/kfpmc_$c
  KF_REPS=4 timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/kfpmc_$c -o p --output-format csv -- python -u tools/prof_kfold.py > gpurun_out/kfpmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/kfpmc_$c.log; exit 1; }
done
python - <<'PY' | tee gpurun_out/kfold_pmc.txt
import csv, glob, json, re
f = json.load(open("profiles/join2_pmc.json"))["fetch_correction"]
print(f"# config-3 one-pass fold (tools/prof_kfold.py), rocprofv3 --pmc per dispatch; FETCH_SIZE x {f:.3f} (calibrated, tools/pmc_traffic.py), WRITE_SIZE as is")
for c, scale in (("FETCH_SIZE", f), ("WRITE_SIZE", 1.0)):
    v = {}
    for p in glob.glob(f"gpurun_out/kfpmc_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            m = re.search(r"(kfold_\w+?)\(", r["Kernel_Name"])
            if m:
                v.setdefault(m.group(1), []).append(float(r["Counter_Value"]))
    for k, x in sorted(v.items()):
        print(f"{c:10s} {k:18s} dispatches {len(x):3d}  MB per launch {sum(x) / len(x) * 1024 * scale / 1e6:9.1f}")
PY
