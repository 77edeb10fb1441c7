# A/B of a library build against the base on the bench's own numbers, alternating:
#   bash tools/ab_bench.sh <variant .so under ab/> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
V=$1; shift
mkdir -p $R/gpurun_out/abb
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$V; else unset DG_LIB_PATH; fi
  timeout -k 10 300 python -u $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/abb/$v.log 2>&1 || { echo FAIL $v; tail -5 $R/gpurun_out/abb/$v.log; exit 1; }
  python3 - $R/gpurun_out/abb/$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
r = d["roofline"]
out = [sys.argv[2], "c2 avg_us %.2f frac %.4f" % (r["avg_launch_us"], r["frac"])]
for k in ("config5", "config3"):
    if k in d:
        out.append("%s frac %.4f us %.1f" % (k, d[k]["roofline"]["frac"], d[k]["roofline"].get("avg_launch_us", 0)))
if "merkle" in d:
    m = d["merkle"]
    out.append("build %.4f diff %.4f" % (m["roofline"]["frac"], m["diff_roofline"]["frac"]))
print(" | ".join(out))
PY
done
