# Config-5 join A/B of library builds (bench.config5_rate alone: the 12.5M-key shard, HIP
# events around back-to-back joins), alternating, two rounds:
#   bash tools/ab_c5.sh <variant .so under ab/>...
set -o pipefail
R=$GRAFT_REPO_ROOT
export DG_LIB_ANY_DIGEST=1
mkdir -p $R/gpurun_out/abc5
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in intree "$@"; do
    if [ $v = intree ]; then unset DG_LIB_PATH; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$v; fi
    timeout -k 10 300 python -u $R/tools/bench_c5_line.py > $R/gpurun_out/abc5/$v.log 2>&1 || { echo FAIL $v; tail -5 $R/gpurun_out/abc5/$v.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$R/gpurun_out/abc5/$v.log') if l.startswith('{')][-1])
r=d['roofline']; print('$v', 'c5 avg_us %.2f frac %.4f' % (r['avg_launch_us'], r['frac']))"
  done
done
