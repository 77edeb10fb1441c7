# Config-2 join A/B of several library builds (the driver's bench settings, configs and
# Merkle off), alternating, two rounds:  bash tools/ab_c2.sh <variant .so under ab/>...
set -o pipefail
R=$GRAFT_REPO_ROOT
export DG_LIB_ANY_DIGEST=1
mkdir -p $R/gpurun_out/abc2
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in intree "$@"; do
    if [ $v = intree ]; then unset DG_LIB_PATH; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$v; fi
    timeout -k 10 300 python -u $R/bench.py --no-cpu-baseline --no-merkle --no-configs --steps 20 --warmup 5 > $R/gpurun_out/abc2/$v.log 2>&1 || { echo FAIL $v; tail -5 $R/gpurun_out/abc2/$v.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('$R/gpurun_out/abc2/$v.log') if l.startswith('{\"metric\"')][-1])
r=d['roofline']; print('$v', 'c2 avg_us %.2f frac %.4f step_med %.2f' % (r['avg_launch_us'], r['frac'], r.get('per_step_event_median_us', 0)))"
  done
done
