# The headline join at the driver's --steps 20 --warmup 5 with and without the settle
# phase, alternating, against a 200-step run: where do short runs lose their microseconds?
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/settle
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for s in 0 300; do
    timeout -k 10 120 python -u bench.py --no-merkle --no-configs --no-cpu-baseline --steps 20 --warmup 5 --settle-ms $s > $O/s${s}_$i.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/s${s}_$i.log') if l.startswith('{')][-1]); r=d['roofline']; print('settle $s', 'avg', round(r['avg_launch_us'],2), 'step_med', round(r['per_step_event_median_us'],2), 'frac', round(r['frac'],4), 'ms/step', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 120 python -u bench.py --no-merkle --no-configs --no-cpu-baseline --steps 200 --warmup 20 --settle-ms 0 > $O/long.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads([l for l in open('$O/long.log') if l.startswith('{')][-1]); r=d['roofline']; print('long', 'avg', round(r['avg_launch_us'],2), 'step_med', round(r['per_step_event_median_us'],2), 'frac', round(r['frac'],4))"
