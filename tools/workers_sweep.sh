# Join grid sweep on config 2 (DG_JOIN_WORKERS = persistent workgroups; unset = the occupancy
# query's resident count), plus a rocprofv3 kernel summary of the default launch.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3))'
for w in "" 256 384 448 512; do
  DG_JOIN_WORKERS=$w timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/ws.log 2>&1 || { echo "workers=$w FAILED"; tail -5 gpurun_out/ws.log; exit 1; }
  echo -n "workers=${w:-default}: "; python -c "$BR" < gpurun_out/ws.log
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ws -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-merkle --no-configs > $GRAFT_REPO_ROOT/gpurun_out/prof_ws.log 2>&1 || { echo PROF_FAILED; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_ws.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_ws -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -c1-160 {} | head -8'
