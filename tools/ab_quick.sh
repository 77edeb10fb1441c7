# Quick A/B of the join rate (config 2 bench line, config-5 loop) across builds, twice.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3))'
LIBS=${LIBS:-$(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps)}
for rep in 1 2; do
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/abq_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abq_$l.log; exit 1; }
  echo -n "$l c2: "; python -c "$BR" < gpurun_out/abq_$l.log
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/abq_c5_$l.log 2>&1 || { echo "$l c5 FAILED"; tail -5 gpurun_out/abq_c5_$l.log; exit 1; }
  echo -n "$l c5: "; tail -1 gpurun_out/abq_c5_$l.log
done
done
