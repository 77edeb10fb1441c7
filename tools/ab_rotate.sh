# Join A/B at a larger rotation (ROT distinct replica pairs, so the inputs far exceed the
# 256 MB Infinity Cache): every libdeltagpu*.so in the tree.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3))'
for rep in 1 2; do
for l in $(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps); do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs --rotate ${ROT:-8} > gpurun_out/ab_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/ab_$l.log; exit 1; }
  echo -n "rotate ${ROT:-8} $l: "; python -c "$BR" < gpurun_out/ab_$l.log
done
done
