# Bench each experiment build of libdeltagpu (DG_LIB_PATH) in the current join mode.
set -o pipefail
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],1), "us/launch", round(d["roofline"]["frac"],3))'
for lib in delta_crdt_ex_amd/libdeltagpu*.so; do
  case $lib in *stamps*) continue;; esac
  DG_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/v.log 2>&1 || { echo "$lib FAILED"; tail -5 gpurun_out/v.log; exit 1; }
  echo -n "$lib: "; python -c "$BR" < gpurun_out/v.log
done
