set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3), "c3", round(d.get("config3",{}).get("ms_per_batch",0),3), "c5join", round(d.get("config5",{}).get("ms_per_join",0),4), "c5read", round(d.get("config5",{}).get("ms_per_read",0),4))'
timeout -k 10 300 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for l in $(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps); do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle ${AB_FLAGS:-} > gpurun_out/ab_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/ab_$l.log; exit 1; }
  echo -n "$l: "; python -c "$BR" < gpurun_out/ab_$l.log
done
done
