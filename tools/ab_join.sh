# A/B of the join kernel across libdeltagpu builds (default + libdeltagpu_DG*.so):
# join parity tests once per build, then alternating config-2 bench and config-5 rate.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3))'
LIBS=$(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps)
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -m gpu -k "join or golden or config" > gpurun_out/abj_t.log 2>&1 || { echo "$l TESTS_FAILED"; tail -30 gpurun_out/abj_t.log; exit 1; }
  echo "$l tests: $(tail -1 gpurun_out/abj_t.log)"
done
for rep in 1 2; do
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/abj_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abj_$l.log; exit 1; }
  echo -n "$l c2: "; python -c "$BR" < gpurun_out/abj_$l.log
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/abj_c5_$l.log 2>&1 || { echo "$l c5 FAILED"; tail -5 gpurun_out/abj_c5_$l.log; exit 1; }
  echo -n "$l c5: "; tail -1 gpurun_out/abj_c5_$l.log
done
done
