# Concurrent joins of two engines with and without the cooperative launch, and the
# config-2 / config-5 join rates of both launch kinds.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],2), "us/launch", round(d["roofline"]["frac"],3))'
for c in 0 1; do
  DG_JOIN_COOP=$c timeout -k 10 200 python -u -m pytest tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/coop_$c.log 2>&1
  echo "coop=$c concurrency test rc=$? $(tail -1 gpurun_out/coop_$c.log)"
done
for rep in 1 2; do for c in 0 1; do
  DG_JOIN_COOP=$c timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/coopb.log 2>&1 || { echo "bench coop=$c FAILED"; tail -5 gpurun_out/coopb.log; exit 1; }
  echo -n "coop=$c c2: "; python -c "$BR" < gpurun_out/coopb.log
  DG_JOIN_COOP=$c timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/coopc5.log 2>&1 || { echo "c5 coop=$c FAILED"; tail -5 gpurun_out/coopc5.log; exit 1; }
  echo -n "coop=$c c5: "; tail -1 gpurun_out/coopc5.log
done; done
