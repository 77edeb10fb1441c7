# One GPU iteration: parity tests, join stamps, bench of the default build and of any
# experiment builds (libdeltagpu_DG*.so).
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],1), "us/launch", round(d["roofline"]["frac"],3))'
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
DG_JOIN_MODE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k join > gpurun_out/gpu_tests2.log 2>&1 || { echo TESTS2_FAILED; tail -30 gpurun_out/gpu_tests2.log; exit 1; }
tail -1 gpurun_out/gpu_tests2.log
timeout -k 10 120 python -u tools/join_stamps.py || exit 1
DG_JOIN_MODE=1 timeout -k 10 120 python -u tools/join_stamps.py || exit 1
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle > gpurun_out/bench1.log 2>&1 || exit 1
echo -n "default: "; python -c "$BR" < gpurun_out/bench1.log
DG_JOIN_MODE=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle > gpurun_out/bench2.log 2>&1 || exit 1
echo -n "single-pass mode: "; python -c "$BR" < gpurun_out/bench2.log
for lib in delta_crdt_ex_amd/libdeltagpu_DG*.so; do
  [ -e "$lib" ] || continue
  DG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k join > gpurun_out/v_tests.log 2>&1 || { echo "$lib TESTS_FAILED"; tail -30 gpurun_out/v_tests.log; exit 1; }
  DG_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle > gpurun_out/v.log 2>&1 || { echo "$lib FAILED"; tail -5 gpurun_out/v.log; exit 1; }
  echo -n "$lib: "; python -c "$BR" < gpurun_out/v.log
done
bash tools/prof_join.sh iter > gpurun_out/prof_iter.txt 2>&1 || { tail -5 gpurun_out/prof_iter.txt; exit 1; }
head -8 gpurun_out/prof_iter.txt
