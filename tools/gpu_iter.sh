# One GPU iteration: the full GPU parity suite on the default build, then for the default
# build and every experiment build (libdeltagpu_DG*.so): join parity + bench in both join
# modes (MODES: 1 = single-pass stream kernel, the default; 2 = two-pass), join stamps of the default build,
# and a rocprofv3 kernel summary of the default bench.
set -o pipefail
mkdir -p gpurun_out
BR='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]/1e9,2), "Gdots/s", round(d["roofline"]["avg_launch_us"],1), "us/launch", round(d["roofline"]["frac"],3))'
timeout -k 10 400 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for lib in delta_crdt_ex_amd/libdeltagpu.so delta_crdt_ex_amd/libdeltagpu_DG*.so; do
  [ -e "$lib" ] || continue
  for mode in ${MODES:-1}; do
    DG_JOIN_MODE=$mode DG_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread -m gpu -k "join or golden" > gpurun_out/v_tests.log 2>&1 || { echo "$lib mode $mode TESTS_FAILED"; tail -30 gpurun_out/v_tests.log; exit 1; }
    DG_JOIN_MODE=$mode DG_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-merkle --no-configs > gpurun_out/v.log 2>&1 || { echo "$lib FAILED"; tail -5 gpurun_out/v.log; exit 1; }
    echo -n "$lib mode $mode ($(tail -1 gpurun_out/v_tests.log)): "; python -c "$BR" < gpurun_out/v.log
    if [ -n "$PROF_ALL" ]; then
      DG_JOIN_MODE=$mode DG_LIB_PATH=$PWD/$lib bash tools/prof_join.sh v > gpurun_out/prof_v.txt 2>&1 || { tail -5 gpurun_out/prof_v.txt; exit 1; }
      grep join2 gpurun_out/prof_v.txt | grep avg_us | sed 's/(dg::.*calls/ calls/'
    fi
  done
done
for mode in ${MODES:-1}; do
  echo "stamps mode $mode"; DG_JOIN_MODE=$mode C5_CONFIG=2 C5_STAMPS=gpurun_out/c2_stamps_$mode.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/libdeltagpu_stamps.so timeout -k 10 120 python -u tools/prof_c5.py && python tools/stamps_report.py gpurun_out/c2_stamps_$mode.npy || exit 1
done
bash tools/prof_join.sh iter > gpurun_out/prof_iter.txt 2>&1 || { tail -5 gpurun_out/prof_iter.txt; exit 1; }
head -8 gpurun_out/prof_iter.txt
