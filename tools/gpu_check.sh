# One GPU call: the GPU test suite, then the default bench line.  Usage: bash tools/gpu_check.sh
# Test failures (rc 1) still let the bench run; a crash, abort or time limit ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q --maxfail=5 --timeout 600 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
  [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
exit $rc
