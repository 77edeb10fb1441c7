# GPU suite, then the synchronous-call times (bare C-ABI and the Python mirror).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do timeout -k 10 120 python -u tools/sync_call_time.py 2>&1 | tail -2 || exit 1; done
