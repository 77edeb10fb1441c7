# GPU suite on the default build, then the synchronous-call overhead A/B
# (tools/sync_call_time.py, config 2) of the default build against libdeltagpu_base.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for l in libdeltagpu.so libdeltagpu_base.so; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 120 python -u tools/sync_call_time.py 2>&1 | tail -1 || exit 1
done
done
