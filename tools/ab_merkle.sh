set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do for l in libdeltagpu.so libdeltagpu_DG_BASE.so; do
DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-configs > gpurun_out/mk.log 2>&1 || { echo FAIL; tail -5 gpurun_out/mk.log; exit 1; }
echo -n "$l: "; python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["merkle"]["ms_per_round"],4), "ms/merkle round", d["merkle"]["differing_keys"])' < gpurun_out/mk.log
done; done
