# Changed-key path per build: the changes tests, then config-2 changes_rate and the
# config-4 round (keyed join with changes), twice.
set -o pipefail
mkdir -p gpurun_out
LIBS=$(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps)
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u -m pytest tests/test_gpu_changes.py tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread -m gpu -x > gpurun_out/abc_t.log 2>&1 || { echo "$l TESTS_FAILED"; tail -30 gpurun_out/abc_t.log; exit 1; }
  echo "$l tests: $(tail -1 gpurun_out/abc_t.log)"
done
for rep in 1 2; do
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abc_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abc_$l.log; exit 1; }
  echo -n "$l: "; python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['merkle']; c=d['changes']
print('changes', round(c['us_per_call'],1), 'join2', round(c['join2_us_per_call'],1), 'round', {k: round(v,1) for k,v in m['round_us'].items()})" gpurun_out/abc_$l.log
done
done
