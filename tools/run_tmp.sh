set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_delta.py tests/test_gpu_binding.py tests/test_gpu_mutate.py tests/test_gpu_splice.py tests/test_gpu_changes.py tests/test_gpu_merkle.py tests/test_c_marshal.py tests/test_gpu_parity.py > gpurun_out/t2.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench1.log; exit 1; }
grep '^{"metric"' gpurun_out/bench1.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); m=d['merkle']
print('headline', round(d['roofline']['frac'],4), d['roofline'].get('avg_launch_us'), 'c5', round(d['config5']['roofline']['frac'],4), 'c3', round(d['config3']['roofline']['frac'],4), 'diff', round(m['diff_roofline']['frac'],4))
print(' round_us', m.get('round_us'), 'dev', m.get('join_delta_device_us'))
mu=d.get('mutate',{})
for k in ('keys_1000','keys_10000'):
  x=mu.get(k,{}); print(' ',k, x.get('us'), 'batch', x.get('batch_1000_adds_us'), 'mutate_batch', x.get('mutate_batch_1000_adds_us'))
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pm -o pm -- python3 $R/tools/prof_merkle.py > $R/gpurun_out/pm.log 2>&1 || { echo PM_FAIL; tail -5 $R/gpurun_out/pm.log; exit 1; }
python3 $R/tools/kernel_timeline.py $R/gpurun_out/pm 14 > $R/gpurun_out/pm_tl.txt
rm -f $R/gpurun_out/*/*kernel_trace.csv
