# The driver's N=1 command (python bench.py, no flags) four times back to back on one box
# -> gpurun_out/rep/ and one summary line per run.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/rep; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 400 python -u bench.py > $O/b$i.log 2>&1 || { echo BENCH_FAIL $i; tail -5 $O/b$i.log; exit 1; }
  grep '^{"metric"' $O/b$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); m=d['merkle']; r=d['roofline']
print('run $i headline frac %.4f (%.2f us per launch, %.4g merged dots/s) | config5 %.4f | config3 %.4f | merkle build %.3f diff %.3f | join_delta %.1f us wall, %.1f us C-ABI | steps %d warmup %d' % (r['frac'], r['avg_launch_us'], d['value'], d['config5']['roofline']['frac'], d['config3']['roofline']['frac'], m['roofline']['frac'], m['diff_roofline']['frac'], m['round_us']['join_delta'], m['join_delta_c_abi_us'], d['steps'], d['warmup']))"
done
