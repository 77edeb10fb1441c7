# Config-4 round (merkle build/diff, take, keyed join with changes, update) per build.
set -o pipefail
mkdir -p gpurun_out
LIBS=$(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps)
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs > gpurun_out/abc4_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abc4_$l.log; exit 1; }
  echo -n "$l: "; python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['merkle']
print('build_us', round(m['build_us'],1), 'frac', round(m['roofline']['frac'],3), 'round_us', {k: round(v,1) for k,v in m['round_us'].items()}, 'changes', d.get('changes',{}).get('us_per_call'), 'join2', d.get('changes',{}).get('join2_us_per_call'))" gpurun_out/abc4_$l.log
done
