# A/B of diff count-kernel variants built with DG_VARIANT into delta_crdt_ex_amd/ab/:
# each passes the diff tests, then bench --no-configs (the diff's back-to-back frac) twice,
# alternating, then the config-4 round under rocprofv3 (merkle_diff_count_kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/sub; mkdir -p $O
VARS="intree DG_DIFF_NT1 DG_DIFF_NT2"
use() { if [ $1 = intree ]; then unset DG_LIB_PATH DG_LIB_ANY_DIGEST; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_$1.so DG_LIB_ANY_DIGEST=1; fi; }
for v in $VARS; do use $v
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_merkle.py -m gpu > $O/t_$v.log 2>&1 || { echo TEST_FAIL $v; tail -20 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for round in 1 2; do for v in $VARS; do use $v
  timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 5 > $O/b_$v$round.log 2>&1 || { echo BENCH_FAIL $v; tail -5 $O/b_$v$round.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/b_$v$round.log') if l.startswith('{\"metric\"')][-1]); m=d['merkle']
print('$v', 'diff frac %.4f us %.1f' % (m['diff_roofline']['frac'], m['diff_roofline']['avg_launch_us']))"
done; done
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do use $v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $O/mk_$v.log 2>&1 || { echo MK_FAIL $v; tail -5 $O/mk_$v.log; exit 1; }
  grep -h merkle_diff_count $O/mk_$v/mk_kernel_stats.csv | python3 -c "
import sys,csv
for r in csv.reader(sys.stdin): print('$v round count kernel avg %.1f min %.1f' % (float(r[3])/1e3, float(r[5])/1e3))"
done
find $O -name "*kernel_trace.csv" -delete
# FETCH per dispatch of the count kernel in the config-4 round, per build
for v in $VARS; do use $v
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o p -- python3 $R/tools/prof_merkle.py > $O/pmc_$v.log 2>&1 || { echo PMC_FAILED $v; tail -5 $O/pmc_$v.log; exit 1; }
  python3 - "$O/pmc_$v" "$v" <<'PY'
import csv, glob, os, sys
v = [float(r["Counter_Value"]) for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
     for r in csv.DictReader(open(f)) if "merkle_diff_count" in r["Kernel_Name"]]
print(sys.argv[2], "count kernel FETCH_SIZE per dispatch kB %.1f (%d dispatches)" % (sum(v) / max(len(v), 1), len(v)))
PY
done
find $O -name "*counter_collection.csv" -size +1M -delete
