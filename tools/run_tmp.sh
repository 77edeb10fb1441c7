set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merkle.py tests/test_gpu_binding.py tests/test_gpu_join_delta.py tests/test_gpu_configs.py tests/test_gpu_splice.py -m gpu > gpurun_out/t/tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/t/tests.log; exit 1; }
tail -1 gpurun_out/t/tests.log
for round in 1 2; do for v in base intree; do
  if [ $v = intree ]; then unset DG_LIB_PATH DG_LIB_ANY_DIGEST; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_$v.so DG_LIB_ANY_DIGEST=1; fi
  timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/t/b_$v$round.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/t/b_$v$round.log; exit 1; }
  python3 - gpurun_out/t/b_$v$round.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
m = d["merkle"]
print(sys.argv[2], "join_delta wall %.1f dev %.1f | diff %.1f take %.1f | c2 frac %.4f" % (m["round_us"]["join_delta"], m["join_delta_device_us"], m["round_us"]["diff"], m["round_us"]["take"], d["roofline"]["frac"]))
PY
done; done
unset DG_LIB_PATH DG_LIB_ANY_DIGEST
cd /tmp && export TMPDIR=/tmp
for v in base intree; do
  if [ $v = intree ]; then unset DG_LIB_PATH DG_LIB_ANY_DIGEST; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_$v.so DG_LIB_ANY_DIGEST=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/t/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $R/gpurun_out/t/mk_$v.log 2>&1 || { echo MK_FAIL; tail -5 $R/gpurun_out/t/mk_$v.log; exit 1; }
  echo "== $v"; python3 $R/tools/kernel_timeline.py $R/gpurun_out/t/mk_$v 6 | tail -7
done
rm -f $R/gpurun_out/t/*/*kernel_trace.csv
