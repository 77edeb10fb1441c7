# Round 4, third GPU call: the GPU suite; the config-5 join with the engine created before
# or after the stores (tools/c5_order.py); the diff kernel's phase stamps
# (tools/diff_stamps.py, DG_STAMPS build); one full bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  [ $rc -eq 1 ] || exit $rc
fi
for o in engine_first data_first engine_first data_first; do
  C5_ORDER=$o timeout -k 10 300 python3 $R/tools/c5_order.py > $O/c5_order_$o.log 2>&1 || { echo C5_ORDER_FAILED; tail -5 $O/c5_order_$o.log; exit 1; }
  grep -E "^(engine|data)_first" $O/c5_order_$o.log
done
timeout -k 10 300 python3 $R/tools/diff_stamps.py > $O/diff_stamps.txt 2>&1 || { echo DIFF_STAMPS_FAILED; tail -5 $O/diff_stamps.txt; exit 1; }
cat $O/diff_stamps.txt
timeout -k 10 900 python3 $R/bench.py > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['value'], d['roofline']['frac'], 'c5', d['config5']['roofline']['frac'], 'c3', d['config3']['roofline']['frac'], 'merkle', d['merkle']['roofline']['frac'])"
exit $rc
