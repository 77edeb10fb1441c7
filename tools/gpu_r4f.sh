# Round 4, sixth GPU call: the GPU suite, one full bench line (the diff's roofline from
# back-to-back dg_merkle_diff_async launches), the Merkle round's kernel summary and the
# diff-kernel phase stamps at the final sources.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  exit $rc
fi
timeout -k 10 900 python3 $R/bench.py > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['merkle']; print('headline', round(d['roofline']['frac'],4), 'c5', round(d['config5']['roofline']['frac'],4), 'c3', round(d['config3']['roofline']['frac'],4), 'build', round(m['roofline']['frac'],4), 'diff', round(m['diff_roofline']['frac'],4), m['diff_roofline']['avg_launch_us'], m['diff_roofline']['sync_call_us'], 'round', m['round_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk -o mk -- python3 $R/tools/prof_merkle.py > $O/mk.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/mk 0 > $O/mk_stats.txt; grep -E "diff|chunk_kernel<true" $O/mk_stats.txt
rm -f $O/mk/*kernel_trace.csv
timeout -k 10 300 python3 $R/tools/diff_stamps.py > $O/diff_stamps.txt 2>&1 || { echo DIFF_STAMPS_FAILED; tail -5 $O/diff_stamps.txt; exit 1; }
tail -8 $O/diff_stamps.txt
