# Round 4, second GPU call: the GPU suite; the Merkle round under rocprofv3 (build, diff);
# the mutate bench; config 5's bench line under rocprofv3 (events vs kernel durations).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  [ $rc -eq 1 ] || exit $rc
fi
for n in 1000 10000; do timeout -k 10 120 $R/c_src/_build/bench_mutate $n 300 > $O/mutate_$n.json 2> $O/mutate_$n.err || { echo MUTATE_FAILED; cat $O/mutate_$n.err; exit 1; }; cat $O/mutate_$n.json; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk -o mk -- python3 $R/tools/prof_merkle.py > $O/mk.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/mk 0 > $O/mk_stats.txt; head -14 $O/mk_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/bench_c5_line.py > $O/c5.log 2>&1 || { echo PROF_C5_FAILED; tail -5 $O/c5.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/c5 0 > $O/c5_stats.txt; head -6 $O/c5_stats.txt
grep '^{"metric"' $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 events avg_launch_us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
exit $rc
