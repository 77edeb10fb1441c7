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
  [ $rc -eq 1 ] || (cd $R && timeout -k 10 400 bash tools/pmc_kfold.sh > $O/pmc_kfold.log 2>&1) || { echo PMC_KFOLD_FAILED; tail -5 $O/pmc_kfold.log; exit 1; }
cp $R/gpurun_out/kfold_pmc.txt $O/ && cat $O/kfold_pmc.txt
exit $rc
fi
for n in 1000 10000; do timeout -k 10 120 $R/c_src/_build/bench_mutate $n 300 > $O/mutate_$n.json 2> $O/mutate_$n.err || { echo MUTATE_FAILED; cat $O/mutate_$n.err; exit 1; }; cat $O/mutate_$n.json; done
# kfold: the XCD-sliced fill (default build) vs HEAD~ (ab/libdeltagpu_base.so), rocprofv3
DG_LIB_ANY_DIGEST=1 timeout -k 10 900 bash $R/tools/ab_prof.sh libdeltagpu_base.so tools/prof_kfold.sh 'kfold_kernel|kfold_fill' > $O/ab_kfold.txt 2>&1 || { echo AB_KFOLD_FAILED; tail -5 $O/ab_kfold.txt; exit 1; }
cat $O/ab_kfold.txt
cp $R/gpurun_out/prof_kfold/kf_kernel_stats.csv $O/kfold_kernel_stats.csv 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk -o mk -- python3 $R/tools/prof_merkle.py > $O/mk.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/mk 0 > $O/mk_stats.txt; head -14 $O/mk_stats.txt
# the same round on the base build (one-barrier scans and XCD-sliced kfold fill absent)
DG_LIB_ANY_DIGEST=1 DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_base.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mkbase -o mk -- python3 $R/tools/prof_merkle.py > $O/mkbase.log 2>&1 || { echo PROF_MKBASE_FAILED; tail -5 $O/mkbase.log; exit 1; }
echo "base: $(python3 $R/tools/kernel_timeline.py $O/mkbase 0 | grep -E 'diff_count' | head -1)"
echo "head: $(grep -E 'diff_count' $O/mk_stats.txt | head -1)"
rm -f $O/mkbase/*kernel_trace.csv
# diagnostic diff builds (timing only): no bounds search (EXP1), no row loads (EXP2)
for x in 2; do
  export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_DG_DIFF_EXP$x.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mkx$x -o mk -- python3 $R/tools/prof_merkle.py > $O/mkx$x.log 2>&1 || { echo PROF_MKX_FAILED; tail -5 $O/mkx$x.log; exit 1; }
  echo "EXP$x: $(python3 $R/tools/kernel_timeline.py $O/mkx$x 0 | grep -E 'diff_count' | head -1)"
  rm -f $O/mkx$x/*kernel_trace.csv
done
unset DG_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/bench_c5_line.py > $O/c5.log 2>&1 || { echo PROF_C5_FAILED; tail -5 $O/c5.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/c5 0 > $O/c5_stats.txt; head -6 $O/c5_stats.txt
grep '^{"metric"' $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 events avg_launch_us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
# A/B: stripe_sums' partials double-buffered (base) vs one buffer + barrier (var), config 5
# and config 2 joins back to back (tools/prof_c5.py), rocprofv3 kernel averages
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_DG_JOIN_RED20.so; else unset DG_LIB_PATH; fi
  for c in 5 2; do
    if [ $c = 2 ]; then export C5_CONFIG=2 C5_REPS=200; else unset C5_CONFIG; export C5_REPS=20; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_${v}_c$c -o j -- python3 $R/tools/prof_c5.py > $O/ab_${v}_c$c.log 2>&1 || { echo PROF_AB_FAILED; tail -5 $O/ab_${v}_c$c.log; exit 1; }
    echo "$v c$c: $(python3 $R/tools/kernel_timeline.py $O/ab_${v}_c$c 0 | grep -E 'join2_(stream|partition)' | awk '{print $(NF)}' | tr '\n' ' ')"
    rm -f $O/ab_${v}_c$c/*kernel_trace.csv
  done
done
unset DG_LIB_PATH C5_CONFIG C5_REPS
timeout -k 10 400 bash $R/tools/pmc_diff.sh > $O/pmc_diff.txt 2>&1 || { echo PMC_DIFF_FAILED; tail -5 $O/pmc_diff.txt; exit 1; }
grep -E "diff_count|chunk_kernel<true" $O/pmc_diff.txt
(cd $R && timeout -k 10 400 bash tools/pmc_kfold.sh > $O/pmc_kfold.log 2>&1) || { echo PMC_KFOLD_FAILED; tail -5 $O/pmc_kfold.log; exit 1; }
cp $R/gpurun_out/kfold_pmc.txt $O/ && cat $O/kfold_pmc.txt
exit $rc
