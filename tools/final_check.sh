# The round's final evidence at the final sources -> gpurun_out/final/ (copy to profiles/): the headline join's
# PMC traffic (tools/pmc_traffic.py; copied into this box's profiles/ so the bench line
# below reports it), the GPU suite, one full bench line, rocprofv3 kernel summaries of
# config 2 (the bench's join loop, rotate 4), config 5 (the bench's object under
# rocprofv3: events and kernel durations of the same launches), config 3, the config-4
# round, and smoke().  Every step has its own time limit; the first failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/pmc_traffic.py > $O/pmc_traffic.log 2>&1 || { echo PMC_FAILED; tail -5 $O/pmc_traffic.log; exit 1; }
cp gpurun_out/join2_pmc.json profiles/join2_pmc.json
grep hbm_bytes_per_launch $O/pmc_traffic.log
timeout -k 10 900 python -u -m pytest tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -3 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['merkle']; print('headline', round(d['roofline']['frac'],4), d['roofline']['traffic'], 'c5', round(d['config5']['roofline']['frac'],4), 'c3', round(d['config3']['roofline']['frac'],4), 'build', round(m['roofline']['frac'],4), 'diff', round(m['diff_roofline']['frac'],4))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 $R/bench.py --no-merkle --no-configs --no-cpu-baseline --steps 400 --warmup 50 > $O/c2.log 2>&1 || { echo PROF_C2_FAILED; tail -5 $O/c2.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/c2 0 | head -4
python3 $R/tools/kernel_timeline.py $O/c2 400 join2_stream > $O/c2_timed_window.txt && cat $O/c2_timed_window.txt
grep '^{"metric"' $O/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 under rocprofv3: bench events avg_launch_us', d['roofline']['avg_launch_us'])" >> $O/c2_timed_window.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/tools/bench_c5_line.py > $O/c5.log 2>&1 || { echo PROF_C5_FAILED; tail -5 $O/c5.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/c5 0 | head -4
grep '^{"metric"' $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 events avg_launch_us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kf -o kf -- python3 $R/tools/prof_kfold.py > $O/kf.log 2>&1 || { echo PROF_KF_FAILED; tail -5 $O/kf.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/kf 0 | head -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk -o mk -- python3 $R/tools/prof_merkle.py > $O/mk.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/mk 0 | head -8
rm -f $O/*/*kernel_trace.csv
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
