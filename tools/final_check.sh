# The round's final evidence at the final sources -> gpurun_out/final/ (copy to profiles/):
# the headline join's PMC traffic (tools/pmc_traffic.py; copied into this box's profiles/
# so the bench line below reports it), the GPU suite, one bench line as the driver runs it,
# rocprofv3 kernel summaries of the bench ITSELF (config 3, the config-4 round with
# dg_join_delta's one-wait path, config 5's windows beside the same process's events:
# tools/trace_windows.py), of config 2's timed window (400 launches), the Merkle round's
# FETCH/WRITE per kernel (tools/pmc_diff.sh), and smoke().  Every step has its own time
# limit; the first failure ends the call.
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
grep '^{"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['merkle']; print('headline', round(d['roofline']['frac'],4), d['roofline']['traffic'], 'c5', round(d['config5']['roofline']['frac'],4), 'c3', round(d['config3']['roofline']['frac'],4), 'build', round(m['roofline']['frac'],4), 'diff', round(m['diff_roofline']['frac'],4), 'join_delta', m['round_us']['join_delta'], m['join_delta_device_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_prof -o bp -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_prof.log 2>&1 || { echo PROF_BENCH_FAILED; tail -5 $O/bench_prof.log; exit 1; }
python3 $R/tools/trace_windows.py $O/bench_prof $O/bench_prof.log | tee $O/c5_window.txt
python3 $R/tools/kernel_timeline.py $O/bench_prof 0 | head -40 > $O/bench_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 $R/bench.py --no-merkle --no-configs --no-cpu-baseline --steps 400 --warmup 50 > $O/c2.log 2>&1 || { echo PROF_C2_FAILED; tail -5 $O/c2.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/c2 400 join2_stream > $O/c2_timed_window.txt && cat $O/c2_timed_window.txt
grep '^{"metric"' $O/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 under rocprofv3: bench events avg_launch_us', d['roofline']['avg_launch_us'])" >> $O/c2_timed_window.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk -o mk -- python3 $R/tools/prof_merkle.py > $O/mk.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/mk 14 > $O/mk_timeline.txt
bash $R/tools/pmc_diff.sh > $O/pmc_diff.txt 2>&1 || { echo PMC_DIFF_FAILED; tail -5 $O/pmc_diff.txt; exit 1; }
find $O $R/gpurun_out/pmc_diff -name "*kernel_trace.csv" -delete 2>/dev/null; true
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
