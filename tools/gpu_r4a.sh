# Round 4, first GPU call: the GPU suite, the default bench line, a rocprofv3 kernel summary
# of the bench's config-2 join (rotate 4), and an A/B of the Merkle build loop.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4a
O=$R/gpurun_out/r4a
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 500 python -u $R/bench.py > $O/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 $R/bench.py --no-merkle --no-configs --no-cpu-baseline --steps 400 --warmup 50 > $O/prof_c2.log 2>&1 || { echo PROF_C2_FAILED; tail -5 $O/prof_c2.log; exit 1; }
python3 $R/tools/kernel_timeline.py $O/prof_c2 0 | head -8
for v in base var base var; do
  if [ $v = var ]; then export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_DG_MERKLE_VEC0.so; else unset DG_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $O/mk_$v.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk_$v.log; exit 1; }
  echo "$v: $(python3 $R/tools/kernel_timeline.py $O/mk_$v 0 | grep -E 'chunk_kernel<true|diff_count' | tr '\n' ' ')"
  rm -rf $O/mk_$v/*/*kernel_trace.csv 2>/dev/null
done
exit $rc
