# Round 4: A/B of ab/libdeltagpu_dev.so (a build of the dev branch: the Merkle build's
# loads of a step issued together, the diff write kernel's loads issued together) against
# the default library -- first the Merkle GPU tests on the dev build, then the config-4
# round under rocprofv3, alternating, then bench's Merkle object on both.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h
mkdir -p $O
DEV=$R/delta_crdt_ex_amd/ab/libdeltagpu_dev.so
DG_LIB_ANY_DIGEST=1 DG_LIB_PATH=$DEV timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_merkle.py $R/tests/test_gpu_term_trees.py $R/tests/test_gpu_join_delta.py -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_dev.log 2>&1 || { echo DEV_TESTS_FAILED; tail -3 $O/pytest_dev.log; grep -E "^(FAILED|ERROR)" $O/pytest_dev.log | head; exit 1; }
tail -1 $O/pytest_dev.log
cd /tmp && export TMPDIR=/tmp
for v in head dev head dev; do
  if [ $v = dev ]; then export DG_LIB_ANY_DIGEST=1 DG_LIB_PATH=$DEV; else unset DG_LIB_ANY_DIGEST DG_LIB_PATH; fi
  rm -rf $O/mk_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $O/mk_$v.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk_$v.log; exit 1; }
  echo "$v: $(python3 $R/tools/kernel_timeline.py $O/mk_$v 0 | grep -E 'chunk_kernel<true|diff_count|diff_write' | awk '{print $NF}' | tr '\n' ' ')"
  rm -f $O/mk_$v/*kernel_trace.csv
done
