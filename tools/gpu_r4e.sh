# Round 4, fifth GPU call: the GPU suite; the Merkle diff A/B (default build vs
# ab/libdeltagpu_base.so, rocprofv3, alternating) and the diff-kernel phase stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4e
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for v in head base head base; do
  if [ $v = base ]; then export DG_LIB_ANY_DIGEST=1 DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_base.so; else unset DG_LIB_ANY_DIGEST DG_LIB_PATH; fi
  rm -rf $O/mk_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $O/mk_$v.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk_$v.log; exit 1; }
  echo "$v: $(python3 $R/tools/kernel_timeline.py $O/mk_$v 0 | grep -E 'diff_count' | head -1)"
  rm -f $O/mk_$v/*kernel_trace.csv
done
unset DG_LIB_ANY_DIGEST DG_LIB_PATH
timeout -k 10 300 python3 $R/tools/diff_stamps.py > $O/diff_stamps.txt 2>&1 || { echo DIFF_STAMPS_FAILED; tail -5 $O/diff_stamps.txt; exit 1; }
cat $O/diff_stamps.txt
for cfg in "0 0" "6 0" "0 1" "6 1"; do
  set -- $cfg
  C5_WARM=$1 C5_DEL=$2 timeout -k 10 300 python3 $R/tools/c5_order.py > $O/c5_order_$1_$2.log 2>&1 || { echo C5_ORDER_FAILED; tail -5 $O/c5_order_$1_$2.log; exit 1; }
  grep -E "^engine_first" $O/c5_order_$1_$2.log
done
