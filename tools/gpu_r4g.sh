# Round 4, seventh GPU call: the GPU suite; A/B against ab/libdeltagpu_base.so (the
# previous commit) of the Merkle round (diff without its memset launch) and of the
# config-3 fold (the fill's interpolated state starts), rocprofv3, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -q --maxfail=10 --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  echo "TESTS rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20
  exit $rc
fi
DG_LIB_ANY_DIGEST=1 timeout -k 10 900 bash $R/tools/ab_prof.sh libdeltagpu_base.so tools/prof_kfold.sh 'kfold_kernel|kfold_fill' > $O/ab_kfold.txt 2>&1 || { echo AB_KFOLD_FAILED; tail -5 $O/ab_kfold.txt; exit 1; }
echo "kfold (base = this commit, var = the previous one):"; cat $O/ab_kfold.txt
cd /tmp && export TMPDIR=/tmp
for v in head base head base; do
  if [ $v = base ]; then export DG_LIB_ANY_DIGEST=1 DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_base.so; else unset DG_LIB_ANY_DIGEST DG_LIB_PATH; fi
  rm -rf $O/mk_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mk_$v -o mk -- python3 $R/tools/prof_merkle.py > $O/mk_$v.log 2>&1 || { echo PROF_MK_FAILED; tail -5 $O/mk_$v.log; exit 1; }
  echo "$v: $(python3 $R/tools/kernel_timeline.py $O/mk_$v 0 | grep -E 'diff_(count|write)|fillBuffer' | awk '{print $NF}' | tr '\n' ' ')"
  rm -f $O/mk_$v/*kernel_trace.csv
done
