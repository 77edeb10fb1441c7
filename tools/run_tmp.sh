set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/libdeltagpu_DG_KF_NOTICKET1.so DG_LIB_ANY_DIGEST=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kfold.py > gpurun_out/t3.log 2>&1 || { echo TEST_FAIL; tail -20 gpurun_out/t3.log; exit 1; }
tail -1 gpurun_out/t3.log
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do for v in intree libdeltagpu_DG_KF_NOTICKET1.so; do
  if [ $v = intree ]; then unset DG_LIB_PATH; else export DG_LIB_PATH=$R/delta_crdt_ex_amd/ab/$v DG_LIB_ANY_DIGEST=1; fi
  KF_REPS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kf_$v$round -o kf -- python3 $R/tools/prof_kfold.py > $R/gpurun_out/kf_$v$round.log 2>&1 || { echo KF_FAIL; tail -5 $R/gpurun_out/kf_$v$round.log; exit 1; }
  echo "== $v $round"; grep -h "kfold_kernel\|kfold_fill" $R/gpurun_out/kf_$v$round/*kernel_stats.csv | cut -d, -f1-5
done; done
unset DG_LIB_PATH
rm -f $R/gpurun_out/*/*kernel_trace.csv
for ms in 0 300 0 300; do
  C5_SETTLE_MS=$ms timeout -k 10 300 python3 $R/tools/bench_c5_line.py > $R/gpurun_out/c5s_$ms.log 2>&1 || { echo C5_FAIL; exit 1; }
  python3 -c "
import json
for l in open('$R/gpurun_out/c5s_$ms.log'):
    if l.startswith('{'): d=json.loads(l); print('c5 settle_ms=$ms avg_launch_us', round(d['roofline']['avg_launch_us'],1), 'frac', round(d['roofline']['frac'],4))"
done
