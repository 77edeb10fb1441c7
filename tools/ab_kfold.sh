# A/B of the one-pass fold across libdeltagpu builds: kfold parity tests, then the
# config-3 rate (median of KF_REPS synchronous calls) per build, twice.
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-$(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps | grep -v JOIN)}
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 300 python -u -m pytest tests/test_gpu_kfold.py -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/abk_t.log 2>&1 || echo "$l TESTS_FAILED"
  echo "$l tests: $(tail -1 gpurun_out/abk_t.log)"
done
for rep in 1 2; do
for l in $LIBS; do
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l KF_REPS=8 timeout -k 10 200 python -u tools/prof_kfold.py > gpurun_out/abk_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abk_$l.log; exit 1; }
  echo -n "$l: "; python -c "
import re,sys,statistics
v=[float(m.group(1)) for m in re.finditer(r'rep \d+: ([0-9.]+) ms', open(sys.argv[1]).read())]
print('median', round(statistics.median(v[2:]),3), 'ms  min', round(min(v),3))" gpurun_out/abk_$l.log
done
done
