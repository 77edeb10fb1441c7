# rocprofv3 kernel trace + stats of the config-3 one-pass fold -> gpurun_out/prof_kfold/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_kfold
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kfold -o kf --output-format csv -- python -u tools/prof_kfold.py > gpurun_out/prof_kfold/run.log 2>&1 || { tail -20 gpurun_out/prof_kfold/run.log; exit 1; }
tail -3 gpurun_out/prof_kfold/run.log
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_kfold/kf_kernel_stats.csv")):
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
