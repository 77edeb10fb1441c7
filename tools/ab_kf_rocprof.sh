# Per-kernel rocprof stats of the config-3 fold for each libdeltagpu build (A/B of the
# fold's kernels without the host-call noise of tools/ab_kfold.sh).
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-"libdeltagpu.so libdeltagpu_base.so"}
for l in $LIBS; do
  rm -rf gpurun_out/abkp_$l
  DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l KF_REPS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abkp_$l -o kf --output-format csv -- python -u tools/prof_kfold.py > gpurun_out/abkp_$l.log 2>&1 || { echo "$l FAILED"; tail -5 gpurun_out/abkp_$l.log; exit 1; }
  echo "== $l"
  python -c "
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/**/kf_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'kfold' in r['Name'] or 'sort' in r['Name'].lower():
        print('%-40s calls %5s avg %9.2f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))" gpurun_out/abkp_$l
done
