# Round evidence for profiles/<tag>/: rocprofv3 kernel trace + stats of the bench's join
# loop, the FETCH_SIZE/WRITE_SIZE traffic passes, and one full default bench line.
# Usage (on the GPU box):  bash tools/profile_round.sh r1
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/profiles_$TAG
mkdir -p $OUT
bash tools/prof_join.sh $TAG > $OUT/prof_summary.txt 2>&1 || { cat $OUT/prof_summary.txt; exit 1; }
cp gpurun_out/prof_$TAG/${TAG}_kernel_stats.csv $OUT/join2_kernel_stats.csv
cat $OUT/prof_summary.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/pmc_traffic.py > $OUT/pmc_traffic.log 2>&1 || { tail -20 $OUT/pmc_traffic.log; exit 1; }
cp gpurun_out/join2_pmc.json $OUT/join2_pmc.json
cp gpurun_out/pmc_traffic/fetch/*counter_collection.csv $OUT/join2_fetch_size.csv
cp gpurun_out/pmc_traffic/write/*counter_collection.csv $OUT/join2_write_size.csv
mkdir -p profiles && cp $OUT/join2_pmc.json profiles/join2_pmc.json  # (box-side copy for the bench below; locally, copy gpurun_out/profiles_TAG/join2_pmc.json to profiles/ afterwards)
timeout -k 10 400 python -u bench.py > $OUT/bench_full.log 2>&1 || { tail -20 $OUT/bench_full.log; exit 1; }
tail -1 $OUT/bench_full.log
