set -o pipefail
mkdir -p gpurun_out/c5
for k in 12500000 1000000; do
C5_KEYS=$k C5_STAMPS=gpurun_out/c5/stamps_$k.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/libdeltagpu_stamps.so timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/c5/stamps.log 2>&1 || { tail -20 gpurun_out/c5/stamps.log; exit 1; }
echo "keys $k"; python tools/stamps_report.py gpurun_out/c5/stamps_$k.npy
done
