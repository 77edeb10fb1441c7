# GPU suite on the default build, then the join A/B (config 2 / config 5) of the default
# build against libdeltagpu_base.so.  Usage (GPU box): bash tools/ab_join2.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="libdeltagpu.so libdeltagpu_base.so" bash tools/ab_quick.sh
# config-2 join stamps (prologue split out)
C5_CONFIG=2 C5_STAMPS=gpurun_out/c2_stamps.npy DG_LIB_PATH=$PWD/delta_crdt_ex_amd/libdeltagpu_stamps.so timeout -k 10 200 python -u tools/prof_c5.py > gpurun_out/c2_stamps_run.log 2>&1 && python tools/stamps_report.py gpurun_out/c2_stamps.npy
