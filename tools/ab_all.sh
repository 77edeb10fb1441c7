# GPU suite on the default build, then the join (config 2 / config 5) and kfold (config
# 3) A/B of the default build against libdeltagpu_base.so (the committed HEAD, built
# aside).  Usage (GPU box): bash tools/ab_all.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
LIBS="libdeltagpu.so libdeltagpu_base.so" bash tools/ab_quick.sh || exit 1
LIBS="libdeltagpu.so libdeltagpu_base.so" bash tools/ab_kfold.sh
