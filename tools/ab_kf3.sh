# kfold tests + config-3 A/B (default vs libdeltagpu_base.so) + kfold phase stamps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kfold.py tests/test_gpu_configs.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_kf.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/pytest_kf.log; exit 1; }
tail -1 gpurun_out/pytest_kf.log
LIBS="libdeltagpu.so libdeltagpu_base.so" bash tools/ab_kfold.sh || exit 1
timeout -k 10 200 python -u tools/kfold_stamps.py
