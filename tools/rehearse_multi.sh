# Rehearsal of bench.py's N = 2 path on a one-GPU box (two ranks on cuda:0 over gloo;
# the driver's 8-GPU run uses RCCL), then smoke().
set -o pipefail
mkdir -p gpurun_out
DG_BENCH_BACKEND=gloo DG_BENCH_SAME_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_n2.log 2>&1 || { echo N2_FAILED; tail -30 gpurun_out/bench_n2.log; exit 1; }
tail -1 gpurun_out/bench_n2.log | cut -c1-600
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
