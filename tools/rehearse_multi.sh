# Rehearsal of bench.py's N > 1 path on a one-GPU box (N ranks on cuda:0 over gloo; the
# driver's 8-GPU run uses RCCL), then smoke().   N=4 bash tools/rehearse_multi.sh  (default 2)
set -o pipefail
N=${N:-2}
mkdir -p gpurun_out
DG_BENCH_BACKEND=gloo DG_BENCH_SAME_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_n$N.log 2>&1 || { echo N${N}_FAILED; tail -30 gpurun_out/bench_n$N.log; exit 1; }
tail -1 gpurun_out/bench_n$N.log | cut -c1-600
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
