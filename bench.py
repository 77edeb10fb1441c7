"""bench.py — merged dots/s of the AWLWWMap delta join on MI355X (BASELINE.json metric).

A "step" is one AWLWWMap.join/3 (full-state, all keys) of two replicas resident in
HBM — BASELINE config 2 per GPU: 1M keys, ~10 % concurrent-write conflicts,
N_in = 2M rows, N_out ~= 1.1M rows.  At N GPUs (one process per GPU, launched by
torch.distributed.run) every rank joins its own key-hash range shard of an N x 1M-key
key space (weak scaling); there is no collective in the data path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

Rank 0 prints ONE JSON line.  `value` = Σ input rows over all ranks x K / the max
over ranks of the timed region.  `roofline` prices the join kernel (one launch per
step: rows + context union) by its algorithmic bytes 36·(N_in + N_out) + 12·(|c_a| +
|c_b| + |c_out|) over its average duration from HIP events on the engine stream.
`cpu_baseline` times the C restatement (oracle/deltaref.c, 1 thread) on the same
config-2 inputs, repeated for ~10 s.  A secondary Merkle hash+diff rate (config-4
shape, 1M keys, 1 % differing) is reported under `merkle`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
KEYS_PER_GPU = 1_000_000


def _traffic_from_profiles(n_in, n_out):
    """HBM bytes per launch of the join kernel from the committed PMC summary, if one
    exists for this exact workload (profiles/join2_pmc.json, written by
    tools/pmc_traffic.py); else None."""
    p = os.path.join(ROOT, "profiles", "join2_pmc.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None
    if d.get("rows_in") != n_in or d.get("rows_out") != n_out:
        return None
    return d.get("hbm_bytes_per_launch")


def cpu_baseline(a, b, budget_s=10.0):
    from oracle import ref as R  # the checker / CPU baseline only
    R.lib()
    n_in = len(a["rows"][0]) + len(b["rows"][0])
    reps, t0 = 0, time.perf_counter()
    while True:
        R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 1000:
            break
    return {
        "value": n_in * reps / el,
        "unit": "merged dots/s",
        "cores": 1,
        "kind": "port",
        "sample": f"C restatement of aw_lww_map.ex join/3 (oracle/deltaref.c, gcc -O2, 1 thread) on "
                  f"the same config-2 replicas ({n_in} rows in), {reps} joins in {el:.1f} s",
    }


def merkle_rate(eng, torch, dev, steps=20):
    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Store
    a, b = W.merkle_pair(n_keys=KEYS_PER_GPU, diff_frac=0.01, seed=4)
    sa = Store.from_numpy(*a["rows"], device=dev)
    sb = Store.from_numpy(*b["rows"], device=dev)
    depth = 18
    ta = eng.merkle_build(sa, depth)
    tb = eng.merkle_build(sb, depth)
    d = eng.merkle_diff(ta, tb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.merkle_build(sa, depth, ta)
        eng.merkle_build(sb, depth, tb)
        d = eng.merkle_diff(ta, tb)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    keys = ta.n_keys + tb.n_keys
    return {"metric": "Merkle hash+diff keys/s (config-4 shape, 1 GPU shard)",
            "value": keys / el, "unit": "keys/s", "ms_per_round": el * 1e3,
            "keys": keys, "differing_keys": int(d.numel()), "depth": depth,
            "note": "two builds + one diff per round, synchronous API (includes host syncs)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from delta_crdt_ex_amd import workloads as W
    from delta_crdt_ex_amd.store import Context, Engine, Store

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    a, b = W.config2_shard(rank, world, KEYS_PER_GPU)
    n_in = len(a["rows"][0]) + len(b["rows"][0])
    eng = Engine(local)
    stream = eng.stream
    sa = Store.from_numpy(*a["rows"], device=dev)
    sb = Store.from_numpy(*b["rows"], device=dev)
    ca = Context.from_numpy(*a["ctx"], dev)
    cb = Context.from_numpy(*b["ctx"], dev)
    out = Store.empty(sa.n + sb.n, dev)
    octx = Context.empty(0, ca.n + cb.n, dev)
    d_counts = torch.zeros(8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    launch = eng.prepare_join2(sa, ca, sb, cb, out, octx, d_counts)
    for _ in range(args.warmup):
        launch()
    eng.sync()
    n_out = int(d_counts[0].item())
    n_ctx_out = int(d_counts[1].item())

    # timed region: K back-to-back joins, barrier + sync on both sides
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        launch()
    eng.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()

    # per-launch device time of the join (all its kernels) from HIP events recorded on
    # the engine stream, in a separate pass so the events do not perturb the timed loop
    nev = min(args.steps, 100)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(nev + 1)]
    with torch.cuda.stream(stream):
        for i in range(nev):
            ev[i].record(stream)
            launch()
        ev[nev].record(stream)
    eng.sync()
    torch.cuda.synchronize()
    launch_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(nev)]
    avg_launch_s = float(np.median(launch_ms)) / 1e3

    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(n_in)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    el_max = float(el_t.item())
    total_rows = float(tot.item())

    if rank == 0:
        alg_bytes = 36 * (n_in + n_out) + 12 * (ca.n + cb.n + n_ctx_out)
        achieved = alg_bytes / avg_launch_s / 1e9
        traffic = _traffic_from_profiles(n_in, n_out)
        res = {
            "metric": "merged dots/sec for AWLWWMap delta join + Merkle diff keys/sec at 1\u20138 GPUs",
            "value": total_rows * args.steps / el_max,
            "unit": "merged dots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded config-2 replicas, SURVEY.md §8(d))",
            "config": {
                "workload": "config2: 1M-key AWLWWMap full-state join of two replicas, 10% "
                            "concurrent-write conflicts, per GPU (key-hash range shards)",
                "keys_per_gpu": KEYS_PER_GPU,
                "rows_in_per_gpu": n_in,
                "rows_out_per_gpu": n_out,
                "parallelism": f"key-hash shards x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "join2 = join2_partition_kernel + join2_rows_kernel (events bracket both)",
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_us": avg_launch_s * 1e6,
                "launch_timing": "median of per-step HIP event pairs on the engine stream",
            },
        }
        if not args.no_merkle:
            res["merkle"] = merkle_rate(eng, torch, dev)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(a, b)
        elif not args.no_cpu_baseline:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
