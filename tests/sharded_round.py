"""A config-4 anti-entropy round on key-hash shards, one process per shard, all on
cuda:0, through libdeltagpu.

    python tests/sharded_round.py [--world 2] [--keys-per-rank 40000]

The parent only spawns the ranks (it never touches the GPU, so no process that has
initialised the GPU starts another program).  Collectives are gloo on the CPU (two
processes cannot share one GPU through RCCL); bench.py --gpus N runs the same round over
RCCL.  Each rank, on its shard of two replicas A and B that differ on 2 % of the keys:

  * builds both replicas' shard Merkle trees (dg_merkle_build over the shard's key
    range); the all-gathered shard roots fold (dg_merkle_fold_roots) to the C oracle's
    root of the UNSHARDED tree;
  * diffs them on the device (dg_merkle_diff) -- the shard's slice of the oracle's exact
    differing keys -- takes B's sync delta for them (dg_take_keys) and joins it into A
    with its changed keys (dg_join2_changes): the shard's slice of the oracle's
    full-state join;
  * all-reduces the joined version vector (sharding.vv_allreduce_max and, on the
    device tensors, vv_allreduce_max_context): the oracle's;
  * updates A's tree from the changed keys (dg_merkle_update): equal to a fresh build,
    and the joined replica's folded root is the oracle's root of the joined rows.

Exit status 0 and one JSON line per rank on success.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DEPTH = 14


def _rank(rank, world, port, kpr, q):
    try:
        import numpy as np
        import torch
        import torch.distributed as dist

        from delta_crdt_ex_amd import sharding as S
        from delta_crdt_ex_amd import workloads as W
        from delta_crdt_ex_amd.store import Context, Engine, Store, fold_roots, u64
        from oracle import ref as R

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        sb_bits = S.shard_bits(world)
        shards = [W.config4_shard(r, world, keys_per_rank=kpr, diff_frac=0.02) for r in range(world)]
        a, b = shards[rank]

        def cat(side):
            cols = [np.concatenate([s[side]["rows"][i] for s in shards]) for i in range(5)]
            return W.sort_rows(*cols)

        fa, fb = cat(0), cat(1)
        ctx_a, ctx_b = shards[0][0]["ctx"], shards[0][1]["ctx"]  # every shard carries the VV
        want_rows, want_ctx = R.join2(fa, ctx_a, fb, ctx_b)
        want_diff = R.store_diff(fa, fb)

        torch.cuda.set_device(0)
        dev = "cuda:0"
        eng = Engine(0)
        sa, sb = Store.from_numpy(*a["rows"], device=dev), Store.from_numpy(*b["rows"], device=dev)
        ca, cb = Context.from_numpy(*a["ctx"], dev), Context.from_numpy(*b["ctx"], dev)
        d = DEPTH - sb_bits
        ta = eng.merkle_build(sa, d, shard_bits=sb_bits, shard=rank)
        tb = eng.merkle_build(sb, d, shard_bits=sb_bits, shard=rank)
        roots_a, root_a = S.merkle_roots(ta.root())
        roots_b, root_b = S.merkle_roots(tb.root())
        assert root_a == fold_roots(roots_a) == int(R.merkle_build(fa, DEPTH).nodes[0]), "root A"
        assert root_b == int(R.merkle_build(fb, DEPTH).nodes[0]), "root B"

        keys = eng.merkle_diff(ta, tb)
        mine = S.split_rows((want_diff,) * 5, world)[rank][0]
        assert np.array_equal(u64(keys), mine), "shard diff"
        if rank not in S.differing_shards(roots_a, roots_b):
            assert len(mine) == 0
        delta = eng.take_keys(sb, keys)
        out, octx, changed = eng.join2_changes(sa, ca, delta, cb, keys=keys)
        got = out.to_numpy()
        for x, y in zip(got, S.split_rows(want_rows, world)[rank]):
            assert np.array_equal(x, y), "shard join rows"
        node, cnt = S.vv_allreduce_max(*octx.to_numpy())
        assert np.array_equal(node, want_ctx[1]) and np.array_equal(cnt, want_ctx[2]), "VV"
        # on the device tensors themselves (gloo takes a host hop; RCCL stays on the GPU)
        vv = S.vv_allreduce_max_context(octx, len(a["nodes"].dense))
        gn, gc = vv.to_numpy()
        assert np.array_equal(gn, want_ctx[1]) and np.array_equal(gc, want_ctx[2]), "device VV"

        eng.merkle_update(ta, out, changed)
        fresh = eng.merkle_build(out, d, shard_bits=sb_bits, shard=rank)
        assert np.array_equal(ta.nodes.cpu().numpy(), fresh.nodes.cpu().numpy()), "update"
        _, root_j = S.merkle_roots(ta.root())
        assert root_j == int(R.merkle_build(want_rows, DEPTH).nodes[0]), "joined root"
        dist.barrier()
        dist.destroy_process_group()
        eng.close()
        q.put((rank, json.dumps({"rank": rank, "ok": True, "shard_rows": int(sa.n),
                                 "diff_keys": int(keys.numel()), "joined_rows": int(out.n),
                                 "root": hex(root_j)})))
    except Exception as e:  # reported to the parent
        q.put((rank, "".join(traceback.format_exception(e))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--keys-per-rank", type=int, default=40_000)
    args = ap.parse_args()
    import multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, args.world, port, args.keys_per_rank, q))
             for r in range(args.world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    bad = 0
    for rank, msg in sorted(res):
        print(msg, flush=True)
        bad += not msg.startswith("{")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
