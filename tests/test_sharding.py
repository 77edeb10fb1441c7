"""Key-hash range sharding with world_size-2 and -4 torch.distributed/gloo
on the CPU: per-shard joins reassemble the unsharded join exactly, the VV all-reduce
yields the global context union, and Merkle shard roots localise the diff.  The
per-shard compute here is the C oracle (the GPU box runs libdeltagpu per rank)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from delta_crdt_ex_amd import sharding as S
from delta_crdt_ex_amd import workloads as W


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_of_matches_bounds():
    rng = np.random.default_rng(0)
    keys = np.sort(rng.integers(0, 1 << 63, 5000, dtype=np.int64).astype(np.uint64) * np.uint64(2))
    for n in (1, 2, 3, 8):
        sh = S.shard_of(keys, n)
        assert np.all(np.diff(sh) >= 0) and sh.min() >= 0 and sh.max() < n
        for s in range(n):
            lb = S.shard_lower_bound(s, n)
            assert np.all(keys[sh == s] >= np.uint64(lb)) if lb < (1 << 64) else True
            if s > 0:
                assert np.all(keys[sh == s - 1] < np.uint64(lb))
        parts = S.split_rows((keys, keys, keys.view(np.int64), keys.astype(np.uint32), keys), n)
        assert sum(len(p[0]) for p in parts) == len(keys)
        for s, p in enumerate(parts):
            assert np.all(S.shard_of(p[0], n) == s)


def test_fold_roots_matches_c_tree():
    from oracle import ref as R
    # a depth-3 tree over 8 "shard roots" equals fold_roots over the level-3 nodes
    a, _ = W.merkle_pair(n_keys=3000, seed=3)
    t = R.merkle_build(a["rows"], 3)
    lvl3 = t.nodes[7:15]
    assert S.fold_roots(lvl3.tolist()) == int(t.nodes[0]) == R.fold_roots(lvl3)
    with pytest.raises(ValueError):
        S.fold_roots([1, 2, 3])


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from oracle import ref as R
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        rng = np.random.default_rng(7)
        a, b = W.random_pair(rng, n_keys=400, ts_range=5, dense_ctx=False)
        a2, b2 = W.config2(n_keys=6000, seed=3)
        for A, B in ((a, b), (a2, b2)):
            mine_a = S.split_rows(A["rows"], world)[rank]
            mine_b = S.split_rows(B["rows"], world)[rank]
            rows, ctx = R.join2(mine_a, A["ctx"], mine_b, B["ctx"])
            # every shard computed the same (replicated) context union
            node, cnt = S.vv_allreduce_max(ctx[1], ctx[2])
            want_rows, want_ctx = R.join2(A["rows"], A["ctx"], B["rows"], B["ctx"])
            assert np.array_equal(node, want_ctx[1]) and np.array_equal(cnt, want_ctx[2])
            # the same on the context's own tensors (no host arrays): this rank's VV is
            # its own half of the union, the all-reduce restores the whole
            import torch
            from delta_crdt_ex_amd.store import Context
            half = slice(rank, None, world)
            hn, hc = ctx[1][half], ctx[2][half]
            c = Context(ctx[0], torch.from_numpy(hn.astype(np.int32)),
                        torch.from_numpy(np.ascontiguousarray(hc).view(np.int64)), len(hn))
            n_nodes = int(max(A["ctx"][1].max(initial=0), B["ctx"][1].max(initial=0))) + 1
            got = S.vv_allreduce_max_context(c, n_nodes)
            gn, gc = got.to_numpy()
            assert np.array_equal(gn, want_ctx[1]) and np.array_equal(gc, want_ctx[2])
            # the shard's output is exactly the unsharded output's slice
            want_mine = S.split_rows(want_rows, world)[rank]
            for x, y in zip(rows, want_mine):
                assert np.array_equal(x, y)
            # Merkle: shard trees over the shard's key range, roots, the replica root
            # (== the unsharded tree's root), and the diff restricted to differing shards
            depth, sb = 8, S.shard_bits(world)
            ta = R.merkle_build(mine_a, depth - sb, sb, rank)
            tb = R.merkle_build(mine_b, depth - sb, sb, rank)
            ra, root_a = S.merkle_roots(int(ta.nodes[0]))
            rb, root_b = S.merkle_roots(int(tb.nodes[0]))
            assert root_a == int(R.merkle_build(A["rows"], depth).nodes[0])
            assert root_b == int(R.merkle_build(B["rows"], depth).nodes[0])
            diff_local = R.merkle_diff(ta, mine_a, tb, mine_b)
            full = R.store_diff(A["rows"], B["rows"])
            assert np.array_equal(diff_local, S.split_rows((full,) * 5, world)[rank][0])
            assert (root_a != root_b) == (len(full) > 0)
            if rank not in S.differing_shards(ra, rb):
                assert len(diff_local) == 0
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "".join(traceback.format_exception(e))))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sharded_join_and_merkle(world):
    """world_size 2 and 4: the VV all-reduce (host arrays and device contexts), the shard
    roots' all-gather and fold (== the unsharded root), and the diff restricted to the
    differing shards (== the unsharded diff's slice) -- the sync round of
    causal_crdt.ex:252-270 over key-hash shards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, msg in sorted(res):
        assert msg == "ok", f"rank {rank}: {msg}"


@pytest.mark.gpu
def test_sharded_round_through_libdeltagpu():
    """tests/sharded_round.py: two (and four) processes on cuda:0, one key-hash shard each, run the
    config-4 round through libdeltagpu (shard Merkle trees whose roots fold to the
    unsharded root, diff, take, keyed join, VV all-reduce, incremental Merkle update)
    against the C oracle's unsharded results.  Started at session start, before this
    process touches the GPU (conftest.EARLY_CMDS).  Unmeasured at 8 GPUs: the driver's
    SCALE run is the 8-GPU measurement."""
    from conftest import early_result
    for name, world in (("sharded2", 2), ("sharded4", 4)):
        rc, out = early_result(name)
        assert rc == 0, out
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        assert len(lines) == world and all('"ok": true' in ln for ln in lines), out
