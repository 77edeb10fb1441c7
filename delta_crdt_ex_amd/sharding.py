"""Key-hash range sharding of a replica across GPUs.

Key ids are 64-bit hashes, so a store sorted by key id is also sorted by shard:
shard s of N owns key ids in [ceil(s * 2^64 / N), ceil((s + 1) * 2^64 / N)), i.e.
floor(key * N / 2^64) == s.  Join and read are per key, so every rank joins its own
shard with no data exchange.  The only cross-rank steps are tiny:

* the causal context: every shard carries the replica's full VV, so the union is
  computed redundantly on every rank; `vv_allreduce_max_context` is the RCCL (or gloo)
  all-reduce that keeps them identical when shards were updated independently -- on the
  context's own device tensors (`vv_allreduce_max` is the host-array form);
* the Merkle tree: each rank builds the tree of its shard's key range (a level-log2(N)
  subtree of the unsharded tree); `merkle_roots` all-gathers the N shard roots (8 bytes
  each) and folds them into the replica's root -- the unsharded tree's root, so roots
  compare across shard counts; a diff descends only into shards whose roots differ
  (`differing_shards`).

One process per GPU (torch.distributed: "nccl" = RCCL over xGMI on MI355X; "gloo" in
the CPU tests).  Nothing here moves rows between GPUs.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1


def shard_of(key_ids: np.ndarray, n_shards: int) -> np.ndarray:
    """floor(key * n / 2^64) for a uint64 array (exact, no 128-bit arithmetic)."""
    key_ids = np.asarray(key_ids, np.uint64)
    hi = key_ids >> np.uint64(32)
    lo = key_ids & np.uint64(0xFFFFFFFF)
    s = np.uint64(n_shards)
    with np.errstate(over="ignore"):
        return ((hi * s + ((lo * s) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def shard_lower_bound(shard: int, n_shards: int) -> int:
    """Smallest key id owned by `shard` (0 for shard 0; 2^64 past the last shard)."""
    if shard <= 0:
        return 0
    if shard >= n_shards:
        return 1 << 64
    # smallest k with floor(k * n / 2^64) >= shard  <=>  k >= ceil(shard * 2^64 / n)
    return -((-shard << 64) // n_shards)


def split_rows(rows, n_shards: int):
    """Split sorted SoA rows (key, val, ts, node, cnt) into n contiguous shard slices."""
    key = np.asarray(rows[0], np.uint64)
    cuts = [0]
    for s in range(1, n_shards):
        b = shard_lower_bound(s, n_shards)
        cuts.append(int(np.searchsorted(key, np.uint64(b), side="left")) if b < (1 << 64)
                    else len(key))
    cuts.append(len(key))
    return [tuple(np.ascontiguousarray(c[cuts[s]:cuts[s + 1]]) for c in rows)
            for s in range(n_shards)]


def vv_merge_max(parts):
    """Per-node max over a list of (node u32[], cnt u64[]) version vectors."""
    acc: dict = {}
    for node, cnt in parts:
        for a, b in zip(np.asarray(node).tolist(), np.asarray(cnt).tolist()):
            if b > acc.get(a, -1):
                acc[a] = b
    items = sorted(acc.items())
    return (np.array([a for a, _ in items], np.uint32), np.array([b for _, b in items], np.uint64))


def _coll_device(group):
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def vv_allreduce_max(node: np.ndarray, cnt: np.ndarray, group=None):
    """All-reduce(max) of a version vector across the ranks of `group`
    (Dots.union/2 of VVs, aw_lww_map.ex:39-52, across key-hash shards).

    Node ids are dense interned ids (interning.py), so a VV is a dense counter vector
    indexed by node id: one all-reduce(MAX) of the vector lengths, then one
    all-reduce(MAX) of the vectors (counter + 1, 0 = absent node).  On RCCL these are
    two latency-bound all-reduces of a few hundred bytes."""
    import torch
    import torch.distributed as dist

    dev = _coll_device(group)
    node = np.asarray(node, np.int64)
    n = torch.tensor([int(node.max()) + 1 if len(node) else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
    m = int(n.item())
    dense = np.zeros(max(m, 1), np.int64)
    c = np.asarray(cnt, np.uint64)
    if np.any(c >= np.uint64((1 << 63) - 1)):
        raise OverflowError("a counter >= 2^63 - 1 does not fit the int64 all-reduce")
    dense[node] = c.astype(np.int64) + 1
    t = torch.from_numpy(dense).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    out = t.cpu().numpy()[:m]
    have = np.flatnonzero(out)
    return have.astype(np.uint32), (out[have] - 1).astype(np.uint64)


def vv_allreduce_max_context(ctx, n_nodes: int, group=None):
    """All-reduce(max) of a device version vector (store.Context, kind VV) across the
    ranks of `group`, without leaving the device: the VV is scattered into a dense counter
    vector indexed by node id (counter + 1; 0 = absent), all-reduced with MAX (RCCL over
    xGMI on MI355X: one latency-bound all-reduce of n_nodes x 8 bytes), and compacted back
    to (node, counter) pairs.  The ranks' node ids must be one interning (a replica set's
    shards share its dense ids) and n_nodes their common count; counters < 2^63 - 1.
    Dots.union/2 of VVs (aw_lww_map.ex:39-52) across key-hash shards."""
    import torch
    import torch.distributed as dist

    from .store import DG_CTX_VV, Context
    if ctx.kind != DG_CTX_VV:
        raise ValueError("vv_allreduce_max_context: the context is not a version vector")
    dev = ctx.node.device
    cdev = _coll_device(group)
    n = ctx.n
    dense = torch.zeros(max(int(n_nodes), 1), dtype=torch.int64, device=dev)
    if n:
        dense.scatter_(0, ctx.node[:n].long(), ctx.cnt[:n] + 1)
    t = dense if cdev.type == dev.type else dense.to(cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if t is not dense:
        dense = t.to(dev)
    node = torch.nonzero(dense).squeeze(1)
    m = int(node.numel())
    out = Context.empty(DG_CTX_VV, max(m, 1), dev)
    out.node[:m] = node.to(torch.int32)
    out.cnt[:m] = dense[node] - 1
    out.n = m
    return out


def _mix64(x: int) -> int:
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & MASK64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & MASK64
    x ^= x >> 31
    return x


def node_hash(left: int, right: int) -> int:
    """The Merkle parent hash of csrc/dg_hash.h (host copy)."""
    return _mix64(left ^ _mix64(right ^ 0xD6E8FEB86659FD93))


def fold_roots(roots) -> int:
    """Replica root over the 2^b shard roots (shard order): the top b levels of the
    unsharded tree (dg_merkle_fold_roots), parents = node_hash(left, right).  A shard's
    tree covers exactly its key range (dg_merkle shard_bits/shard), so the result equals
    the root of the unsharded tree of depth b + the shard depth."""
    level = [int(r) & MASK64 for r in roots]
    if len(level) & (len(level) - 1):
        raise ValueError("Merkle shard roots fold only for a power-of-two shard count")
    while len(level) > 1:
        level = [node_hash(level[i], level[i + 1]) for i in range(0, len(level), 2)]
    return level[0]


def merkle_roots(local_root: int, group=None):
    """All-gather the shard roots (one u64 per rank); returns (roots, replica_root)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = _coll_device(group)
    t = torch.tensor([int(np.array([local_root], np.uint64).view(np.int64)[0])], dtype=torch.int64,
                     device=dev)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    roots = [int(np.array([o.item()], np.int64).view(np.uint64)[0]) for o in outs]
    return roots, fold_roots(roots)


def shard_bits(n_shards: int) -> int:
    """log2 of a power-of-two shard count (the Merkle shard trees need one)."""
    b = int(n_shards).bit_length() - 1
    if n_shards != 1 << b:
        raise ValueError(f"{n_shards} shards: Merkle shard trees need a power of two")
    return b


def differing_shards(roots_a, roots_b):
    """Shards whose subtree roots differ: the only ones a diff descends into."""
    return [s for s, (x, y) in enumerate(zip(roots_a, roots_b)) if x != y]
