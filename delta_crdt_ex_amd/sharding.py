"""Key-hash range sharding of a replica across GPUs.

Key ids are 64-bit hashes, so a store sorted by key id is also sorted by shard:
shard s of N owns key ids in [ceil(s * 2^64 / N), ceil((s + 1) * 2^64 / N)), i.e.
floor(key * N / 2^64) == s.  Join and read are per key, so every rank joins its own
shard with no data exchange.  The only cross-rank steps are tiny:

* the causal context: every shard carries the replica's full VV, so the union is
  computed redundantly on every rank; `vv_allreduce_max` is the RCCL (or gloo)
  all-reduce that keeps them identical when shards were updated independently;
* the Merkle tree: each rank builds the tree of its shard; `merkle_roots` all-gathers
  the N shard roots (8 bytes each) and folds them into the replica's root; a diff
  descends only into shards whose roots differ (`differing_shards`).

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


def vv_allreduce_max(node: np.ndarray, cnt: np.ndarray, group=None):
    """All-reduce(max) of a version vector across the ranks of `group`.

    VVs of different ranks may name different nodes, so this all-gathers the (padded)
    node/counter arrays and merges them: a few KB at most (one entry per replica)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    n = torch.tensor([len(node)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(x.item()) for x in sizes))
    buf = torch.zeros((max(m, 1), 2), dtype=torch.int64, device=dev)
    if len(node):
        buf[: len(node), 0] = torch.from_numpy(np.asarray(node, np.int64))
        buf[: len(node), 1] = torch.from_numpy(np.asarray(cnt, np.uint64).view(np.int64))
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = []
    for r, o in enumerate(outs):
        k = int(sizes[r].item())
        a = o[:k].cpu().numpy()
        parts.append((a[:, 0].astype(np.uint32), a[:, 1].view(np.uint64)))
    return vv_merge_max(parts)


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
    """Replica root over the shard roots: a binary tree over the N roots (padded with
    0 to a power of two), parents = node_hash(left, right)."""
    level = [int(r) & MASK64 for r in roots]
    while len(level) & (len(level) - 1):
        level.append(0)
    while len(level) > 1:
        level = [node_hash(level[i], level[i + 1]) for i in range(0, len(level), 2)]
    return level[0]


def merkle_roots(local_root: int, group=None):
    """All-gather the shard roots (one u64 per rank); returns (roots, replica_root)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([int(np.array([local_root], np.uint64).view(np.int64)[0])], dtype=torch.int64,
                     device=dev)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    roots = [int(np.array([o.item()], np.int64).view(np.uint64)[0]) for o in outs]
    return roots, fold_roots(roots)


def differing_shards(roots_a, roots_b):
    """Shards whose subtree roots differ: the only ones a diff descends into."""
    return [s for s, (x, y) in enumerate(zip(roots_a, roots_b)) if x != y]
