"""Seeded synthetic replicas for BASELINE.json's configs.

Every generator builds exactly the state the reference's mutators would reach
(`AWLWWMap.add/4` :99-112 and `remove/3` :133-146 applied through
`join(state, delta, [key])` as CausalCrdt does, causal_crdt.ex:337-342,383-384),
but vectorised with numpy: keys/values are integers (as in
bench/basic_operations.exs:4), key ids are splitmix64(k), value ids the
order-preserving integer encoding, ts i64.  Node ids are what the boundary's
marshalling produces for REAL replica ids: every replica draws a 30-bit node id as
CausalCrdt does (`:rand.uniform(1_000_000_000)`, causal_crdt.ex:65) and a Universe
interns those terms to dense u32 ids (interning.py), so the kernels see the dense ids
a NIF caller would hand them.  tests/ check the generators against the term-level
oracle replaying the same operations with the 30-bit terms.

A replica is a dict: {"rows": (key, val, ts, node, cnt) sorted, "ctx": (kind, node, cnt),
"nodes": NodeTable}.
"""
from __future__ import annotations

import numpy as np

from .interning import Universe, encode_int_value, splitmix64_np
from .sharding import shard_of

VV, DOTS = 0, 1


def node_terms(n: int, seed: int) -> np.ndarray:
    """n distinct replica node ids as CausalCrdt draws them,
    :rand.uniform(1_000_000_000) (1..1e9, 30 bits; causal_crdt.ex:65)."""
    rng = np.random.default_rng([seed, 0x6E6F6465])
    out: list[int] = []
    seen: set[int] = set()
    while len(out) < n:
        for x in rng.integers(1, 1_000_000_001, n).tolist():
            if x not in seen and len(out) < n:
                seen.add(x)
                out.append(x)
    return np.array(out, np.int64)


class NodeTable:
    """Logical replica i of a workload has the 30-bit node term raw[i]; the rows and
    contexts carry the dense id the boundary's interning gives that term
    (Universe.node_ids over all of them: dense ids follow ascending term order)."""

    def __init__(self, n: int, seed: int):
        self.raw = node_terms(n, seed)
        self.universe = Universe()
        self.dense = self.universe.node_ids(self.raw).astype(np.uint32)

    def __getitem__(self, logical) -> int:
        return int(self.dense[logical])

    def ids(self, logical: np.ndarray) -> np.ndarray:
        return self.dense[np.asarray(logical, np.int64)]

    def term_of_dense(self) -> dict:
        return {int(d): int(r) for d, r in zip(self.dense, self.raw)}

    def dense_of_term(self) -> dict:
        return {int(r): int(d) for d, r in zip(self.dense, self.raw)}


def sort_rows(k, v, t, n, c):
    order = np.lexsort((c, n, t, v, k))
    return (np.ascontiguousarray(k[order], np.uint64), np.ascontiguousarray(v[order], np.uint64),
            np.ascontiguousarray(t[order], np.int64), np.ascontiguousarray(n[order], np.uint32),
            np.ascontiguousarray(c[order], np.uint64))


def vv(d: dict):
    items = sorted(d.items())
    return (VV, np.array([a for a, _ in items], np.uint32), np.array([b for _, b in items], np.uint64))


def config1(n_keys: int = 10_000, nodes: NodeTable | None = None):
    """Config 1 (bench/basic_operations.exs-style, CPU plumbing): replica 1 adds
    k => k for k = 1..n; B := A; A removes k % 10 == 0; B (replica 2) re-adds
    k % 10 == 5 with v = k + 1.  Returns (A, B)."""
    N = nodes or NodeTable(3, 1)
    k = np.arange(1, n_keys + 1, dtype=np.uint64)
    key = splitmix64_np(k)
    val = encode_int_value(k.astype(np.int64))
    ts = k.astype(np.int64) * 1000
    node = np.full(n_keys, N[1], np.uint32)
    cnt = k.copy()
    # A: removes k % 10 == 0 (remove/3 ctx = the removed dots; the VV absorbs them)
    keep_a = (k % 10) != 0
    A = {"rows": sort_rows(key[keep_a], val[keep_a], ts[keep_a], node[keep_a], cnt[keep_a]),
         "ctx": vv({N[1]: n_keys}), "nodes": N}
    # B: re-adds k % 10 == 5 with v = k + 1 as node 2, counters 1.. in key order
    re = (k % 10) == 5
    nre = int(re.sum())
    val_b = val.copy()
    ts_b = ts.copy()
    node_b = node.copy()
    cnt_b = cnt.copy()
    val_b[re] = encode_int_value(k[re].astype(np.int64) + 1)
    ts_b[re] = n_keys * 1000 + k[re].astype(np.int64)
    node_b[re] = N[2]
    cnt_b[re] = np.arange(1, nre + 1, dtype=np.uint64)
    B = {"rows": sort_rows(key, val_b, ts_b, node_b, cnt_b), "ctx": vv({N[1]: n_keys, N[2]: nre}),
         "nodes": N}
    return A, B


def config2(n_keys: int = 1_000_000, seed: int = 2, key_lo: int = 1, keys=None,
            nodes: NodeTable | None = None):
    """Config 2: base replica 0 writes k = key_lo..key_lo+n-1 (counter = k,
    ts = k * 1000); replicas A (1) and B (2) both overwrite the ~10 % of
    keys with splitmix64(k ^ seed) % 10 == 0 with fresh random values, ts = base +
    U[0, 1e9).  `keys` (uint64 array of k) overrides the key range (sharding).
    Returns (A, B); N_in ~= 2 n, N_out ~= 1.1 n."""
    N = nodes or NodeTable(3, 2)
    if keys is None:
        k = np.arange(key_lo, key_lo + n_keys, dtype=np.uint64)
    else:
        k = np.asarray(keys, np.uint64)
    n = len(k)
    key = splitmix64_np(k)
    val = encode_int_value(k.astype(np.int64))
    ts = k.astype(np.int64) * 1000
    cnt0 = k.copy()  # node 0 wrote key k as its k-th add
    conflict = (splitmix64_np(k ^ np.uint64(seed)) % np.uint64(10)) == 0
    nc = int(conflict.sum())
    rng = np.random.default_rng(seed)
    ts_base = int(ts.max()) + 1000 if n else 0
    out = []
    for node_id in (1, 2):
        v_new = rng.integers(0, 1 << 62, nc, dtype=np.int64)
        t_new = ts_base + rng.integers(0, 1_000_000_000, nc, dtype=np.int64)
        val_r = val.copy()
        ts_r = ts.copy()
        node_r = np.full(n, N[0], np.uint32)
        cnt_r = cnt0.copy()
        val_r[conflict] = encode_int_value(v_new)
        ts_r[conflict] = t_new
        node_r[conflict] = N[node_id]
        cnt_r[conflict] = np.arange(1, nc + 1, dtype=np.uint64)
        out.append({"rows": sort_rows(key, val_r, ts_r, node_r, cnt_r),
                    "ctx": vv({N[0]: int(k.max()) if n else 0, N[node_id]: nc}), "nodes": N})
    return out[0], out[1]


def config2_shard(rank: int, world: int, keys_per_rank: int = 1_000_000, seed: int = 2):
    """Config 2 at weak scaling: the global key space 1..world*keys_per_rank is
    range-sharded by key hash and rank `rank` builds its shard of A and B."""
    k = np.arange(1, world * keys_per_rank + 1, dtype=np.uint64)
    mine = shard_of(splitmix64_np(k), world) == rank
    return config2(seed=seed, keys=k[mine], nodes=NodeTable(3, 2))


def merkle_pair(n_keys: int = 1_000_000, diff_frac: float = 0.01, seed: int = 4, keys=None,
                nodes: NodeTable | None = None, n_total: int | None = None):
    """Config-4-shaped pair: two replicas of the same base (replica 0 wrote key k with
    counter k, ts = k * 1000) that differ on ~diff_frac of the keys (replica 2 re-added
    them: counter k, ts past the base, a value drawn from k).  Every choice is a function
    of the key alone, so the rows of a key-hash shard (`keys`, a subset of 1..n_total) are
    exactly that shard's slice of the whole replica pair, and each shard carries the
    replicas' full version vectors ({0: n_total}, {0: n_total, 2: n_total}).  Returns
    (A, B)."""
    N = nodes or NodeTable(3, 4)
    if keys is None:
        k = np.arange(1, n_keys + 1, dtype=np.uint64)
    else:
        k = np.asarray(keys, np.uint64)
    total = int(n_total if n_total is not None else (int(k.max()) if len(k) else 0))
    n = len(k)
    key = splitmix64_np(k)
    val = encode_int_value(k.astype(np.int64))
    ts = k.astype(np.int64) * 1000
    node = np.full(n, N[0], np.uint32)
    cnt = k.copy()
    A = {"rows": sort_rows(key, val, ts, node, cnt), "ctx": vv({N[0]: total}), "nodes": N}
    h = splitmix64_np(k ^ np.uint64(seed * 0x9E3779B97F4A7C15 & ((1 << 64) - 1)))
    d = (h % np.uint64(1 << 20)).astype(np.float64) < diff_frac * (1 << 20)
    hv = splitmix64_np(h)
    val_b, ts_b, node_b = val.copy(), ts.copy(), node.copy()
    val_b[d] = encode_int_value((hv[d] >> np.uint64(2)).astype(np.int64))
    ts_b[d] = total * 1000 + 1000 + (hv[d] % np.uint64(1_000_000_000)).astype(np.int64)
    node_b[d] = N[2]
    B = {"rows": sort_rows(key, val_b, ts_b, node_b, cnt.copy()),
         "ctx": vv({N[0]: total, N[2]: total}), "nodes": N}
    return A, B


def random_pair(rng: np.random.Generator, n_keys: int, n_nodes: int = 4, max_entries: int = 3,
                p_remove: float = 0.3, ts_range: int = 1 << 40, dense_ctx: bool = True,
                ctx_kind: int = VV):
    """Two replicas of one key space that evolved independently from a common base,
    with concurrent adds, removes, LWW ties (small ts_range) and — unless dense_ctx —
    stores that are NOT covered by their own VV (the sync path's
    VV-snapshot + current-values shape).  Used by the randomized parity tests."""
    keys = splitmix64_np(rng.choice(1 << 40, n_keys, replace=False).astype(np.uint64))
    reps = []
    for r in range(2):
        ks, vs, ts, ns, cs = [], [], [], [], []
        counters = {}
        for kid in keys:
            if rng.random() < p_remove:
                continue
            for _ in range(int(rng.integers(1, max_entries + 1))):
                nd = int(rng.integers(0, n_nodes))
                c = counters.get(nd, 0) + 1 + int(rng.integers(0, 3))
                counters[nd] = c
                ks.append(kid)
                vs.append(int(rng.integers(0, 8)) + (1 << 62))
                ts.append(int(rng.integers(-ts_range, ts_range)))
                ns.append(nd)
                cs.append(c)
        rows = (np.array(ks, np.uint64), np.array(vs, np.uint64), np.array(ts, np.int64),
                np.array(ns, np.uint32), np.array(cs, np.uint64))
        rows = sort_rows(*rows)
        # dedupe identical rows (a store is a set)
        if len(rows[0]):
            m = np.ones(len(rows[0]), bool)
            m[1:] = ~((rows[0][1:] == rows[0][:-1]) & (rows[1][1:] == rows[1][:-1]) &
                      (rows[2][1:] == rows[2][:-1]) & (rows[3][1:] == rows[3][:-1]) &
                      (rows[4][1:] == rows[4][:-1]))
            rows = tuple(c[m] for c in rows)
        if ctx_kind == VV:
            vvd = {}
            for nd in range(n_nodes):
                top = counters.get(nd, 0)
                vvd[nd] = top if dense_ctx else int(rng.integers(0, top + 2))
            ctx = vv(vvd)
        else:
            dots = set()
            for nd in range(n_nodes):
                top = counters.get(nd, 0)
                for c in range(1, top + 1):
                    if dense_ctx or rng.random() < 0.5:
                        dots.add((nd, c))
            dots = sorted(dots)
            ctx = (DOTS, np.array([d[0] for d in dots], np.uint32),
                   np.array([d[1] for d in dots], np.uint64))
        reps.append({"rows": rows, "ctx": ctx})
    # shared rows: copy a slice of A into B so that "in both" happens
    a, b = reps
    if len(a["rows"][0]):
        take = rng.random(len(a["rows"][0])) < 0.4
        merged = tuple(np.concatenate([b["rows"][i], a["rows"][i][take]]) for i in range(5))
        merged = sort_rows(*merged)
        m = np.ones(len(merged[0]), bool)
        if len(merged[0]) > 1:
            m[1:] = ~((merged[0][1:] == merged[0][:-1]) & (merged[1][1:] == merged[1][:-1]) &
                      (merged[2][1:] == merged[2][:-1]) & (merged[3][1:] == merged[3][:-1]) &
                      (merged[4][1:] == merged[4][:-1]))
        b["rows"] = tuple(c[m] for c in merged)
    return a, b


def _take_rows(rows, key_ids):
    """Rows whose key is in the sorted array key_ids (Map.take on the SoA store)."""
    m = np.isin(rows[0], key_ids)
    return tuple(c[m] for c in rows)


def config3(n_keys: int = 10_000_000, n_replicas: int = 64, touch: float = 0.01,
            remove_frac: float = 0.2, seed: int = 3, nodes: NodeTable | None = None, keys=None):
    """Config 3: a base state (node 0 wrote k = 1..n, counter k, ts = k * 1000) and
    `n_replicas` replicas (nodes 1..R) that each touched ~touch * n keys of it: 80 %
    re-added (AWLWWMap.add/4: the key's old entries go, one new entry with dot
    {r, c}, c = 1, 2, ... in key order) and 20 % removed (remove/3).  Each replica
    ships a sync-shaped delta (causal_crdt.ex:324-335): its VV, the rows of its touched
    keys (Map.take) and the touched keys themselves.

    Returns (base, deltas) where base = {"rows", "ctx"} and each delta =
    {"rows", "ctx", "keys"} (keys: ascending unique key ids).  Applying them is the
    fold join(state, delta_r, keys_r) over r = 1..R (causal_crdt.ex:383-384).
    `keys` (uint64 array of k) overrides the key range (a key-hash shard)."""
    N = nodes or NodeTable(n_replicas + 1, seed)
    k = np.arange(1, n_keys + 1, dtype=np.uint64) if keys is None else np.asarray(keys, np.uint64)
    n_keys = len(k)
    key = splitmix64_np(k)
    base = {"rows": sort_rows(key, encode_int_value(k.astype(np.int64)),
                              k.astype(np.int64) * 1000, np.full(n_keys, N[0], np.uint32), k.copy()),
            "ctx": vv({N[0]: n_keys}), "nodes": N}
    rng = np.random.default_rng(seed)
    ts_base = n_keys * 1000 + 1000
    m = max(1, int(round(touch * n_keys)))
    deltas = []
    for r in range(1, n_replicas + 1):
        idx = np.unique(rng.integers(0, n_keys, m))  # touched keys (by index into k)
        kid = key[idx]
        order = np.argsort(kid)  # key-id order: counters follow it
        kid = kid[order]
        added = rng.random(len(kid)) >= remove_frac
        na = int(added.sum())
        vals = encode_int_value(rng.integers(0, 1 << 62, na, dtype=np.int64))
        ts = ts_base + rng.integers(0, 1_000_000_000, na, dtype=np.int64)
        rows = sort_rows(kid[added], vals, ts, np.full(na, N[r], np.uint32),
                         np.arange(1, na + 1, dtype=np.uint64))
        deltas.append({"rows": rows, "ctx": vv({N[0]: n_keys, N[r]: na}), "keys": kid, "nodes": N})
    return base, deltas


def config4_shard(rank: int, world: int, keys_per_rank: int = 12_500_000,
                  diff_frac: float = 0.01, seed: int = 4):
    """Config 4, one key-hash shard: the shard `rank` of a world * keys_per_rank key
    space of two replicas that differ on ~diff_frac of the keys (merkle_pair: the
    shard's exact slice of the whole pair, with the replicas' full version vectors)."""
    k = np.arange(1, world * keys_per_rank + 1, dtype=np.uint64)
    mine = shard_of(splitmix64_np(k), world) == rank
    return merkle_pair(keys=k[mine], diff_frac=diff_frac, seed=seed, nodes=NodeTable(3, seed),
                       n_total=world * keys_per_rank)


def shard_keys(rank: int, world: int, n_total: int) -> np.ndarray:
    """The integer keys k in 1..n_total whose key id falls in key-hash shard `rank`."""
    k = np.arange(1, n_total + 1, dtype=np.uint64)
    if world == 1:
        return k
    return k[shard_of(splitmix64_np(k), world) == rank]


def config5_shard(rank: int, world: int, keys_per_rank: int = 12_500_000, seed: int = 5):
    """Config 5 at weak scaling: key-hash shard `rank` of world * keys_per_rank keys (100M
    over 8 GPUs).  config5 draws every choice from the key alone, so the shards are exact
    slices of ONE replica pair of world * keys_per_rank keys (they used to be
    independent pairs)."""
    n_total = world * keys_per_rank
    return config5(keys=shard_keys(rank, world, n_total), n_nodes=64, seed=seed, n_total=n_total)


def config3_shard(rank: int, world: int, n_keys: int = 10_000_000, seed: int = 3):
    """Config 3 split over ranks (strong scaling): key-hash shard `rank` of the 10M-key
    state and of every replica's delta (each touches 1 % of the shard's keys)."""
    return config3(keys=shard_keys(rank, world, n_keys), n_replicas=64, touch=0.01,
                   seed=seed + 1000 * rank if world > 1 else seed)


def sync_delta(rep, keys):
    """The sync message a replica sends for `keys` (causal_crdt.ex:324-335): its
    context and Map.take of its rows; `keys` ascending unique key ids."""
    keys = np.asarray(keys, np.uint64)
    return {"rows": _take_rows(rep["rows"], keys), "ctx": rep["ctx"], "keys": keys}


def _draw(k, seed, salt):
    """A per-key pseudo-random u64: splitmix64 of (key, seed, salt) -- every choice of a
    generator that must give the same rows for a key however the key space is sharded."""
    return splitmix64_np(splitmix64_np(k ^ np.uint64((seed * 0x9E3779B97F4A7C15 + salt) & (2**64 - 1)))
                         ^ np.uint64(salt))


def config5(n_keys: int = 100_000_000, n_nodes: int = 64, remove_frac: float = 0.5,
            readd_frac: float = 0.2, ts_range: int = 16, max_entries: int = 3, seed: int = 5,
            nodes: NodeTable | None = None, keys=None, n_total: int | None = None):
    """Config 5, remove-heavy adversarial pair.  Base: every key holds 1..max_entries
    concurrent entries written by distinct nodes of 0..n_nodes-3 (dots {node, c} with
    c = k * max_entries + j + 1 for entry j of key k: unique per node), small values and ts
    in [0, ts_range) so LWW ties are everywhere.  Replicas A (node n_nodes-2) and B (node
    n_nodes-1) each saw the whole base (dense VVs: they cover every dot they hold) and then
    independently removed `remove_frac` of the keys and re-added (add/4: the key's entries
    replaced by one new entry, dot {A or B, k}) `readd_frac` of the rest.  Every choice is
    a function of the key (and seed), so a key-hash shard (`keys`, a subset of
    1..n_total) is exactly that shard's slice of the whole pair, with the pair's full VVs.
    Returns (A, B)."""
    N = nodes or NodeTable(n_nodes, seed)
    k = np.arange(1, n_keys + 1, dtype=np.uint64) if keys is None else np.asarray(keys, np.uint64)
    total = int(n_total if n_total is not None else (int(k.max()) if len(k) else 0))
    n_keys = len(k)
    key = splitmix64_np(k)
    W = n_nodes - 2  # base writers
    me = min(max_entries, W)
    ne = (_draw(k, seed, 1) % np.uint64(me)).astype(np.int64) + 1
    ekey = np.repeat(key, ne)
    E = len(ekey)
    kidx = np.repeat(np.arange(n_keys), ne)
    # entry j of key x comes from writer (h_x + j) mod W: distinct writers per key (a
    # writer's second add to a key would replace its first)
    first = np.r_[0, np.cumsum(ne)[:-1]]
    j = (np.arange(E) - np.repeat(first, ne)).astype(np.uint64)
    h = (_draw(k, seed, 2) % np.uint64(W))
    enode = ((h[kidx] + j) % np.uint64(W)).astype(np.uint32)  # logical writer
    cnt = k[kidx] * np.uint64(me) + j + np.uint64(1)
    ek = k[kidx] * np.uint64(me) + j  # per-entry draws
    eval_ = encode_int_value((_draw(ek, seed, 3) % np.uint64(4)).astype(np.int64))
    ets = (_draw(ek, seed, 4) % np.uint64(ts_range)).astype(np.int64)
    base_vv = {N[w]: total * me + me for w in range(W)}  # covers every base dot
    enode = N.ids(enode).astype(np.uint32)  # the interned (dense) ids of the writers
    reps = []
    for r, node_id in enumerate((n_nodes - 2, n_nodes - 1)):
        u = _draw(k, seed, 10 + r)
        removed = (u % np.uint64(1 << 20)).astype(np.float64) < remove_frac * (1 << 20)
        v = _draw(k, seed, 20 + r)
        readd = (~removed) & ((v % np.uint64(1 << 20)).astype(np.float64) < readd_frac * (1 << 20))
        keep_e = ~(removed | readd)[kidx]
        na = int(readd.sum())
        ak = key[readd]
        av = encode_int_value((_draw(k[readd], seed, 30 + r) % np.uint64(4)).astype(np.int64))
        at = (_draw(k[readd], seed, 40 + r) % np.uint64(ts_range)).astype(np.int64)
        rows = sort_rows(np.concatenate([ekey[keep_e], ak]), np.concatenate([eval_[keep_e], av]),
                         np.concatenate([ets[keep_e], at]),
                         np.concatenate([enode[keep_e], np.full(na, N[node_id], np.uint32)]),
                         np.concatenate([cnt[keep_e], k[readd]]))
        reps.append({"rows": rows, "ctx": vv({**base_vv, N[node_id]: total}), "nodes": N})
    return reps[0], reps[1]
