"""Adversarial inputs for dg_apply_deltas (the keyed delta fold of causal_crdt.ex:383-384):
a state and k deltas drawn from one pool of rows, so the same tuple sits in the state and
in several deltas; keysets that miss keys the delta has rows for (right-biased carry,
aw_lww_map.ex:185-188) and name keys it has no rows for (removals); random version
vectors that cover some dots and not others.  Test data only (seeded numpy)."""
import numpy as np

from delta_crdt_ex_amd.interning import splitmix64_np

VV, DOTS = 0, 1


def _sort_order(key, val, ts, node, cnt):
    return np.lexsort((cnt, node, ts, val, key))


def random_fold(seed, n_keys=2000, k=8, n_nodes=12, rows_per_key=3, hashed=True, node_base=0,
                ctx_node_max=None, dots_ctx=False, p_state=0.6, p_keys=0.06, p_take=0.5,
                p_outside=0.01, p_full=0.0):
    rng = np.random.default_rng(seed)
    ids = np.arange(1, n_keys + 1, dtype=np.uint64)
    keys = splitmix64_np(ids) if hashed else ids
    nr = rng.integers(1, rows_per_key + 1, n_keys)
    E = int(nr.sum())
    kidx = np.repeat(np.arange(n_keys), nr)
    kcol = keys[kidx]
    val = rng.integers(0, 4, E).astype(np.uint64) + np.uint64(1 << 62)
    ts = rng.integers(0, 8, E).astype(np.int64)
    node = (rng.integers(0, n_nodes, E) + node_base).astype(np.uint32)
    cnt = np.zeros(E, np.uint64)
    for nd in np.unique(node):  # dots are unique: counters numbered per node
        w = np.flatnonzero(node == nd)
        cnt[w] = rng.permutation(len(w)).astype(np.uint64) + 1
    o = _sort_order(kcol, val, ts, node, cnt)
    pool = tuple(np.ascontiguousarray(c[o]) for c in (kcol, val, ts, node, cnt))
    pkidx = kidx[o]  # key index of every pool row
    nodes = np.unique(pool[3])
    maxc = {int(nd): int(pool[4][pool[3] == nd].max()) for nd in nodes}

    def take(mask):
        return tuple(c[mask] for c in pool)

    def context():
        if dots_ctx:
            m = rng.random(E) < 0.5
            o = np.lexsort((pool[4][m], pool[3][m]))
            return (DOTS, np.ascontiguousarray(pool[3][m][o]), np.ascontiguousarray(pool[4][m][o]))
        ns = nodes if ctx_node_max is None else nodes[nodes < ctx_node_max]
        ns = ns[rng.random(len(ns)) < 0.8]
        c = np.array([rng.integers(0, maxc[int(x)] + 1) for x in ns], np.uint64)
        return (VV, ns.astype(np.uint32), c)

    state = {"rows": take(rng.random(E) < p_state), "ctx": context()}
    deltas = []
    for _ in range(k):
        kmask = rng.random(n_keys) < p_keys
        in_k = kmask[pkidx]
        # rows of the delta's keys, plus a few rows of keys outside its keyset
        rmask = (in_k & (rng.random(E) < p_take)) | (~in_k & (rng.random(E) < p_outside))
        full = rng.random() < p_full
        ks = None if full else np.sort(keys[kmask])
        deltas.append({"rows": take(rmask), "ctx": context(), "keys": ks})
    return state, deltas
