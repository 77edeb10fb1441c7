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
                p_outside=0.01, p_full=0.0, delta_dots=False):
    """dots_ctx: every context a dot set (the state's too); delta_dots: the deltas'
    contexts dot sets (MapSet deltas, aw_lww_map.ex:124-146), the state's a VV."""
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

    def context(dots=False):
        if dots_ctx or dots:
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
        deltas.append({"rows": take(rmask), "ctx": context(delta_dots), "keys": ks})
    return state, deltas


def mutation_fold(seed, n_keys=20_000, k=16, ops=300, p_remove=0.3, p_new=0.3):
    """k mutation deltas, each a batch of add/remove ops by its own replica against the
    same state (concurrent replicas' mutate_async batches), as dg_mutate_batch / the
    reference's add/remove build them (aw_lww_map.ex:99-146): dot-set contexts (the
    touched keys' dots plus every add's fresh dot) and keys = the touched keys.  The
    state is a VV replica.  Folding them with their keys is applying them in order."""
    from oracle import ref as R
    rng = np.random.default_rng(seed)
    st, _ = random_fold(seed, n_keys=n_keys, k=0, n_nodes=6, rows_per_key=2, p_state=0.8)
    st = {"rows": st["rows"], "ctx": st["ctx"]}
    keys = np.unique(st["rows"][0])
    deltas = []
    for i in range(k):
        node = 100 + i  # a replica of its own
        batch = []
        for j in range(ops):
            r = rng.random()
            if r < p_remove:
                batch.append(("remove", int(rng.choice(keys)), 0, 0))
            elif r < p_remove + p_new:
                batch.append(("add", int(splitmix64_np(np.array([rng.integers(1 << 40)],
                                                               np.uint64))[0]),
                              int(rng.integers(1 << 30)) + (1 << 62), 10**9 + j))
            else:
                batch.append(("add", int(rng.choice(keys)), int(rng.integers(1 << 30)) + (1 << 62),
                              10**9 + j))
        batch.sort(key=lambda o: o[1])  # by key, batch order within a key (stable)
        rows, ctx, ks = R.mutate_batch(st["rows"], st["ctx"], node, batch)
        deltas.append({"rows": rows, "ctx": ctx, "keys": ks})
    return st, deltas
