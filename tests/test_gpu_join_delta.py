"""dg_join_delta: CausalCrdt.update_state_with_delta (causal_crdt.ex:383-404) on a
device-resident state -- the keyed join with a sync delta (in place when every joined key
keeps its row count, through the spare store otherwise), the changed keys (diff/3) and
the MerkleMap update -- bit-exact against the C oracle's keyed join, its changed keys and
a fresh tree of the joined state."""
import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Context, MerkleTree, Store, TermHashes, u64
from oracle import ref as R
from test_gpu_parity import DEV, ctx_eq, rows_eq

pytestmark = pytest.mark.gpu


def kdev(keys):
    return torch.from_numpy(np.ascontiguousarray(keys, np.uint64).view(np.int64)).to(DEV)


def state_of(rep, extra_ctx=64):
    rows, ctx = rep["rows"], rep["ctx"]
    s = Store.from_numpy(*rows, device=DEV)
    c = Context.empty(ctx[0], len(ctx[1]) + extra_ctx, DEV)
    c.node[: len(ctx[1])].copy_(torch.from_numpy(ctx[1].view(np.int32)))
    c.cnt[: len(ctx[2])].copy_(torch.from_numpy(ctx[2].view(np.int64)))
    c.n = len(ctx[1])
    return s, c


def up(rep):
    rows, ctx = rep["rows"], rep["ctx"]
    return Store.from_numpy(*rows, device=DEV), Context.from_numpy(ctx[0], ctx[1], ctx[2], DEV)


def apply(engine, a, d, keys, depth=10, terms=None, with_tree=True, home=False):
    """home: through dg_join_delta_home (the fused small-delta path, one host wait), which
    must take the delta (no DG_HOME_FALLBACK) and give what dg_join_delta_rows gives."""
    keys = np.unique(np.asarray(keys, np.uint64))
    st, sc = state_of(a, extra_ctx=len(d["ctx"][1]))
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, depth, MerkleTree.empty(depth, DEV, terms=terms)) if with_tree else None
    wr, wc = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=keys)
    wch = R.changed_keys(a["rows"], wr, keys)
    if home:
        got = engine.join_delta_home(st, sc, sd, cd, kdev(keys), spare, tree)
        assert got is not None, "the small path declined"
        changed, hrows, hctx, swapped = got
        assert np.array_equal(changed, wch)
        want_rows = tuple(c[np.isin(wr[0], wch)] for c in wr)
        for x, y in zip(hrows, want_rows):
            assert np.array_equal(x, y)
        assert np.array_equal(hctx[0], wc[1]) and np.array_equal(hctx[1], wc[2])
    else:
        # (dg_join_delta_rows: the changed keys' joined rows come back too, taken from the
        # join's edit of the keyset on the in-place and moved paths)
        rows = Store.empty(st.n + sd.n, DEV)
        changed, swapped = engine.join_delta(st, sc, sd, cd, kdev(keys), spare, tree, rows=rows)
        assert np.array_equal(u64(changed), wch)
        rows_eq(rows, tuple(c[np.isin(wr[0], wch)] for c in wr))
    rows_eq(st, wr)
    ctx_eq(sc, wc)
    if with_tree:
        fresh = engine.merkle_build(st, depth, MerkleTree.empty(depth, DEV, terms=terms))
        assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
        assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())
        assert tree.n_keys == fresh.n_keys
        # the chunk index moved with the rows (dg_merkle.starts)
        assert np.array_equal(tree.starts.cpu().numpy(), fresh.starts.cpu().numpy())
    return st, sc, swapped, wr


def test_sync_delta_in_place(engine):
    """Config-4 shaped: every differing key's one row is replaced by one row -- nothing
    outside the keyset moves; the tree over node terms follows."""
    a, b = W.config4_shard(2, 8, keys_per_rank=80_000, diff_frac=0.01)
    want = R.store_diff(a["rows"], b["rows"])
    terms = TermHashes(*a["nodes"].universe.term_tables(), DEV)
    st, sc, swapped, _ = apply(engine, a, W.sync_delta(b, want), want, depth=14, terms=terms)
    assert not swapped
    rows_eq(st, R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])[0])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sync_delta_with_moves(engine, seed):
    """Random replicas: joined keys gain and lose rows (concurrent adds, removes), so the
    rows outside the keyset move -- through the spare store."""
    rng = np.random.default_rng(seed)
    a, b = W.random_pair(rng, 20_000, n_nodes=5, ts_range=1 << 10, dense_ctx=bool(seed % 2))
    kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    keys = np.sort(rng.choice(kb, 300, replace=False))
    _, _, swapped, _ = apply(engine, a, W.sync_delta(b, keys), keys)
    assert swapped


def test_not_a_sync_delta_takes_the_full_join(engine):
    rng = np.random.default_rng(9)
    a, b = W.random_pair(rng, 20_000, n_nodes=4)
    kb = np.unique(b["rows"][0])
    keys = kb[::100]
    d = W.sync_delta(b, np.union1d(keys, kb[7:9]))  # two delta keys outside the keyset
    # (no tree check: like the reference's MerkleMap, the tree follows the changed keys
    # of the keyset only -- diff/3 over `keys`, causal_crdt.ex:386-394 -- so the carried
    # keys' leaves stay as they were)
    apply(engine, a, d, keys, with_tree=False)


def test_changed_rows_past_their_capacity(engine):
    """dg_join_delta_rows with a rows buffer too small: the join is complete (state,
    context, changed keys as with room), rows.n reports how many rows there are, and
    dg_take_keys of the changed keys returns them."""
    a, b = W.config4_shard(1, 8, keys_per_rank=40_000, diff_frac=0.02)
    want = R.store_diff(a["rows"], b["rows"])
    d = W.sync_delta(b, want)
    st, sc = state_of(a, extra_ctx=8)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    small = Store.empty(3, DEV)
    changed, _ = engine.join_delta(st, sc, sd, cd, kdev(want), spare, None, rows=small)
    wr, wc = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=want)
    rows_eq(st, wr)
    ctx_eq(sc, wc)
    wch = R.changed_keys(a["rows"], wr, want)
    assert np.array_equal(u64(changed), wch)
    sel = np.isin(wr[0], wch)
    assert small.n == int(sel.sum()) > small.cap
    rows_eq(engine.take_keys(st, changed), tuple(c[sel] for c in wr))


def test_applied_twice_changes_nothing(engine):
    a, b = W.config4_shard(0, 8, keys_per_rank=40_000, diff_frac=0.02)
    want = R.store_diff(a["rows"], b["rows"])
    d = W.sync_delta(b, want)
    st, sc = state_of(a, extra_ctx=8)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, 12)
    c1, _ = engine.join_delta(st, sc, sd, cd, kdev(want), spare, tree)
    root = tree.root()
    c2, sw2 = engine.join_delta(st, sc, sd, cd, kdev(want), spare, tree)
    assert c1.numel() == len(want) and c2.numel() == 0 and not sw2 and tree.root() == root
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(st, wr)


def test_join_delta_edges(engine):
    """An empty keyset, an empty delta, and a state that is empty."""
    rng = np.random.default_rng(4)
    a, b = W.random_pair(rng, 5_000, n_nodes=3)
    kb = np.unique(b["rows"][0])
    # empty keyset (the delta's keys all outside it: the right-biased carry replaces them)
    apply(engine, a, W.sync_delta(b, kb[:10]), np.zeros(0, np.uint64), with_tree=False)
    # a delta without rows, keyset of present keys: removals only
    empty = {"rows": tuple(c[:0] for c in b["rows"]), "ctx": b["ctx"]}
    apply(engine, a, empty, np.unique(a["rows"][0])[::50])
    # an empty state receiving a sync delta
    none = {"rows": tuple(c[:0] for c in a["rows"]), "ctx": a["ctx"]}
    apply(engine, none, W.sync_delta(b, kb[::20]), kb[::20], with_tree=False)


# ---------------------------------------------------------------- local mutations
# handle_operation (causal_crdt.ex:337-342): every mutate is a one-key delta whose context
# is a MapSet (aw_lww_map.ex:124-146), joined into the replica's VV state with keys = [key]
# through update_state_with_delta (:383-404) -- the path INTEGRATION.md routes to
# dg_join_delta on a GPU-attached state.

def _mutation_state(n_keys=20_000, seed=31):
    rng = np.random.default_rng(seed)
    a, _ = W.random_pair(rng, n_keys, n_nodes=4, max_entries=2)
    return a, rng


@pytest.mark.parametrize("home", [False, True])
@pytest.mark.parametrize("case", ["update", "new_key", "remove", "remove_absent", "nil_value",
                                  "same_value"])
def test_one_key_mutation_delta(engine, case, home):
    """A one-key add/remove delta with a dot-set context into a VV state: rows, context,
    changed keys and the tree against the C oracle and a fresh build.  `update` keeps the
    key's row count (in place when the key held one row), `new_key` and `remove` move rows
    (through the spare store), `remove_absent` changes nothing."""
    a, rng = _mutation_state()
    keys = np.unique(a["rows"][0])
    counts = np.bincount(np.searchsorted(keys, a["rows"][0]), minlength=len(keys))
    one = keys[counts == 1]
    node = int(a["ctx"][1][0])
    nil_id = (1 << 63) - 12345  # the interned id of :nil (any value id; the join never reads it)
    if case == "update":
        ops = [("add", int(one[17]), 424242, 10 ** 12)]
    elif case == "same_value":
        k = int(one[3])
        v = int(a["rows"][1][np.searchsorted(a["rows"][0], k)])
        ops = [("add", k, v, 10 ** 12)]
    elif case == "nil_value":
        ops = [("add", int(one[5]), nil_id, 10 ** 12)]
    elif case == "new_key":
        k = int(keys[100]) + 1
        assert k not in set(keys.tolist())
        ops = [("add", k, 7, 10 ** 12)]
    elif case == "remove":
        ops = [("remove", int(keys[len(keys) // 2]), 0, 0)]
    else:
        ops = [("remove", int(keys[200]) + 1, 0, 0)]
    drows, dctx, dkeys = R.mutate_batch(a["rows"], a["ctx"], node, ops)
    d = {"rows": drows, "ctx": dctx}
    st, sc, swapped, wr = apply(engine, a, d, dkeys, depth=12, home=home)
    assert swapped == (case in ("new_key", "remove"))
    assert sc.kind == 0  # map ⊔ MapSet folds the dots into the VV (aw_lww_map.ex:45-52)


def test_mutation_sequence_matches_the_oracle(engine):
    """200 mutations in a row (adds of new and existing keys, removes, re-adds), each its
    own dg_join_delta on one resident state + tree, against the oracle's fold."""
    a, rng = _mutation_state(n_keys=30_000, seed=32)
    st, sc = state_of(a, extra_ctx=4)
    spare = Store.empty(st.n + 8, DEV)
    tree = engine.merkle_build(st, 12)
    rows, ctx = a["rows"], a["ctx"]
    node = int(ctx[1][1])
    keys = np.unique(rows[0])
    for i in range(200):
        r = rng.random()
        if r < 0.4:
            op = ("add", int(rng.choice(keys)), int(rng.integers(1 << 40)), 10 ** 12 + i)
        elif r < 0.7:
            op = ("add", int(rng.integers(1 << 63)) | 1, int(rng.integers(1 << 40)), 10 ** 12 + i)
        else:
            op = ("remove", int(rng.choice(keys)), 0, 0)
        drows, dctx, dkeys = R.mutate_batch(rows, ctx, node, [op])
        sd, cd = up({"rows": drows, "ctx": dctx})
        if spare.cap < st.n + sd.n:
            spare = Store.empty(st.n + sd.n + 64, DEV)
        changed, _ = engine.join_delta(st, sc, sd, cd, kdev(dkeys), spare, tree)
        wr, wc = R.join2(rows, ctx, drows, dctx, keys=dkeys)
        assert np.array_equal(u64(changed), R.changed_keys(rows, wr, dkeys))
        rows, ctx = wr, wc
    rows_eq(st, rows)
    ctx_eq(sc, ctx)
    fresh = engine.merkle_build(st, 12)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    assert tree.n_keys == fresh.n_keys


# ---------------------------------------------------------------- all or nothing

def _snapshot(st, sc, tree):
    return ([c.copy() for c in st.to_numpy()], [c.copy() for c in sc.to_numpy()], sc.kind,
            tree.nodes.cpu().numpy().copy(), tree.bucket_counts().copy(), tree.n_keys,
            tree.starts.cpu().numpy().copy())


def _assert_unchanged(st, sc, tree, snap):
    rows, ctx, kind, nodes, counts, nk, starts = snap
    assert np.array_equal(tree.starts.cpu().numpy(), starts)
    for x, y in zip(st.to_numpy(), rows):
        assert np.array_equal(x, y)
    for x, y in zip(sc.to_numpy(), ctx):
        assert np.array_equal(x, y)
    assert sc.kind == kind
    assert np.array_equal(tree.nodes.cpu().numpy(), nodes)
    assert np.array_equal(tree.bucket_counts(), counts)
    assert tree.n_keys == nk


def _rows(keys, node, cnt0):
    n = len(keys)
    return (np.asarray(keys, np.uint64), np.arange(n, dtype=np.uint64) + 5, np.full(n, 1, np.int64),
            np.full(n, node, np.uint32), np.arange(n, dtype=np.uint64) + cnt0)


def test_failed_tree_update_leaves_the_state_alone(engine):
    """A delta whose joined rows overflow a bucket's 16-bit row count (depth-1 tree,
    65530 rows in bucket 0, 10 new keys there): DG_E_CAPACITY, and the state's rows,
    context and tree are exactly what they were (the moved path: rows go to the spare)."""
    from delta_crdt_ex_amd._abi import CapacityError
    rng = np.random.default_rng(5)
    keys = np.unique(rng.integers(0, 1 << 63, 65540, dtype=np.uint64))
    low, extra = keys[:65530], keys[65530:65540]
    a = {"rows": _rows(low, 0, 1), "ctx": (0, np.array([0], np.uint32), np.array([65530], np.uint64))}
    d = {"rows": _rows(extra, 1, 1), "ctx": (0, np.array([1], np.uint32), np.array([10], np.uint64))}
    st, sc = state_of(a, extra_ctx=1)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, 1)
    snap = _snapshot(st, sc, tree)
    with pytest.raises(CapacityError, match="65535"):
        engine.join_delta(st, sc, sd, cd, kdev(extra), spare, tree)
    _assert_unchanged(st, sc, tree, snap)
    # the engine is usable afterwards: a deeper tree takes the same delta
    apply(engine, a, d, extra, depth=8)


def test_failed_tree_update_full_join_path(engine):
    """A keyset key outside the tree's key-hash shard changes (DG_E_INVAL), on the path of
    a delta with a key outside its keyset (the full join into the spare store)."""
    from delta_crdt_ex_amd._abi import DeltaGpuError
    rng = np.random.default_rng(6)
    low = np.unique(rng.integers(0, 1 << 63, 5000, dtype=np.uint64))      # shard 0 of 2
    out_key = np.array([(1 << 63) + 77], np.uint64)                        # shard 1
    stray = np.array([int(low[10]) + 1], np.uint64)                        # outside the keyset
    dk = np.sort(np.concatenate([out_key, stray]))
    a = {"rows": _rows(low, 0, 1), "ctx": (0, np.array([0], np.uint32), np.array([5000], np.uint64))}
    d = {"rows": _rows(dk, 1, 1), "ctx": (0, np.array([1], np.uint32), np.array([2], np.uint64))}
    st, sc = state_of(a, extra_ctx=1)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, 8, shard_bits=1, shard=0)
    snap = _snapshot(st, sc, tree)
    with pytest.raises(DeltaGpuError, match="shard"):
        engine.join_delta(st, sc, sd, cd, kdev(out_key), spare, tree)
    _assert_unchanged(st, sc, tree, snap)


def test_failed_tree_update_in_place_path(engine):
    """The in-place path: a key outside the tree's shard keeps its row count but changes
    (the tree was built over the shard's rows only); E's rows and the context are written
    by kernels that see the failed update and skip, so nothing changes."""
    from delta_crdt_ex_amd._abi import DeltaGpuError
    rng = np.random.default_rng(7)
    low = np.unique(rng.integers(0, 1 << 63, 5000, dtype=np.uint64))
    x = np.array([(1 << 63) + 99], np.uint64)
    allk = np.concatenate([low, x])
    a = {"rows": _rows(allk, 0, 1), "ctx": (0, np.array([0], np.uint32), np.array([5001], np.uint64))}
    inside = {"rows": tuple(c[:-1] for c in a["rows"]), "ctx": a["ctx"]}
    d = {"rows": (x, np.array([999], np.uint64), np.array([2], np.int64), np.array([1], np.uint32),
                  np.array([1], np.uint64)),
         "ctx": (0, np.array([0, 1], np.uint32), np.array([5001, 1], np.uint64))}
    st, sc = state_of(a, extra_ctx=2)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    si, _ = up(inside)
    tree = engine.merkle_build(si, 8, shard_bits=1, shard=0)
    snap = _snapshot(st, sc, tree)
    with pytest.raises(DeltaGpuError, match="shard"):
        engine.join_delta(st, sc, sd, cd, kdev(x), spare, tree)
    _assert_unchanged(st, sc, tree, snap)


def test_join_delta_retries_an_aborted_grid(monkeypatch):
    """the splice's edit join on an over-sized persistent grid
    (DG_JOIN_WORKERS=1024, 512 fit) aborts; dg_join_delta re-runs the edit on a small grid
    (nothing of the state is written before) and ends equal to a co-resident engine."""
    from delta_crdt_ex_amd.store import Engine
    a, b = W.config4_shard(1, 8, keys_per_rank=5_000_000, diff_frac=0.06)
    want = R.store_diff(a["rows"], b["rows"])
    d = W.sync_delta(b, want)
    results = []
    for workers in (None, "1024"):
        if workers:
            monkeypatch.setenv("DG_JOIN_WORKERS", workers)
        eng = Engine(0)
        st, sc = state_of(a, extra_ctx=8)
        sd, cd = up(d)
        spare = Store.empty(st.n + sd.n, DEV)
        tree = eng.merkle_build(st, 16)
        changed, _ = eng.join_delta(st, sc, sd, cd, kdev(want), spare, tree)
        results.append(([c.copy() for c in st.to_numpy()], u64(changed).copy(), tree.root()))
        eng.close()
    (r0, c0, t0), (r1, c1, t1) = results
    assert len(c0) > 200_000 and np.array_equal(c0, c1) and t0 == t1
    for x, y in zip(r0, r1):
        assert np.array_equal(x, y)


# ---------------------------------------------------------------- dg_join_delta_home
# The fused small-delta path (csrc/small.hip): one launch chain, one host wait, the
# result in page-locked memory -- what the NIF's join_delta / mutate_batch use for
# mutations and small sync deltas (c_src/replica.c).

@pytest.mark.parametrize("n_keys", [30_000, 300_000])
def test_mutation_sequence_home(engine, n_keys):
    """200 one-key mutations through dg_join_delta_home on one resident state + tree
    (30k rows: the moved-rows copy is enqueued behind the join; 300k: after the wait),
    against the oracle's fold, step by step."""
    a, rng = _mutation_state(n_keys=n_keys, seed=33)
    st, sc = state_of(a, extra_ctx=4)
    spare = Store.empty(st.n + 300, DEV)
    tree = engine.merkle_build(st, 14)
    rows, ctx = a["rows"], a["ctx"]
    node = int(ctx[1][1])
    keys = np.unique(rows[0])
    moved = 0
    for i in range(200):
        r = rng.random()
        if r < 0.4:
            op = ("add", int(rng.choice(keys)), int(rng.integers(1 << 40)), 10 ** 12 + i)
        elif r < 0.7:
            op = ("add", int(rng.integers(1 << 63)) | 1, int(rng.integers(1 << 40)), 10 ** 12 + i)
        else:
            op = ("remove", int(rng.choice(keys)), 0, 0)
        drows, dctx, dkeys = R.mutate_batch(rows, ctx, node, [op])
        sd, cd = up({"rows": drows, "ctx": dctx})
        if spare.cap < st.n + sd.n:  # (after a swap the spare is the old state's buffer)
            spare = Store.empty(st.n + sd.n + 64, DEV)
        got = engine.join_delta_home(st, sc, sd, cd, kdev(dkeys), spare, tree)
        assert got is not None
        changed, hrows, hctx, swapped = got
        moved += swapped
        wr, wc = R.join2(rows, ctx, drows, dctx, keys=dkeys)
        wch = R.changed_keys(rows, wr, dkeys)
        assert np.array_equal(changed, wch)
        for x, y in zip(hrows, tuple(c[np.isin(wr[0], wch)] for c in wr)):
            assert np.array_equal(x, y)
        assert np.array_equal(hctx[0], wc[1]) and np.array_equal(hctx[1], wc[2])
        rows, ctx = wr, wc
    assert moved > 20
    rows_eq(st, rows)
    ctx_eq(sc, ctx)
    fresh = engine.merkle_build(st, 14)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())
    assert np.array_equal(tree.starts.cpu().numpy(), fresh.starts.cpu().numpy())
    assert tree.n_keys == fresh.n_keys


@pytest.mark.parametrize("seed", [0, 1])
def test_small_sync_deltas_home(engine, seed):
    """Sync deltas of a few hundred keys: with moves (random replicas, VV or dot-set
    contexts) and in place over node terms (config-4 shaped)."""
    rng = np.random.default_rng(40 + seed)
    a, b = W.random_pair(rng, 20_000, n_nodes=5, ts_range=1 << 10, dense_ctx=bool(seed))
    kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    keys = np.sort(rng.choice(kb, 120, replace=False))  # (<= 512 delta rows)
    d = W.sync_delta(b, keys)
    assert len(d["rows"][0]) <= 512
    # (depth 10: one chunk; 18: 128 chunks, every bucket path its own up to level ~7 and
    # the chunk index moved past each changed chunk)
    apply(engine, a, d, keys, depth=10 if seed == 0 else 18, home=True)
    a, b = W.config4_shard(seed, 8, keys_per_rank=30_000, diff_frac=0.01)
    want = R.store_diff(a["rows"], b["rows"])
    assert 0 < len(want) <= 512
    terms = TermHashes(*a["nodes"].universe.term_tables(), DEV)
    _, _, swapped, _ = apply(engine, a, W.sync_delta(b, want), want, depth=13, terms=terms, home=True)
    assert not swapped


def test_home_declines_and_leaves_the_state(engine):
    """A delta with a key outside the keyset (the right-biased carry: the general path),
    or more keys than the small path takes: DG_HOME_FALLBACK, nothing touched."""
    rng = np.random.default_rng(5)
    a, b = W.random_pair(rng, 8_000, n_nodes=3)
    kb = np.unique(b["rows"][0])
    st, sc = state_of(a, extra_ctx=8)
    tree = engine.merkle_build(st, 11)
    snap = _snapshot(st, sc, tree)
    for keys, dkeys in ((kb[:20], kb[:22]), (kb[:600], kb[:600])):
        sd, cd = up(W.sync_delta(b, dkeys))
        spare = Store.empty(st.n + sd.n, DEV)
        assert engine.join_delta_home(st, sc, sd, cd, kdev(keys), spare, tree) is None
        _assert_unchanged(st, sc, tree, snap)


@pytest.mark.parametrize("with_tree", [False, True])
def test_home_from_an_empty_state(engine, with_tree):
    """A replica's first mutations (causal_crdt.ex:337-342 on a fresh AWLWWMap): the small
    path from an empty state -- no state rows to search or move -- then more adds and a
    remove, each against the oracle's fold (and a fresh tree)."""
    rows = (np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.int64),
            np.zeros(0, np.uint32), np.zeros(0, np.uint64))
    ctx = (R.VV, np.array([0], np.uint32), np.array([0], np.uint64))
    st = Store.empty(64, DEV)
    sc = Context.empty(R.VV, 8, DEV)
    sc.node[0] = 0
    sc.cnt[0] = 0
    sc.n = 1
    spare = Store.empty(64, DEV)
    tree = engine.merkle_build(st, 6) if with_tree else None
    ops = [("add", 5 << 58, 7, 100), ("add", 3 << 60, 8, 101), ("add", 5 << 58, 9, 102),
           ("remove", 3 << 60, 0, 0), ("add", 1, 1, 103)]
    for op in ops:
        drows, dctx, dkeys = R.mutate_batch(rows, ctx, 0, [op])
        sd, cd = up({"rows": drows, "ctx": dctx})
        got = engine.join_delta_home(st, sc, sd, cd, kdev(dkeys), spare, tree)
        assert got is not None
        changed, hrows, hctx, swapped = got
        if swapped:
            spare = Store.empty(64, DEV)
        wr, wc = R.join2(rows, ctx, drows, dctx, keys=dkeys)
        assert np.array_equal(changed, R.changed_keys(rows, wr, dkeys))
        rows, ctx = wr, wc
        rows_eq(st, rows)
        ctx_eq(sc, ctx)
        if with_tree:
            fresh = engine.merkle_build(st, 6)
            assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
            assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())


# ---------------------------------------------------------------- wave_find
# The small path's per-key search (small.hip wave_find): its first row and run, against
# np.searchsorted, at the sizes where the 64-ary narrowing ends on a window edge (every n in
# [2^20, 1040^2) leaves hi - lo = 64 after the first round) and on shard-prefixed keys (the
# interpolated probe misses: 64-ary rounds from the whole range).

def _wave_find(a, q):
    import ctypes as C
    from delta_crdt_ex_amd import _abi
    f = _abi.load().dg_debug_wave_find
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    da, dq = kdev(a), kdev(q)
    lo = torch.empty(len(q), dtype=torch.int64, device=DEV)
    run = torch.empty(len(q), dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    assert f(da.data_ptr(), len(a), dq.data_ptr(), len(q), lo.data_ptr(), run.data_ptr()) == 0
    return u64(lo), run.cpu().numpy()


def _keys_with_runs(rng, n, prefix_bits=0, prefix=0):
    u = np.unique(rng.integers(0, 1 << 63, n, dtype=np.uint64) >> np.uint64(prefix_bits))
    if prefix_bits:
        u = u | np.uint64(prefix << (64 - prefix_bits))
    reps = rng.choice([1, 1, 1, 2, 3], len(u))
    a = np.repeat(u, reps)[:n]
    return a, u


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 10_000, 1 << 20, (1 << 20) + 1, 1_060_000, 1040 ** 2 - 1,
                               1040 ** 2, 3_000_000])
@pytest.mark.parametrize("prefix_bits", [0, 3])
def test_wave_find_matches_searchsorted(n, prefix_bits):
    rng = np.random.default_rng(n + prefix_bits)
    a, u = _keys_with_runs(rng, n, prefix_bits, 5)
    assert len(a) == n
    q = np.concatenate([np.unique(a), (np.unique(a) + np.uint64(1)) if n else a,
                        np.array([0, (1 << 64) - 1, 5 << 61], np.uint64)])
    lo, run = _wave_find(a, q)
    want_lo = np.searchsorted(a, q, side="left")
    want_run = np.searchsorted(a, q, side="right") - want_lo
    bad = np.nonzero((lo != want_lo) | (run != want_run))[0]
    assert len(bad) == 0, (n, prefix_bits, len(bad), q[bad[:4]], lo[bad[:4]], want_lo[bad[:4]], run[bad[:4]])


def _unique_key_state(rng, n, prefix_bits=0, prefix=0):
    """n rows, one per key (node 0..3 round robin), VV covering them all."""
    keys = np.unique(rng.integers(0, 1 << 63, n + n // 50, dtype=np.uint64) >> np.uint64(prefix_bits))[:n]
    if prefix_bits:
        keys = keys | np.uint64(prefix << (64 - prefix_bits))
    assert len(keys) == n
    node = (np.arange(n) % 4).astype(np.uint32)
    cnt = (np.arange(n) // 4 + 1).astype(np.uint64)
    rows = (keys, rng.integers(0, 1 << 40, n).astype(np.uint64), np.full(n, 7, np.int64), node, cnt)
    ctx = (R.VV, np.arange(4, dtype=np.uint32), np.full(4, (n + 3) // 4, np.uint64))
    return {"rows": rows, "ctx": ctx}


@pytest.mark.parametrize("n_rows,prefix_bits", [(1_060_000, 0), (1_060_000, 3)])
def test_mutation_sequence_home_1m(engine, n_rows, prefix_bits):
    """one-key mutations through dg_join_delta_home on a 1.06M-row state (where
    wave_find's narrowing ends on the window edge) and on a shard-prefixed one, each step
    against R.join2 (rows of changed keys and context) and the state at the end."""
    rng = np.random.default_rng(n_rows + prefix_bits)
    a = _unique_key_state(rng, n_rows, prefix_bits, 6)
    st, sc = state_of(a, extra_ctx=4)
    spare = Store.empty(st.n + 300, DEV)
    tree = engine.merkle_build(st, 16, shard_bits=prefix_bits, shard=6 if prefix_bits else 0)
    rows, ctx = a["rows"], a["ctx"]
    keys = rows[0]
    # every key whose first row sits on a probe edge is as likely as any: 300 ops over
    # existing keys, plus new keys and removes
    for i in range(300):
        r = rng.random()
        if r < 0.5:
            op = ("add", int(rng.choice(keys)), int(rng.integers(1 << 40)), 10 ** 12 + i)
        elif r < 0.65:
            k = int(rng.integers(1 << 63) >> prefix_bits) | (6 << (64 - prefix_bits) if prefix_bits else 0)
            op = ("add", k, int(rng.integers(1 << 40)), 10 ** 12 + i)
        else:
            op = ("remove", int(rng.choice(keys)), 0, 0)
        drows, dctx, dkeys = R.mutate_batch(rows, ctx, 2, [op])
        sd, cd = up({"rows": drows, "ctx": dctx})
        if spare.cap < st.n + sd.n:
            spare = Store.empty(st.n + sd.n + 64, DEV)
        got = engine.join_delta_home(st, sc, sd, cd, kdev(dkeys), spare, tree)
        assert got is not None
        changed, hrows, hctx, _ = got
        wr, wc = R.join2(rows, ctx, drows, dctx, keys=dkeys)
        wch = R.changed_keys(rows, wr, dkeys)
        assert np.array_equal(changed, wch), (i, op)
        for x, y in zip(hrows, tuple(c[np.isin(wr[0], wch)] for c in wr)):
            assert np.array_equal(x, y), (i, op)
        rows, ctx = wr, wc
    rows_eq(st, rows)
    ctx_eq(sc, ctx)
    fresh = engine.merkle_build(st, 16, shard_bits=prefix_bits, shard=6 if prefix_bits else 0)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())


@pytest.mark.parametrize("home", [False, True])
def test_counter_zero_dots(engine, home):
    """a dot with counter 0 on a node absent from a VV is covered
    (Map.get(vv, node, 0) >= 0, aw_lww_map.ex:67-70) on the small and the general path
    alike: the delta's cnt-0 row is dropped, and a state row with cnt 0 on a node the
    delta's VV lacks goes."""
    rng = np.random.default_rng(77)
    n = 2000
    keys = np.unique(rng.integers(0, 1 << 63, n + 50, dtype=np.uint64))[:n]
    node = np.zeros(n, np.uint32)
    cnt = np.arange(1, n + 1, dtype=np.uint64)
    node[10], cnt[10] = 3, 0  # (node 3 is in no VV)
    a = {"rows": (keys, np.arange(n, dtype=np.uint64), np.full(n, 5, np.int64), node, cnt),
         "ctx": (R.VV, np.array([0], np.uint32), np.array([n], np.uint64))}
    dk = np.sort(np.array([keys[10], keys[20], keys[30]], np.uint64))
    d = {"rows": (dk, np.array([7, 8, 9], np.uint64), np.full(3, 9, np.int64), np.full(3, 7, np.uint32),
                  np.array([0, 0, 1], np.uint64)),
         "ctx": (R.VV, np.array([7], np.uint32), np.array([1], np.uint64))}
    st, sc, _, wr = apply(engine, a, d, dk, depth=8, home=home)
    assert not (wr[3] == 3).any() and not ((wr[3] == 7) & (wr[4] == 0)).any() and ((wr[3] == 7) & (wr[4] == 1)).any()


# ---------------------------------------------------------------- the one-wait path (kdelta.hip)
# dg_join_delta's per-key path for deltas of any size: its fallbacks leave nothing written,
# and it equals the splice path (DG_KD=0) bit for bit.

def _kd_engine(monkeypatch, on):
    from delta_crdt_ex_amd.store import Engine
    monkeypatch.setenv("DG_KD", "1" if on else "0")
    return Engine(0)


@pytest.mark.parametrize("seed", [3, 4])
def test_kd_equals_the_splice_path(monkeypatch, seed):
    """Sync deltas with moves and with dot-set contexts, through both paths on fresh
    engines: the same state, context, changed keys, rows and tree."""
    rng = np.random.default_rng(seed)
    a, b = W.random_pair(rng, 30_000, n_nodes=6, ts_range=1 << 10, dense_ctx=bool(seed % 2))
    kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    keys = np.sort(rng.choice(kb, 4_000, replace=False))
    d = W.sync_delta(b, keys)
    out = []
    for on in (True, False):
        eng = _kd_engine(monkeypatch, on)
        st, sc = state_of(a, extra_ctx=len(d["ctx"][1]))
        sd, cd = up(d)
        spare = Store.empty(st.n + sd.n, DEV)
        rows = Store.empty(st.n + sd.n, DEV)
        tree = eng.merkle_build(st, 12)
        changed, swapped = eng.join_delta(st, sc, sd, cd, kdev(keys), spare, tree, rows=rows)
        out.append(([c.copy() for c in st.to_numpy()], [c.copy() for c in sc.to_numpy()], u64(changed).copy(),
                    [c.copy() for c in rows.to_numpy()], tree.nodes.cpu().numpy().copy(),
                    tree.starts.cpu().numpy().copy(), tree.n_keys, swapped))
        eng.close()
    x, y = out
    for p, q in zip(x[:2], y[:2]):
        for c1, c2 in zip(p, q):
            assert np.array_equal(c1, c2)
    assert np.array_equal(x[2], y[2])
    for c1, c2 in zip(x[3], y[3]):
        assert np.array_equal(c1, c2)
    assert np.array_equal(x[4], y[4]) and np.array_equal(x[5], y[5]) and x[6] == y[6] and x[7] == y[7]
    wr, _ = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=keys)
    assert all(np.array_equal(c1, c2) for c1, c2 in zip(x[0], wr))


def test_kd_long_key_runs_fall_back(engine):
    """A key with more rows than the per-key path takes (KD_RUN = 64): the call still
    applies (the splice path), equal to the oracle, and the tree equals a fresh build."""
    rng = np.random.default_rng(12)
    n = 5000
    keys = np.unique(rng.integers(0, 1 << 63, n + 10, dtype=np.uint64))[:n]
    big = keys[100]
    rk = np.concatenate([keys, np.full(79, big, np.uint64)])
    node = np.zeros(len(rk), np.uint32)
    cnt = np.arange(1, len(rk) + 1, dtype=np.uint64)
    val = np.arange(len(rk), dtype=np.uint64)
    order = np.lexsort((cnt, node, np.zeros(len(rk)), val, rk))
    rows = (rk[order], val[order], np.full(len(rk), 3, np.int64), node[order], cnt[order])
    a = {"rows": rows, "ctx": (R.VV, np.array([0], np.uint32), np.array([len(rk)], np.uint64))}
    dk = np.sort(np.array([big, keys[7]], np.uint64))
    d = {"rows": (dk, np.array([1, 2], np.uint64), np.full(2, 9, np.int64), np.full(2, 1, np.uint32),
                  np.array([1, 2], np.uint64)),
         "ctx": (R.VV, np.array([0, 1], np.uint32), np.array([len(rk), 2], np.uint64))}
    apply(engine, a, d, dk, depth=9)


def test_kd_changed_keys_past_their_capacity(engine):
    """More changed keys than the caller's buffer: DG_E_CAPACITY, and the state, context and
    tree are exactly what they were (the count kernel's tree update undone)."""
    from delta_crdt_ex_amd._abi import CapacityError
    a, b = W.config4_shard(2, 8, keys_per_rank=60_000, diff_frac=0.02)
    want = R.store_diff(a["rows"], b["rows"])
    d = W.sync_delta(b, want)
    st, sc = state_of(a, extra_ctx=8)
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, 12)
    snap = _snapshot(st, sc, tree)
    small = torch.empty(5, dtype=torch.int64, device=DEV)
    with pytest.raises(CapacityError):
        engine.join_delta(st, sc, sd, cd, kdev(want), spare, tree, changed=small)
    _assert_unchanged(st, sc, tree, snap)
    apply(engine, a, d, want, depth=12)  # and the engine goes on



@pytest.mark.parametrize("depth,moves", [(24, False), (24, True), (11, True)])
def test_kd_deep_and_one_chunk_trees(engine, depth, moves):
    """The one-wait path's tree re-reduction by persistent workgroups: a depth-24 tree (8192
    chunks: sixteen per workgroup) and a one-chunk tree, in place and with moved rows;
    the tree equals a fresh build (apply checks nodes, counts, keys and the chunk index)."""
    rng = np.random.default_rng(depth + moves)
    if moves:
        a, b = W.random_pair(rng, 60_000, n_nodes=5, ts_range=1 << 10)
        kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
        keys = np.sort(rng.choice(kb, 3_000, replace=False))
    else:
        a, b = W.config4_shard(1, 8, keys_per_rank=200_000, diff_frac=0.02)
        keys = R.store_diff(a["rows"], b["rows"])
    assert len(keys) > 512  # (not the small path)
    _, _, swapped, _ = apply(engine, a, W.sync_delta(b, keys), keys, depth=depth)
    assert swapped == moves


def _runs_state(rng, n, big, run):
    """n keys with one row each, key `big` with `run` rows (distinct dots of node 0)."""
    keys = np.unique(rng.integers(0, 1 << 63, n + 10, dtype=np.uint64))[:n]
    rk = np.concatenate([keys, np.full(run - 1, keys[big], np.uint64)])
    node = np.zeros(len(rk), np.uint32)
    cnt = np.arange(1, len(rk) + 1, dtype=np.uint64)
    val = np.arange(len(rk), dtype=np.uint64)
    order = np.lexsort((cnt, node, np.zeros(len(rk)), val, rk))
    rows = (rk[order], val[order], np.full(len(rk), 3, np.int64), node[order], cnt[order])
    return keys, {"rows": rows, "ctx": (R.VV, np.array([0], np.uint32), np.array([len(rk)], np.uint64))}


@pytest.mark.parametrize("run", [64, 65])
def test_kd_key_run_at_the_limit(engine, run):
    """A state key with exactly KD_RUN (64) rows stays on the per-key path; 65 rows fall
    back (the splice path); both equal the oracle and a fresh tree, the delta replacing
    every row of the key (a covering context) and adding one."""
    rng = np.random.default_rng(run)
    keys, a = _runs_state(rng, 3000, 100, run)
    big = keys[100]
    dk = np.sort(np.array([big, keys[5], keys[2000]], np.uint64))
    d = {"rows": (dk, np.array([7, 8, 9], np.uint64), np.full(3, 9, np.int64), np.full(3, 1, np.uint32),
                  np.array([1, 2, 3], np.uint64)),
         "ctx": (R.VV, np.array([0, 1], np.uint32), np.array([len(a["rows"][0]), 3], np.uint64))}
    _, _, swapped, _ = apply(engine, a, d, dk, depth=9)
    assert swapped  # (the big key's run shrinks to one row)


def test_kd_node_ids_past_the_lds_tables(engine):
    """Contexts naming node ids >= 1024 (past the count kernel's LDS VV tables): coverage
    through the searched context, on a delta of more than 512 keys."""
    rng = np.random.default_rng(31)
    n = 4000
    keys = np.unique(rng.integers(0, 1 << 63, n + 10, dtype=np.uint64))[:n]
    nodes = np.array([3, 1500, 70000], np.uint32)
    node = nodes[rng.integers(0, 3, n)]
    cnt = np.arange(1, n + 1, dtype=np.uint64)
    a = {"rows": (keys, np.arange(n, dtype=np.uint64), np.full(n, 5, np.int64), node, cnt),
         "ctx": (R.VV, nodes, np.array([n, n, n], np.uint64))}
    sel = np.sort(rng.choice(n, 900, replace=False))
    dk = keys[sel]
    dnode = np.full(len(dk), 2000, np.uint32)
    dcnt = np.arange(1, len(dk) + 1, dtype=np.uint64)
    d = {"rows": (dk, np.arange(len(dk), dtype=np.uint64) + 10 ** 6, np.full(len(dk), 9, np.int64), dnode, dcnt),
         # covers nodes 3 and 70000 up to half of the counters: those rows go, the others stay
         "ctx": (R.VV, np.array([3, 2000, 70000], np.uint32), np.array([n // 2, len(dk), n // 2], np.uint64))}
    apply(engine, a, d, dk, depth=10)


def test_kd_removal_only_keys(engine):
    """Keyset keys the delta has no rows for (a remove synced: its context covers the
    state's dots), beside keys it updates -- more than 512 keys, rows move."""
    rng = np.random.default_rng(32)
    a, b = W.random_pair(rng, 20_000, n_nodes=4, ts_range=1 << 10)
    kb = np.unique(b["rows"][0])
    upd = np.sort(rng.choice(kb, 600, replace=False))
    gone = np.setdiff1d(np.unique(a["rows"][0]), kb)[:400]  # keys B has none of
    keys = np.union1d(upd, gone)
    d = W.sync_delta(b, keys)  # (rows only for `upd`; B's context covers A's dots or not)
    apply(engine, a, d, keys, depth=11)


@pytest.mark.parametrize("moves", [False, True])
def test_kd_sharded_tree(engine, moves):
    """A shard tree (shard_bits 3) over one key-hash shard, through the per-key path with
    and without moved rows: the tree (and its chunk index) equals a fresh shard build."""
    from delta_crdt_ex_amd.store import MerkleTree
    rng = np.random.default_rng(33 + moves)
    if moves:
        a, b = W.random_pair(rng, 80_000, n_nodes=5, ts_range=1 << 10)
    else:
        a, b = W.config4_shard(0, 1, keys_per_rank=400_000, diff_frac=0.02)
    sh = lambda k: (np.asarray(k, np.uint64) >> np.uint64(61)) == 2  # noqa: E731  (shard 2 of 8)
    cut = lambda rep: {**rep, "rows": tuple(c[sh(rep["rows"][0])] for c in rep["rows"])}  # noqa: E731
    a, b = cut(a), cut(b)
    kb = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    keys = np.sort(rng.choice(kb, min(2000, len(kb)), replace=False)) if moves else R.store_diff(a["rows"], b["rows"])
    assert len(keys) > 512
    d = W.sync_delta(b, keys)
    st, sc = state_of(a, extra_ctx=len(d["ctx"][1]))
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, 14, MerkleTree.empty(14, DEV, 3, 2), 3, 2)
    changed, swapped = engine.join_delta(st, sc, sd, cd, kdev(keys), spare, tree)
    wr, wc = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=keys)
    rows_eq(st, wr)
    ctx_eq(sc, wc)
    assert np.array_equal(u64(changed), R.changed_keys(a["rows"], wr, keys))
    fresh = engine.merkle_build(st, 14, MerkleTree.empty(14, DEV, 3, 2), 3, 2)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())
    assert np.array_equal(tree.starts.cpu().numpy(), fresh.starts.cpu().numpy())
    assert swapped == moves
