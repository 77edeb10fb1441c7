"""The MerkleMap role on the GPU (csrc/merkle.hip) against the C oracle
(oracle/deltaref.c ref_merkle_build, oracle/ref.py): build, incremental
put/delete + update_hashes from a join's changed keys (causal_crdt.ex:383-394),
the truncating diff (max_sync_size, :98,105,206-214), the partial-diff ping-pong
(prepare_partial_diff / continue_partial_diff / truncate_diff, :91-110,252-289) and
key-hash shard trees that fold to the unsharded root.  The hash itself
is "parity unpinned" (merkle_map 0.2.0 is not vendored); the GPU tree is bit-exact
against the C restatement of the same hash, and the differing keys are exactly the
keys whose raw value maps differ."""
import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd._abi import DeltaGpuError
from delta_crdt_ex_amd.sharding import shard_of
from delta_crdt_ex_amd.store import Context, Store, fold_roots, u64
from oracle import ref as R

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def up(rep):
    rows, ctx = rep["rows"], rep["ctx"]
    return Store.from_numpy(*rows, device=DEV), Context.from_numpy(ctx[0], ctx[1], ctx[2], DEV)


def nodes(t):
    return t.nodes.cpu().numpy().view(np.uint64)


def keys_dev(k):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(k, np.uint64)).view(np.int64)).to(DEV)


@pytest.mark.parametrize("depth", [1, 5, 8, 11, 12, 16, 20])
def test_build_and_diff(engine, depth):
    a, b = W.merkle_pair(n_keys=20000, diff_frac=0.01, seed=depth)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    ra, rb = R.merkle_build(a["rows"], depth), R.merkle_build(b["rows"], depth)
    for t, r in ((ta, ra), (tb, rb)):
        assert t.n_keys == r.n_keys
        assert np.array_equal(nodes(t), r.nodes)
        assert np.array_equal(t.bucket_counts(), r.counts)
    d = engine.merkle_diff(ta, tb)
    assert np.array_equal(u64(d), R.store_diff(a["rows"], b["rows"]))
    assert engine.merkle_diff(ta, ta).numel() == 0


def test_build_edges(engine):
    # empty store, one row, every row in one bucket, rows at both ends of the key space
    for rows in (tuple(np.zeros(0, dt) for dt in (np.uint64, np.uint64, np.int64, np.uint32, np.uint64)),
                 (np.array([5], np.uint64), np.array([1], np.uint64), np.array([-3], np.int64),
                  np.array([2], np.uint32), np.array([9], np.uint64))):
        s = Store.from_numpy(*rows, device=DEV)
        s.n = len(rows[0])
        for depth in (1, 9):
            t = engine.merkle_build(s, depth)
            assert np.array_equal(nodes(t), R.merkle_build(rows, depth).nodes)
    k = np.array([0, 1, 2, 3, (1 << 64) - 2, (1 << 64) - 1], np.uint64)
    rows = (k, k, k.view(np.int64), (k & np.uint64(7)).astype(np.uint32), k)
    s = Store.from_numpy(*rows, device=DEV)
    for depth in (1, 4, 20):
        assert np.array_equal(nodes(engine.merkle_build(s, depth)), R.merkle_build(rows, depth).nodes)
    # runs of one bucket across many 64-row chunks (the atomic-add path)
    a, _ = W.merkle_pair(n_keys=50000, seed=9)
    sa, _ = up(a)
    for depth in (2, 6):
        assert np.array_equal(nodes(engine.merkle_build(sa, depth)), R.merkle_build(a["rows"], depth).nodes)


@pytest.mark.parametrize("seed", range(4))
def test_update_after_join_equals_fresh_build(engine, seed):
    """put/delete + update_hashes of dg_join2_changes's changed keys == dg_merkle_build
    of the joined store, bit for bit."""
    rng = np.random.default_rng(seed)
    a, b = W.random_pair(rng, n_keys=3000, ts_range=8, dense_ctx=bool(seed % 2))
    keys = None
    if seed >= 2:  # a keyed sync delta: {VV, Map.take(value, keys)}, keys (causal_crdt.ex:324-335)
        ks = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
        sel = ks[rng.random(len(ks)) < 0.5]
        b = W.sync_delta(b, sel)
        keys = keys_dev(sel)
    sa, ca = up(a)
    sb, cb = up(b)
    for depth in (6, 12):
        t = engine.merkle_build(sa, depth)
        out, octx, changed = engine.join2_changes(sa, ca, sb, cb, keys=keys)
        engine.merkle_update(t, out, changed)
        fresh = engine.merkle_build(out, depth)
        assert np.array_equal(nodes(t), nodes(fresh))
        assert np.array_equal(t.bucket_counts(), fresh.bucket_counts())
        assert t.n_keys == fresh.n_keys
        assert t.store is out


def test_update_config2_scale(engine):
    a, b = W.config2(n_keys=400_000, seed=11)
    sa, ca = up(a)
    sb, cb = up(b)
    t = engine.merkle_build(sa, 17)
    out, octx, changed = engine.join2_changes(sa, ca, sb, cb)
    engine.merkle_update(t, out, changed)
    fresh = engine.merkle_build(out, 17)
    assert np.array_equal(nodes(t), nodes(fresh))
    assert np.array_equal(t.bucket_counts(), fresh.bucket_counts())
    # no change: an update with no keys leaves the tree as it is
    before = nodes(t).copy()
    engine.merkle_update(t, out, keys_dev(np.zeros(0, np.uint64)))
    assert np.array_equal(before, nodes(t))


@pytest.mark.parametrize("cap", [0, 1, 5, 100, 10**6])
def test_truncated_diff_is_the_prefix(engine, cap):
    a, b = W.merkle_pair(n_keys=30000, diff_frac=0.05, seed=3)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, 12), engine.merkle_build(sb, 12)
    full = R.store_diff(a["rows"], b["rows"])
    got, total = engine.merkle_diff(ta, tb, cap=cap, with_total=True)
    assert total == len(full)
    assert np.array_equal(u64(got), full[:cap])


@pytest.mark.parametrize("n_keys,depth", [(800, 12), (900, 12), (3000, 14)])
def test_more_differing_buckets_than_lanes(engine, n_keys, depth):
    """A subtree whose differing buckets (about 300-450) outnumber the count kernel's
    lanes while their rows still fit the LDS stage: each lane merges several buckets, and
    the keys must still come out in key order."""
    a, b = W.merkle_pair(n_keys=n_keys, diff_frac=0.5, seed=9)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    assert np.array_equal(u64(engine.merkle_diff(ta, tb)), R.store_diff(a["rows"], b["rows"]))


def test_async_diff_equals_the_synchronous_one(engine):
    """dg_merkle_diff_async: back-to-back launches into one output, the total on the
    device, several caps and depths (small subtrees included), and after an asynchronous
    join that is still pending (the call settles it first)."""
    a, b = W.merkle_pair(n_keys=30000, diff_frac=0.05, seed=4)
    sa, ca = up(a)
    sb, cb = up(b)
    full = R.store_diff(a["rows"], b["rows"])
    for depth, cap in ((3, 10**6), (12, 7), (14, 10**6), (14, 0)):
        ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
        out = torch.zeros(max(cap, 1), dtype=torch.int64, device=DEV)
        d_total = torch.zeros(1, dtype=torch.int64, device=DEV)
        launch = engine.prepare_merkle_diff(ta, tb, out, cap, d_total)
        for _ in range(3):
            launch()
        engine.sync()
        n = min(len(full), cap)
        assert int(d_total[0]) == len(full)
        assert np.array_equal(u64(out[:n]), full[:n])
    # a pending asynchronous join whose output the diff reads
    j = Store.empty(sa.n + sb.n, DEV)
    jc = Context.empty(0, ca.n + cb.n, DEV)
    d_counts = torch.zeros(8, dtype=torch.int64, device=DEV)
    engine.join2_async(sa, ca, sb, cb, j, jc, d_counts=d_counts)
    engine.sync()
    j.n = int(d_counts[0])
    tj, tb = engine.merkle_build(j, 12), engine.merkle_build(sb, 12)
    wj, _ = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    out = torch.zeros(len(full) + 1, dtype=torch.int64, device=DEV)
    d_total = torch.zeros(1, dtype=torch.int64, device=DEV)
    engine.join2_async(sa, ca, sb, cb, j, jc, d_counts=d_counts)  # pending
    engine.prepare_merkle_diff(tj, tb, out, len(full) + 1, d_total)()
    engine.sync()
    want = R.store_diff(wj, b["rows"])
    assert int(d_total[0]) == len(want)
    assert np.array_equal(u64(out[: len(want)]), want)


def test_diffs_of_different_depths_in_sequence(engine):
    """The diff's per-group key sums live in two engine buffers that alternate by call; a
    shallow diff between two deep ones must not leave the deep one's second group stale
    (depth 21: 512 subtrees in 2 groups; depth 12: one)."""
    a, b = W.merkle_pair(n_keys=200_000, diff_frac=0.01, seed=21)
    sa, _ = up(a)
    sb, _ = up(b)
    full = R.store_diff(a["rows"], b["rows"])
    deep = (engine.merkle_build(sa, 21), engine.merkle_build(sb, 21))
    shallow = (engine.merkle_build(sa, 12), engine.merkle_build(sb, 12))
    for trees in (deep, shallow, deep, deep, shallow, deep):
        got, total = engine.merkle_diff(*trees, with_total=True)
        assert total == len(full) and np.array_equal(u64(got), full)


@pytest.mark.parametrize("levels,depth", [(8, 18), (3, 10), (1, 4), (8, 8)])
def test_partial_diff_ping_pong(engine, levels, depth):
    """A.prepare -> B.continue -> A.continue -> ... ends with the differing keys, hop
    for hop equal to the oracle's continuations."""
    a, b = W.merkle_pair(n_keys=40000, diff_frac=0.005, seed=levels)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    ra, rb = R.merkle_build(a["rows"], depth), R.merkle_build(b["rows"], depth)
    cont = engine.merkle_prepare(ta, levels)
    rc = R.merkle_prepare(ra, levels)
    side = [(tb, rb, b["rows"]), (ta, ra, a["rows"])]
    hops = 0
    while True:
        t, r, rows = side[hops % 2]
        res = engine.merkle_continue(t, cont, levels)
        rres = R.merkle_continue(r, rows, rc, levels)
        hops += 1
        assert res[0] == rres[0]
        if res[0] == "ok":
            break
        cont, rc = res[1], rres[1]
        if rc[0] == "node":
            assert cont.level == rc[1] and not cont.leaf
            assert np.array_equal(u64(cont.pos[: cont.n]), rc[2])
            assert np.array_equal(u64(cont.hash[: cont.n]), rc[3])
        else:
            assert cont.level == depth + 1
            assert np.array_equal(u64(cont.bucket[: cont.n_buckets]), rc[1])
            assert np.array_equal(u64(cont.pos[: cont.n]), rc[2])
            assert np.array_equal(u64(cont.hash[: cont.n]), rc[3])
    full = R.store_diff(a["rows"], b["rows"])
    assert np.array_equal(u64(res[1]), full) and res[2] == len(full)
    assert np.array_equal(rres[1], full)


@pytest.mark.parametrize("levels,depth,max_sync", [(8, 18, 200), (3, 10, 7), (1, 4, None), (8, 8, 200),
                                                    (8, 14, None), (4, 12, 1)])
def test_continue_home_matches_the_general_hop(engine, levels, depth, max_sync):
    """dg_merkle_continue_home (one launch, one host wait) against dg_merkle_continue +
    dg_merkle_truncate on the same continuation, hop for hop on both sides: node form,
    node -> leaf form, leaf form -> keys; the general calls where it declines."""
    a, b = W.merkle_pair(n_keys=40000, diff_frac=0.005, seed=levels + depth)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    cont = engine.merkle_prepare(ta, levels)
    side = [tb, ta]
    hops = homed = 0
    while True:
        t = side[hops % 2]
        want = engine.merkle_continue(t, cont, levels)
        if want[0] == "continue" and max_sync is not None:
            engine.merkle_truncate(t, want[1], max_sync)
        got = engine.merkle_continue_home(t, cont, levels, max_sync)
        hops += 1
        if got[0] == "declined":
            assert cont.n > 4096 or cont.n_buckets > 512
            got = want
        else:
            homed += 1
        assert got[0] == want[0]
        if got[0] == "ok":
            assert got[2] == want[2] and np.array_equal(u64(got[1]), u64(want[1]))
            break
        g, w = got[1], want[1]
        assert (g.level, g.n, g.n_buckets) == (w.level, w.n, w.n_buckets)
        assert np.array_equal(u64(g.pos[: g.n]), u64(w.pos[: w.n]))
        assert np.array_equal(u64(g.hash[: g.n]), u64(w.hash[: w.n]))
        assert np.array_equal(u64(g.bucket[: g.n_buckets]), u64(w.bucket[: w.n_buckets]))
        cont = w
    assert homed >= 1  # (depth 8: the leaf-form hop carries ~31k pairs, over the limit)


def test_continue_home_rejects_positions_outside_the_tree(engine):
    a, _ = W.merkle_pair(n_keys=2000, diff_frac=0.01, seed=3)
    t = engine.merkle_build(up(a)[0], 10)
    cont = engine.merkle_prepare(t, 4)
    cont.pos[3] = 1 << 4  # level 4 holds positions 0..15
    with pytest.raises(DeltaGpuError, match="outside the tree"):
        engine.merkle_continue_home(t, cont, 4, 200)
    # the engine is usable afterwards
    cont = engine.merkle_prepare(t, 4)
    res = engine.merkle_continue_home(t, cont, 4, 200)  # (its own tree: nothing differs)
    assert res[0] == "ok" and res[2] == 0


def test_partial_diff_equal_trees_and_truncation(engine):
    a, b = W.merkle_pair(n_keys=20000, diff_frac=0.02, seed=5)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, 10), engine.merkle_build(sb, 10)
    # identical trees: {:ok, []} on the first hop
    res = engine.merkle_continue(engine.merkle_build(sa, 10), engine.merkle_prepare(ta, 8), 8)
    assert res[0] == "ok" and res[1].numel() == 0
    # truncate_diff of a node-form continuation keeps its first entries
    c = engine.merkle_continue(tb, engine.merkle_prepare(ta, 4), 4)[1]
    n0 = c.n
    engine.merkle_truncate(tb, c, 3)
    assert c.n == min(3, n0)
    # leaf form: only the pairs of the first buckets are kept, and the keys that come
    # out are the differing keys of those buckets
    c = engine.merkle_continue(tb, engine.merkle_prepare(ta, 10), 10)[1]
    assert c.leaf
    bk = u64(c.bucket[: c.n_buckets])
    engine.merkle_truncate(tb, c, 4)
    assert c.n_buckets == 4
    res = engine.merkle_continue(ta, c, 10)
    full = R.store_diff(a["rows"], b["rows"])
    want = full[np.isin(R.Tree(10).bucket_of(full), bk[:4].astype(np.int64))]
    assert res[0] == "ok" and np.array_equal(u64(res[1]), want)


@pytest.mark.parametrize("bits", [1, 3])
def test_shard_trees_fold_to_the_unsharded_root(engine, bits):
    a, _ = W.merkle_pair(n_keys=60000, seed=bits)
    depth = 14
    whole = engine.merkle_build(up(a)[0], depth)
    roots = []
    for s in range(1 << bits):
        m = shard_of(a["rows"][0], 1 << bits) == s
        rows = tuple(c[m] for c in a["rows"])
        t = engine.merkle_build(Store.from_numpy(*rows, device=DEV), depth - bits, shard_bits=bits,
                                shard=s)
        assert np.array_equal(nodes(t), R.merkle_build(rows, depth - bits, bits, s).nodes)
        roots.append(t.root())
    assert fold_roots(roots) == whole.root()
    with pytest.raises(DeltaGpuError):  # rows outside the tree's shard
        engine.merkle_build(up(a)[0], depth - bits, shard_bits=bits, shard=0)


@pytest.mark.parametrize("depth,n_keys", [(12, 60000), (14, 60000), (3, 2000)])
def test_dense_diff(engine, depth, n_keys):
    """Every key differs: a subtree's differing rows overflow the LDS stage and its
    buckets merge over global memory (and depth 3: subtrees of fewer than 16 buckets)."""
    a, b = W.merkle_pair(n_keys=n_keys, diff_frac=1.0, seed=depth)
    sa, _ = up(a)
    sb, _ = up(b)
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    full = R.store_diff(a["rows"], b["rows"])
    assert len(full) == n_keys
    got, total = engine.merkle_diff(ta, tb, cap=len(full) // 3, with_total=True)
    assert total == len(full) and np.array_equal(u64(got), full[: len(full) // 3])
    # one replica empty: every key of the other
    e = Store.empty(1, DEV)
    te = engine.merkle_build(e, depth)
    assert np.array_equal(u64(engine.merkle_diff(ta, te)), np.unique(a["rows"][0]))


@pytest.mark.parametrize("n_keys,depth", [(300, 8), (1500, 9), (1, 4)])
def test_diff_against_an_empty_store_in_lds(engine, n_keys, depth):
    """One store empty, few enough rows that the subtree's rows are staged in LDS: every
    staged row comes from the other store, and the lanes past the staged rows load a row
    of the non-empty store (both orders)."""
    a, _ = W.merkle_pair(n_keys=n_keys, diff_frac=0.0, seed=n_keys)
    sa, _ = up(a)
    e = Store.empty(1, DEV)
    ta, te = engine.merkle_build(sa, depth), engine.merkle_build(e, depth)
    want = np.unique(a["rows"][0])
    assert np.array_equal(u64(engine.merkle_diff(ta, te)), want)
    assert np.array_equal(u64(engine.merkle_diff(te, ta)), want)
    assert u64(engine.merkle_diff(te, te)).size == 0


def test_bucket_over_65535_rows_is_refused(engine):
    k = np.zeros(70000, np.uint64)  # one key, 70,000 entries: one bucket
    rows = (k, np.arange(70000, dtype=np.uint64), np.zeros(70000, np.int64),
            np.zeros(70000, np.uint32), np.arange(1, 70001, dtype=np.uint64))
    from delta_crdt_ex_amd._abi import CapacityError
    with pytest.raises(CapacityError):
        engine.merkle_build(Store.from_numpy(*rows, device=DEV), 4)


def test_config4_shard_full_size(engine):
    """BASELINE config 4 at the bench's per-GPU shard: 12.5M keys (a key-hash eighth of
    100M), depth 22, the replicas differing on 1 % of the keys.  Diff == the exact
    row-set diff; the sync delta Map.take(B.value, keys) joined into A over those keys
    == the C oracle's join; the Merkle update of the changed keys == a fresh build."""
    a, b = W.config4_shard(0, 8, keys_per_rank=12_500_000, diff_frac=0.01)
    sa, ca = up(a)
    sb, cb = up(b)
    depth = 22
    ta = engine.merkle_build(sa, depth, shard_bits=3, shard=0)
    tb = engine.merkle_build(sb, depth, shard_bits=3, shard=0)
    ra = R.merkle_build(a["rows"], depth, 3, 0)
    assert np.array_equal(nodes(ta), ra.nodes) and np.array_equal(ta.bucket_counts(), ra.counts)
    want = R.store_diff(a["rows"], b["rows"])
    keys, total = engine.merkle_diff(ta, tb, with_total=True)
    assert total == len(want) and np.array_equal(u64(keys), want)
    delta = engine.take_keys(sb, keys)
    out, octx, changed = engine.join2_changes(sa, ca, delta, cb, keys=keys)
    wrows, wctx = R.join2(a["rows"], a["ctx"], tuple(c for c in delta.to_numpy()), b["ctx"], keys=want)
    for x, y in zip(out.to_numpy(), wrows):
        assert np.array_equal(x, y)
    engine.merkle_update(ta, out, changed)
    fresh = engine.merkle_build(out, depth, shard_bits=3, shard=0)
    assert np.array_equal(nodes(ta), nodes(fresh))
    assert np.array_equal(ta.bucket_counts(), fresh.bucket_counts())


@pytest.mark.parametrize("home", [False, True])
@pytest.mark.parametrize("max_sync_size", [200, None])
def test_partial_diff_config4_shard(engine, max_sync_size, home):
    """The partial-diff protocol at the scale and shape CausalCrdt runs it:
    a config-4 shard (12.5M keys, 1 % differing, depth 22), prepare_partial_diff(mm, 8) on
    the originator (causal_crdt.ex:255), then continue_partial_diff(cont, mm, 8) ping-pong
    between the replicas (:96), each {:continue, c} truncated to max_sync_size before it
    is sent (:98, default 200: delta_crdt.ex:32; None: :infinite), and the final keys
    truncated too (:105).  Every hop's continuation equals the C oracle's, hashes and
    all; the keys are the first differing keys of the buckets the truncations kept.
    home: each hop through dg_merkle_continue_home (continue + truncate, one launch, one
    wait), the general calls where it declines (a continuation over its limits)."""
    a, b = W.config4_shard(3, 8, keys_per_rank=12_500_000, diff_frac=0.01)
    sa, _ = up(a)
    sb, _ = up(b)
    depth, levels = 22, 8
    ta = engine.merkle_build(sa, depth, shard_bits=3, shard=3)
    tb = engine.merkle_build(sb, depth, shard_bits=3, shard=3)
    ra = R.merkle_build(a["rows"], depth, 3, 3)
    rb = R.merkle_build(b["rows"], depth, 3, 3)
    cont, rc = engine.merkle_prepare(ta, levels), R.merkle_prepare(ra, levels)
    assert cont.n == rc[2].size == 256
    side = [(tb, rb, b["rows"]), (ta, ra, a["rows"])]
    hops, sizes = 0, []
    homed = 0
    while True:
        t, r, rows = side[hops % 2]
        res = engine.merkle_continue_home(t, cont, levels, max_sync_size) if home else ("declined",)
        truncated = res[0] != "declined"
        homed += truncated
        if not truncated:
            res = engine.merkle_continue(t, cont, levels)
        rres = R.merkle_continue(r, rows, rc, levels)
        hops += 1
        assert res[0] == rres[0]
        if res[0] == "ok":
            break
        cont, rc = res[1], rres[1]
        if max_sync_size is not None:
            if not truncated:
                engine.merkle_truncate(t, cont, max_sync_size)
            rc = R.merkle_truncate(r, rc, max_sync_size)
        sizes.append((cont.n, cont.n_buckets))
        if rc[0] == "node":
            assert cont.level == rc[1] and not cont.leaf
        else:
            assert cont.level == depth + 1
            assert np.array_equal(u64(cont.bucket[: cont.n_buckets]), rc[1])
        assert np.array_equal(u64(cont.pos[: cont.n]), rc[2])
        assert np.array_equal(u64(cont.hash[: cont.n]), rc[3])
    assert hops == 4  # level 8 -> 16 -> 22 -> leaf form -> keys
    if home:  # (infinite: the first hop only -- 65,536 entries come back, over the limit)
        assert homed == (4 if max_sync_size is not None else 1)
    keys = u64(res[1])
    assert np.array_equal(keys, rres[1])
    full = R.store_diff(a["rows"], b["rows"])
    if max_sync_size is None:
        assert np.array_equal(keys, full)
        assert sizes[0][0] == 256 * 256  # every level-8 subtree differs at 1 %
    else:
        # the keys of the kept buckets: a subset of the diff, every one of them differing
        assert all(n <= max_sync_size for n, nb in sizes[:2])
        assert sizes[2][1] <= max_sync_size
        assert 0 < len(keys) and np.all(np.isin(keys, full))
        want = full[np.isin(R.Tree(depth, 3, 3).bucket_of(full),
                            u64(cont.bucket[: cont.n_buckets]).astype(np.int64))]
        assert np.array_equal(keys, want)
        assert len(keys[:max_sync_size]) <= max_sync_size  # send_diff's truncate (:105)


def test_chunk_index_follows_the_rows(engine):
    """dg_merkle.starts (each 2^11-bucket chunk's first row): the build's equals the host's
    search of the store; an update that changes rows per key (adds, removes) moves it
    exactly as a fresh build would; and a diff reads the same keys with the index as
    without it (starts = NULL: the key-column search)."""
    rng = np.random.default_rng(17)
    a, b = W.random_pair(rng, 60_000, n_nodes=4, max_entries=3)
    sa, ca = up(a)
    sb, cb = up(b)
    depth = 14
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    keys = a["rows"][0]
    chunk_first = (np.arange(1 << (depth - 11), dtype=np.uint64) << np.uint64(64 - depth + 11))
    want = np.r_[np.searchsorted(keys, chunk_first), len(keys)].astype(np.uint64)
    assert np.array_equal(u64(ta.starts), want)
    out, octx, changed = engine.join2_changes(sa, ca, sb, cb)
    assert out.n != sa.n  # rows moved
    engine.merkle_update(ta, out, changed)
    fresh = engine.merkle_build(out, depth)
    assert np.array_equal(u64(ta.starts), u64(fresh.starts))
    assert np.array_equal(nodes(ta), nodes(fresh))
    ta2, tb2 = engine.merkle_build(out, depth), engine.merkle_build(sb, depth)
    with_index = u64(engine.merkle_diff(ta2, tb2))
    ta2.starts = tb2.starts = None
    assert np.array_equal(u64(engine.merkle_diff(ta2, tb2)), with_index)
    assert np.array_equal(with_index, R.store_diff(out.to_numpy(), b["rows"]))


def test_diff_against_a_store_the_index_does_not_describe(engine):
    """a tree's chunk index describes the store it was built / updated against.
    Handed another store -- here one whose row count changed without dg_merkle_update --
    the diff must not trust it (it would read past the store or return wrong keys): it
    searches the store instead, exactly as a tree without an index does.  Where the tree
    counts more rows than the store holds, nothing is read past the store and the diff is
    an input error (DG_DIFF_MISMATCH), with or without the index."""
    rng = np.random.default_rng(23)
    a, b = W.random_pair(rng, 50_000, n_nodes=4, max_entries=3)
    sa, ca = up(a)
    sb, cb = up(b)
    depth = 14
    ta, tb = engine.merkle_build(sa, depth), engine.merkle_build(sb, depth)
    for cut in (a["rows"][0].size // 2, 10):  # fewer rows than the index says
        short = Store.from_numpy(*(c[:cut] for c in a["rows"]), device=DEV)
        ta.store = short
        with pytest.raises(DeltaGpuError, match="more rows than its store"):
            engine.merkle_diff(ta, tb)
        ta.starts, kept = None, ta.starts
        with pytest.raises(DeltaGpuError, match="more rows than its store"):
            engine.merkle_diff(ta, tb)
        ta.starts = kept
    # the engine is usable after the error: the matching pair diffs as the oracle says
    ta.store = sa
    assert np.array_equal(u64(engine.merkle_diff(ta, tb)), R.store_diff(a["rows"], b["rows"]))
    # a join's output under a tree of the old state (here it holds fewer rows: the join drops
    # the dots the other context covers); with and without the index the diff agrees
    out, _ = engine.join2(sa, ca, sb, cb)
    assert out.n != sa.n
    ta.store = out

    def outcome():  # the keys, or the input error where a subtree overruns the store
        try:
            return u64(engine.merkle_diff(ta, tb)).tolist()
        except DeltaGpuError as ex:
            assert "more rows than its store" in str(ex)
            return "mismatch"

    got = outcome()
    ta.starts, kept = None, ta.starts
    assert got == outcome()
    ta.starts, ta.store = kept, sa
    assert np.array_equal(u64(engine.merkle_diff(ta, tb)), R.store_diff(a["rows"], b["rows"]))


@pytest.mark.parametrize("rows_per_key", [1, 9])
def test_take_keys_output_sizing(engine, rows_per_key):
    """Map.take(value, keys): the Python binding sizes the output for four rows per key and
    runs again into a store-sized output when the keys hold more (DG_E_CAPACITY inside)."""
    rng = np.random.default_rng(rows_per_key)
    kk = np.unique(rng.integers(0, 1 << 63, 400, dtype=np.uint64))
    key = np.repeat(kk, rows_per_key)
    n = len(key)
    rows = (key, np.arange(n, dtype=np.uint64), np.zeros(n, np.int64), np.zeros(n, np.uint32),
            np.arange(1, n + 1, dtype=np.uint64))
    s = Store.from_numpy(*rows, device=DEV)
    want_keys = np.sort(rng.choice(kk, 100, replace=False))
    got = engine.take_keys(s, torch.from_numpy(want_keys.view(np.int64)).to(DEV))
    sel = np.isin(key, want_keys)
    assert got.n == int(sel.sum())
    for c_got, c_all in zip(got.to_numpy(), rows):
        assert np.array_equal(c_got, c_all[sel])
