"""GPU parity: libdeltagpu (through its C-ABI, on cuda:0) against the C oracle and
the golden fixtures.  Integer work => bit-exact equality everywhere."""
import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd._abi import CapacityError, FunctionClauseError
from delta_crdt_ex_amd.store import Context, Store, u64
from oracle import ref as R

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def up(rep):
    rows, ctx = rep["rows"], rep["ctx"]
    return Store.from_numpy(*rows, device=DEV), Context.from_numpy(ctx[0], ctx[1], ctx[2], DEV)


def rows_eq(got: Store, want):
    g = got.to_numpy()
    assert got.n == len(want[0]), (got.n, len(want[0]))
    for i, (x, y) in enumerate(zip(g, want)):
        assert np.array_equal(x, y), f"column {i} differs"


def ctx_eq(got: Context, want):
    assert got.kind == want[0]
    node, cnt = got.to_numpy()
    assert np.array_equal(node, want[1]) and np.array_equal(cnt, want[2])


def check_join(engine, a, b, keys=None):
    sa, ca = up(a)
    sb, cb = up(b)
    kt = None
    if keys is not None:
        ku = np.unique(np.asarray(keys, np.uint64))
        kt = torch.from_numpy(ku.view(np.int64)).to(DEV)
    out, octx = engine.join2(sa, ca, sb, cb, keys=kt)
    wrows, wctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"], keys=keys)
    rows_eq(out, wrows)
    ctx_eq(octx, wctx)
    return out, octx


CASES = [
    dict(n_keys=40, ts_range=1 << 40, dense_ctx=True, ctx_kind=W.VV),
    dict(n_keys=40, ts_range=2, dense_ctx=True, ctx_kind=W.VV),
    dict(n_keys=40, ts_range=1 << 40, dense_ctx=False, ctx_kind=W.VV),
    dict(n_keys=30, ts_range=4, dense_ctx=False, ctx_kind=W.DOTS),
    dict(n_keys=30, ts_range=4, dense_ctx=True, ctx_kind=W.DOTS),
    dict(n_keys=0, ts_range=4, dense_ctx=True, ctx_kind=W.VV),
    dict(n_keys=3000, ts_range=1 << 20, dense_ctx=False, ctx_kind=W.VV),   # multi-tile
    dict(n_keys=2000, ts_range=3, dense_ctx=False, ctx_kind=W.DOTS),       # multi-tile, ties
]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("seed", range(4))
def test_join2_random(engine, case, seed):
    rng = np.random.default_rng(1000 * case + seed)
    a, b = W.random_pair(rng, **CASES[case])
    check_join(engine, a, b)
    check_join(engine, b, a)
    keys = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    if len(keys):
        check_join(engine, a, b, keys=keys[::2])
        check_join(engine, a, b, keys=np.concatenate([keys[1::3], np.array([12345], np.uint64)]))


@pytest.mark.parametrize("n_keys", [200_000, 3_000_000])  # fused splits / partition launch
def test_join2_keyed_slices(engine, n_keys):
    """Keyed joins through the per-tile keyset slices: sparse keysets (a few keys per
    tile: the slice staged in LDS), a clustered run of keys (tiles whose slice is longer
    than the LDS slice: global search) next to tiles with no key at all, keys absent
    from both stores, and every key."""
    a, b = W.config2(n_keys=n_keys, seed=21)
    keys = np.unique(np.concatenate([a["rows"][0], b["rows"][0]]))
    rng = np.random.default_rng(n_keys)
    sparse = np.concatenate([rng.choice(keys, len(keys) // 100, replace=False),
                             rng.integers(0, 2**63, 50, dtype=np.uint64)])
    lo = len(keys) // 3
    clustered = np.concatenate([keys[lo:lo + 5000], keys[::997]])
    for ks in (sparse, clustered, keys, np.zeros(0, np.uint64)):
        check_join(engine, a, b, keys=ks)


def test_join2_identical_and_subset(engine):
    """Every row duplicated across the stores: dedup at every tile seam."""
    a, b = W.config2(n_keys=20000, seed=9)
    check_join(engine, a, a)
    # b's store as a subset of a's, contexts equal
    sub = {"rows": tuple(c[::3] for c in a["rows"]), "ctx": a["ctx"]}
    check_join(engine, a, sub)
    check_join(engine, sub, a)


def test_join2_empty_sides(engine):
    a, b = W.config2(n_keys=5000, seed=3)
    empty = {"rows": R.empty_rows(0), "ctx": W.vv({})}
    check_join(engine, a, empty)
    check_join(engine, empty, b)
    check_join(engine, empty, empty)


def test_join2_config2_full_size(engine):
    """BASELINE config 2 at its full size (1M keys, 2M rows in)."""
    a, b = W.config2()
    out, octx = check_join(engine, a, b)
    assert 1_050_000 < out.n < 1_150_000
    engine.store_check(out)


def test_join2_properties_full_size(engine):
    """Size-independent CRDT laws at config-2 size: commutativity, idempotence."""
    a, b = W.config2(seed=11)
    sa, ca = up(a)
    sb, cb = up(b)
    ab, cab = engine.join2(sa, ca, sb, cb)
    ba, cba = engine.join2(sb, cb, sa, ca)
    for x, y in zip(ab.to_numpy(), ba.to_numpy()):
        assert np.array_equal(x, y)
    aa, caa = engine.join2(ab, cab, ab, cab)
    for x, y in zip(aa.to_numpy(), ab.to_numpy()):
        assert np.array_equal(x, y)


def test_join2_capacity_error(engine):
    a, b = W.config2(n_keys=1000, seed=1)
    sa, ca = up(a)
    sb, cb = up(b)
    small = Store.empty(10, DEV)
    with pytest.raises(CapacityError):
        engine.join2(sa, ca, sb, cb, out=small)


def test_join2_async_counts(engine):
    a, b = W.config2(n_keys=50000, seed=4)
    sa, ca = up(a)
    sb, cb = up(b)
    out = Store.empty(sa.n + sb.n, DEV)
    octx = Context.empty(0, ca.n + cb.n, DEV)
    d = torch.zeros(8, dtype=torch.int64, device=DEV)
    for _ in range(3):
        engine.join2_async(sa, ca, sb, cb, out, octx, d_counts=d)
    engine.sync()
    out.n, octx.n = int(d[0]), int(d[1])
    wrows, wctx = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wrows)
    ctx_eq(octx, wctx)


@pytest.mark.parametrize("seed", range(6))
def test_read_lww(engine, seed):
    rng = np.random.default_rng(seed)
    a, _ = W.random_pair(rng, n_keys=3000 if seed % 2 else 50, ts_range=3)
    s, _c = up(a)
    ok, ov = engine.read_lww(s)
    wk, wv = R.read_lww(a["rows"])
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)
    sub = wk[::3]
    kt = torch.from_numpy(np.ascontiguousarray(sub).view(np.int64)).to(DEV)
    ok, ov = engine.read_lww(s, keys=kt)
    wk, wv = R.read_lww(a["rows"], keys=sub)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)


def runs_store(rng, lens, ts_range):
    """A sorted, unique store whose key i has lens[i] rows (values ascending, ts drawn
    from a small range so LWW ties are common)."""
    n = int(lens.sum())
    keys = np.sort(rng.choice(2**62, len(lens), replace=False).astype(np.uint64))
    key = np.repeat(keys, lens)
    val = rng.integers(0, 1 << 20, n, dtype=np.uint64)
    ts = rng.integers(-ts_range, ts_range, n).astype(np.int64)
    node = rng.integers(0, 64, n).astype(np.uint32)
    cnt = np.arange(1, n + 1, dtype=np.uint64)
    o = np.lexsort((cnt, node, ts, val, key))
    return tuple(c[o] for c in (key, val, ts, node, cnt))


@pytest.mark.parametrize("shape", ["short", "up_to_32", "long", "giant", "tile_seams"])
def test_read_lww_run_lengths(engine, shape):
    """read/1 over key runs of every length: the segmented reduction carries a run across
    lanes, waves and tiles (1024 rows), with ts ties broken toward the earlier row."""
    rng = np.random.default_rng(len(shape))
    if shape == "short":
        lens = rng.integers(1, 4, 30000)
    elif shape == "up_to_32":
        lens = rng.integers(1, 33, 20000)
    elif shape == "long":
        lens = rng.integers(1, 3000, 300)
    elif shape == "giant":
        lens = np.array([3, 70000, 1, 5000, 2], np.int64)
    else:  # runs ending exactly at, and one row past, tile seams
        lens = np.array([1024, 1023, 2, 1024, 1025, 63, 65, 64, 1, 2048], np.int64)
    rows = runs_store(rng, lens.astype(np.int64), ts_range=3)
    s = Store.from_numpy(*rows, device=DEV)
    ok, ov = engine.read_lww(s)
    wk, wv = R.read_lww(rows)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)
    sub = wk[1::2]
    kt = torch.from_numpy(np.ascontiguousarray(sub).view(np.int64)).to(DEV)
    ok, ov = engine.read_lww(s, keys=kt)
    wk, wv = R.read_lww(rows, keys=sub)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)


def test_read_lww_config2(engine):
    a, b = W.config2()
    rows, _ = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    s = Store.from_numpy(*rows, device=DEV)
    ok, ov = engine.read_lww(s)
    wk, wv = R.read_lww(rows)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)


@pytest.mark.parametrize("seed", range(6))
def test_context_union_and_compress(engine, seed):
    rng = np.random.default_rng(seed)
    kinds = [(W.VV, W.VV), (W.DOTS, W.DOTS), (W.VV, W.DOTS)][seed % 3]
    a, _ = W.random_pair(rng, n_keys=200, ctx_kind=kinds[0], dense_ctx=False)
    b, _ = W.random_pair(rng, n_keys=200, ctx_kind=kinds[1], dense_ctx=False)
    _, ca = up(a)
    _, cb = up(b)
    ctx_eq(engine.context_union(ca, cb), R.context_union(a["ctx"], b["ctx"]))
    ctx_eq(engine.context_union(cb, ca), R.context_union(b["ctx"], a["ctx"]))
    if a["ctx"][0] == W.DOTS:
        ctx_eq(engine.compress_dots(ca), R.compress_dots(a["ctx"]))
    else:
        with pytest.raises(FunctionClauseError):
            engine.compress_dots(ca)


def test_large_dot_set_union(engine):
    n = 20000
    rng = np.random.default_rng(5)
    def dots():
        nd = np.sort(rng.integers(0, 50, n).astype(np.uint32))
        c = rng.integers(1, 10**6, n).astype(np.uint64)
        o = np.lexsort((c, nd))
        pairs = np.unique(np.stack([nd[o].astype(np.uint64), c[o]], 1), axis=0)
        return (W.DOTS, pairs[:, 0].astype(np.uint32), pairs[:, 1].astype(np.uint64))
    x, y = dots(), dots()
    cx = Context.from_numpy(*x, DEV)
    cy = Context.from_numpy(*y, DEV)
    ctx_eq(engine.context_union(cx, cy), R.context_union(x, y))
    ctx_eq(engine.compress_dots(cx), R.compress_dots(x))


@pytest.mark.parametrize("seed", range(3))
def test_joink(engine, seed):
    rng = np.random.default_rng(50 + seed)
    reps = []
    for _ in range(3):
        a, b = W.random_pair(rng, n_keys=400, ts_range=8, dense_ctx=bool(seed % 2))
        reps += [a, b]
    stores, ctxs = zip(*[up(r) for r in reps])
    out, octx = engine.joink(list(stores), list(ctxs))
    wr, wc = R.joink([r["rows"] for r in reps], [r["ctx"] for r in reps])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


def test_store_check_detects_unsorted(engine):
    a, _ = W.config2(n_keys=3000, seed=2)
    rows = list(a["rows"])
    s = Store.from_numpy(*rows, device=DEV)
    engine.store_check(s)
    rows = [c.copy() for c in rows]
    rows[0][[10, 11]] = rows[0][[11, 10]]
    bad = Store.from_numpy(*rows, device=DEV)
    with pytest.raises(Exception):
        engine.store_check(bad)


# ------------------------------------------------------------------ dg_sort_store (marshalling)

def _np_sorted_unique(rows):
    k, v, t, n, c = (np.asarray(x) for x in rows)
    o = np.lexsort((c, n, t, v, k))
    cols = [x[o] for x in (k, v, t, n, c)]
    if len(cols[0]) > 1:
        keep = np.ones(len(cols[0]), bool)
        keep[1:] = ~np.all([x[1:] == x[:-1] for x in cols], axis=0)
        cols = [x[keep] for x in cols]
    return tuple(cols)


def _shuffled(rows, rng, dup_frac=0.0):
    n = len(rows[0])
    order = rng.permutation(n)
    if dup_frac and n:
        order = np.concatenate([order, rng.choice(n, int(n * dup_frac))])
        order = rng.permutation(order)
    return tuple(np.ascontiguousarray(c[order]) for c in rows)


@pytest.mark.parametrize("n,seed", [(0, 0), (1, 1), (17, 2), (4095, 3), (4097, 4), (70_000, 5)])
def test_sort_store_random(engine, n, seed):
    rng = np.random.default_rng(seed)
    rows = (rng.integers(0, 1 << 64, n, dtype=np.uint64), rng.integers(0, 1 << 64, n, dtype=np.uint64),
            rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64),
            rng.integers(0, 1 << 32, n, dtype=np.uint32), rng.integers(0, 1 << 64, n, dtype=np.uint64))
    rows = _shuffled(rows, rng, dup_frac=0.1)
    s = Store.from_numpy(*rows, device=DEV)
    s.n = len(rows[0])
    rows_eq(engine.sort_store(s), _np_sorted_unique(rows))


def test_sort_store_ties_everywhere(engine):
    """Equal keys with many entries, equal (key, val) with ts ties of both signs, equal
    (key, val, ts) with several dots: the order falls through every field."""
    rng = np.random.default_rng(9)
    n = 50_000
    rows = (rng.integers(0, 40, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15),
            rng.integers(0, 5, n).astype(np.uint64), rng.integers(-3, 3, n).astype(np.int64),
            rng.integers(0, 4, n).astype(np.uint32), rng.integers(0, 1 << 40, n).astype(np.uint64))
    rows = _shuffled(rows, rng, dup_frac=0.3)
    s = Store.from_numpy(*rows, device=DEV)
    got = engine.sort_store(s)
    rows_eq(got, _np_sorted_unique(rows))
    engine.store_check(got)


def test_sort_then_join_equals_oracle(engine):
    """Config-2 replicas marshalled in a map-walk order (shuffled), sorted on the device,
    then joined: bit-exact with the oracle's join of the sorted replicas."""
    rng = np.random.default_rng(4)
    a, b = W.config2(n_keys=60_000, seed=4)
    sa = engine.sort_store(Store.from_numpy(*_shuffled(a["rows"], rng), device=DEV))
    sb = engine.sort_store(Store.from_numpy(*_shuffled(b["rows"], rng), device=DEV))
    ca = engine.sort_context(Context.from_numpy(a["ctx"][0], *[x[::-1].copy() for x in a["ctx"][1:]], DEV))
    cb = engine.sort_context(Context.from_numpy(b["ctx"][0], *[x[::-1].copy() for x in b["ctx"][1:]], DEV))
    out, octx = engine.join2(sa, ca, sb, cb)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


def test_sort_context_dots(engine):
    rng = np.random.default_rng(2)
    n = 30_000
    pairs = np.unique(np.stack([rng.integers(0, 70, n), rng.integers(0, 1 << 50, n)], 1), axis=0)
    perm = rng.permutation(len(pairs))
    c = Context.from_numpy(W.DOTS, pairs[perm, 0].astype(np.uint32), pairs[perm, 1].astype(np.uint64), DEV)
    got = engine.sort_context(c)
    ctx_eq(got, (W.DOTS, pairs[:, 0].astype(np.uint32), pairs[:, 1].astype(np.uint64)))


def test_remap_values_region_local(engine):
    """dg_remap_values rewrites only the relabelled region's ids (ids outside
    [old_ids[0], old_ids[-1]] -- canonical integers, the other region -- stay), keeps the
    store sorted, and refuses an id inside the region that its table lacks."""
    from delta_crdt_ex_amd._abi import DeltaGpuError
    key = np.repeat(np.arange(1, 5, dtype=np.uint64), 4)
    val = np.tile(np.array([5, 1 << 60, (1 << 60) + 8, 1 << 63], np.uint64), 4)
    rows = (key, val, np.zeros(16, np.int64), np.zeros(16, np.uint32),
            np.arange(1, 17, dtype=np.uint64))
    s = Store.from_numpy(*rows, device=DEV)
    old = np.array([1 << 60, (1 << 60) + 8], np.uint64)
    new = np.array([(1 << 60) - 100, (1 << 60) + 100], np.uint64)
    engine.remap_values(s, old, new)
    got = s.to_numpy()[1]
    want = val.copy()
    want[val == old[0]], want[val == old[1]] = new[0], new[1]
    assert np.array_equal(got, want)
    engine.store_check(s)
    with pytest.raises(DeltaGpuError):  # rows hold (1 << 60) -+ 100: inside, not in the table
        engine.remap_values(s, np.array([(1 << 60) - 200, (1 << 60) + 200], np.uint64),
                            np.array([(1 << 60) - 300, (1 << 60) + 300], np.uint64))
