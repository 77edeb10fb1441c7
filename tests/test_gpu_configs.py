"""BASELINE configs 3, 4 and 5 through libdeltagpu on cuda:0, bit-exact against the C
oracle (which tests/test_configs.py pins to the term oracle), at sizes the oracle
finishes in seconds, plus size-independent properties at larger sizes."""
import numpy as np
import pytest
import torch

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.store import Store, u64
from oracle import ref as R
from test_gpu_parity import DEV, ctx_eq, rows_eq, up

pytestmark = pytest.mark.gpu


def keys_dev(keys):
    return torch.from_numpy(np.ascontiguousarray(keys, np.uint64).view(np.int64)).to(DEV)


def gpu_apply(engine, base, deltas, keys=True):
    sb, cb = up(base)
    ds, dc = zip(*[up(d) for d in deltas]) if deltas else ((), ())
    ks = [keys_dev(d["keys"]) for d in deltas] if keys else None
    return engine.apply_deltas(sb, cb, list(ds), list(dc), ks)


# ------------------------------------------------------------------ config 3

@pytest.mark.parametrize("n_keys,n_rep", [(100_000, 64), (3_000, 8)])
def test_config3_apply_deltas_parity(engine, n_keys, n_rep):
    base, deltas = W.config3(n_keys=n_keys, n_replicas=n_rep, touch=0.01 if n_keys > 10_000
                             else 0.05, seed=1)
    out, octx = gpu_apply(engine, base, deltas)
    wr, wc = R.apply_deltas(base["rows"], base["ctx"], [d["rows"] for d in deltas],
                            [d["ctx"] for d in deltas], [d["keys"] for d in deltas])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


def test_config3_edge_cases(engine):
    base, deltas = W.config3(n_keys=2_000, n_replicas=3, touch=0.05, seed=4)
    # no deltas: the state itself
    out, octx = gpu_apply(engine, base, [])
    rows_eq(out, base["rows"])
    ctx_eq(octx, base["ctx"])
    # an empty keyset joins no key: delta rows are carried right-biased
    d = dict(deltas[0])
    d["keys"] = np.zeros(0, np.uint64)
    out, octx = gpu_apply(engine, base, [d])
    wr, wc = R.join2(base["rows"], base["ctx"], d["rows"], d["ctx"], keys=np.zeros(0, np.uint64))
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    # full-state deltas (keys None) are plain joins
    out, octx = gpu_apply(engine, base, deltas, keys=False)
    wr, wc = R.apply_deltas(base["rows"], base["ctx"], [x["rows"] for x in deltas],
                            [x["ctx"] for x in deltas])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


def test_config3_idempotent_large(engine):
    """Re-applying the same 64 deltas to the result changes nothing (join is
    idempotent), at 2M keys; and the result keeps no base row of a touched key."""
    base, deltas = W.config3(n_keys=2_000_000, n_replicas=64, touch=0.01, seed=7)
    out, octx = gpu_apply(engine, base, deltas)
    ds, dc = zip(*[up(d) for d in deltas])
    again, actx = engine.apply_deltas(out, octx, list(ds), list(dc),
                                      [keys_dev(d["keys"]) for d in deltas])
    a, b = out.to_numpy(), again.to_numpy()
    assert out.n == again.n and all(np.array_equal(x, y) for x, y in zip(a, b))
    assert np.array_equal(octx.to_numpy()[1], actx.to_numpy()[1])
    touched = np.unique(np.concatenate([d["keys"] for d in deltas]))
    assert not np.any(np.isin(a[0][a[3] == base["nodes"][0]], touched))
    engine.store_check(out)


# ------------------------------------------------------------------ config 5

@pytest.mark.parametrize("seed", range(2))
def test_config5_join_read_parity(engine, seed):
    a, b = W.config5(n_keys=200_000, n_nodes=64, seed=seed)
    sa, ca = up(a)
    sb, cb = up(b)
    out, octx = engine.join2(sa, ca, sb, cb)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    ok, ov = engine.read_lww(out)
    wk, wv = R.read_lww(wr)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)


def test_config5_properties_large(engine):
    """2M keys: join(A,B) == join(B,A) row for row, join(J,J) == J, sorted+unique."""
    a, b = W.config5(n_keys=2_000_000, n_nodes=64, seed=9)
    sa, ca = up(a)
    sb, cb = up(b)
    j1, c1 = engine.join2(sa, ca, sb, cb)
    j2, c2 = engine.join2(sb, cb, sa, ca)
    x, y = j1.to_numpy(), j2.to_numpy()
    assert j1.n == j2.n and all(np.array_equal(p, q) for p, q in zip(x, y))
    jj, _ = engine.join2(j1, c1, j1, c1)
    z = jj.to_numpy()
    assert jj.n == j1.n and all(np.array_equal(p, q) for p, q in zip(x, z))
    engine.store_check(j1)


def test_config5_shards_join_to_the_unsharded_join(engine):
    """Config 5 at weak scaling: the 8 key-hash shards of a 4M-key pair are
    exact slices of the unsharded pair, and their 8 independent device joins (as the ranks
    of bench.py --gpus 8 run them, no data-path collective) concatenate to the unsharded
    device join, row for row, with equal contexts and reads."""
    from delta_crdt_ex_amd.sharding import shard_of
    world, per = 8, 500_000
    a, b = W.config5(n_keys=world * per, n_nodes=64, seed=5)
    whole, wctx = engine.join2(*up(a), *up(b))
    wrows = whole.to_numpy()
    sh = shard_of(wrows[0], world)
    for r in range(world):
        pa, pb = W.config5_shard(r, world, keys_per_rank=per)
        for x, y in zip(pa["rows"], tuple(c[shard_of(a["rows"][0], world) == r] for c in a["rows"])):
            assert np.array_equal(x, y)  # the shard is the pair's slice
        out, octx = engine.join2(*up(pa), *up(pb))
        for x, y in zip(out.to_numpy(), (c[sh == r] for c in wrows)):
            assert np.array_equal(x, y)
        ctx_eq(octx, (0,) + tuple(wctx.to_numpy()))
        k1, v1 = engine.read_lww(out)
        k0, v0 = engine.read_lww(whole)
        m = shard_of(u64(k0), world) == r
        assert np.array_equal(u64(k1), u64(k0)[m]) and np.array_equal(u64(v1), u64(v0)[m])


@pytest.mark.timeout(600)
def test_config5_full_share_parity(engine):
    """The bench's config-5 workload itself (one GPU's share of 100M keys: 12.5M keys,
    22.5M rows in), bit-exact against the C oracle's join and read."""
    a, b = W.config5(n_keys=12_500_000, n_nodes=64, seed=5)
    sa, ca = up(a)
    sb, cb = up(b)
    out, octx = engine.join2(sa, ca, sb, cb)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    ok, ov = engine.read_lww(out)
    wk, wv = R.read_lww(wr)
    assert np.array_equal(u64(ok), wk) and np.array_equal(u64(ov), wv)


@pytest.mark.timeout(600)
def test_config3_full_size_parity(engine):
    """The bench's config-3 batch itself (10M keys, 64 keyed deltas) through the one-pass
    fold, bit-exact against the C oracle's delta-by-delta fold."""
    base, deltas = W.config3(n_keys=10_000_000, n_replicas=64, touch=0.01, seed=3)
    out, octx = gpu_apply(engine, base, deltas)
    wr, wc = R.apply_deltas(base["rows"], base["ctx"], [d["rows"] for d in deltas],
                            [d["ctx"] for d in deltas], [d["keys"] for d in deltas])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


# ------------------------------------------------------------------ config 4

@pytest.mark.parametrize("rank", range(8))
def test_config4_shard_round(engine, rank):
    """One key-hash shard of 8: GPU Merkle build + diff finds exactly the differing
    keys, and joining B's sync delta for them into A equals the full join."""
    a, b = W.config4_shard(rank, 8, keys_per_rank=50_000, diff_frac=0.01)
    sa, ca = up(a)
    sb, cb = up(b)
    ta = engine.merkle_build(sa, 11, shard_bits=3, shard=rank)
    tb = engine.merkle_build(sb, 11, shard_bits=3, shard=rank)
    diff = engine.merkle_diff(ta, tb)
    want = R.store_diff(a["rows"], b["rows"])
    assert np.array_equal(u64(diff), want)
    d = W.sync_delta(b, want)
    sd, cd = up(d)
    out, octx = engine.apply_deltas(sa, ca, [sd], [cd], [diff])
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    assert isinstance(out, Store)


# ------------------------------------------------------------------ sync deltas (§8(f).2)

def test_take_keys_edges(engine):
    a, b = W.config4_shard(1, 8, keys_per_rank=20_000, diff_frac=0.02)
    sb, _ = up(b)
    bk = np.unique(b["rows"][0])
    for keys in (np.zeros(0, np.uint64),                       # no key
                 np.array([1, 2, 3], np.uint64),               # keys the store lacks
                 bk,                                            # every key: the store itself
                 bk[::7], np.concatenate([bk[:5], bk[-5:]])):   # spread / both ends
        got = engine.take_keys(sb, keys_dev(keys))
        want = W.sync_delta(b, keys)["rows"]
        rows_eq(got, want)


@pytest.mark.parametrize("rank", [0, 5])
def test_config4_round_device_resident(engine, rank):
    """The anti-entropy round entirely on the device: Merkle build + diff, the sync
    delta Map.take(B.value, diff keys) (dg_take_keys) with B's context, and the keyed
    join into A -- equal to the full-state join of the shard."""
    a, b = W.config4_shard(rank, 8, keys_per_rank=80_000, diff_frac=0.01)
    sa, ca = up(a)
    sb, cb = up(b)
    diff = engine.merkle_diff(engine.merkle_build(sa, 11, shard_bits=3, shard=rank),
                              engine.merkle_build(sb, 11, shard_bits=3, shard=rank))
    delta = engine.take_keys(sb, diff)
    out, octx = engine.join2(sa, ca, delta, cb, keys=diff)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)


@pytest.mark.timeout(600)
def test_config4_full_shard_round(engine):
    """The bench's config-4 round at its own size: one 12.5M-key shard of 100M keys
    (rank 3 of 8, depth 22, trees hashed through node terms), two replicas differing on
    1 % of the keys.  Merkle diff == the oracle's differing keys; the keyed join of the
    sync delta Map.take(B, diff) with its changed keys == the full-state join; the
    incremental tree update == a fresh build of the joined store."""
    from delta_crdt_ex_amd.store import MerkleTree, TermHashes
    rank, world = 3, 8
    a, b = W.config4_shard(rank, world, keys_per_rank=12_500_000, diff_frac=0.01)
    terms = TermHashes(*a["nodes"].universe.term_tables(), DEV)
    sa, ca = up(a)
    sb, cb = up(b)
    depth = 22
    ta = engine.merkle_build(sa, depth, MerkleTree.empty(depth, DEV, 3, rank, terms), 3, rank)
    tb = engine.merkle_build(sb, depth, MerkleTree.empty(depth, DEV, 3, rank, terms), 3, rank)
    diff, total = engine.merkle_diff(ta, tb, with_total=True)
    want = R.store_diff(a["rows"], b["rows"])
    assert total == len(want) and np.array_equal(u64(diff), want)
    cap = 1000  # max_sync_size: the first keys in key order, and the total
    first, total_c = engine.merkle_diff(ta, tb, cap=cap, with_total=True)
    assert total_c == len(want) and np.array_equal(u64(first), want[:cap])
    delta = engine.take_keys(sb, diff)
    rows_eq(delta, W.sync_delta(b, want)["rows"])
    out, octx, changed = engine.join2_changes(sa, ca, delta, cb, keys=diff)
    wr, wc = R.join2(a["rows"], a["ctx"], b["rows"], b["ctx"])
    rows_eq(out, wr)
    ctx_eq(octx, wc)
    tt = ta.clone()
    engine.merkle_update(tt, out, changed)
    fresh = engine.merkle_build(out, depth, None, 3, rank, terms=terms)
    assert np.array_equal(tt.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    assert tt.root() == tb.root()  # the joined shard holds exactly B's rows of the shard
