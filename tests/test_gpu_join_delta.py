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


def apply(engine, a, d, keys, depth=10, terms=None, with_tree=True):
    keys = np.unique(np.asarray(keys, np.uint64))
    st, sc = state_of(a, extra_ctx=len(d["ctx"][1]))
    sd, cd = up(d)
    spare = Store.empty(st.n + sd.n, DEV)
    tree = engine.merkle_build(st, depth, MerkleTree.empty(depth, DEV, terms=terms)) if with_tree else None
    changed, swapped = engine.join_delta(st, sc, sd, cd, kdev(keys), spare, tree)
    wr, wc = R.join2(a["rows"], a["ctx"], d["rows"], d["ctx"], keys=keys)
    rows_eq(st, wr)
    ctx_eq(sc, wc)
    assert np.array_equal(u64(changed), R.changed_keys(a["rows"], wr, keys))
    if with_tree:
        fresh = engine.merkle_build(st, depth, MerkleTree.empty(depth, DEV, terms=terms))
        assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
        assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())
        assert tree.n_keys == fresh.n_keys
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
