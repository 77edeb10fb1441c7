"""Merkle trees over TERMS (dg_term_hashes): two replicas whose
Universes interned the same terms in different orders -- as two BEAM nodes do -- build
bit-identical trees for equal states, their diff is exactly the keys whose raw value maps
differ, and a tree stays valid across a value relabel.  The reference hashes each key's
raw value map (causal_crdt.ex:390-394) and syncs with neighbours on other nodes
(causal_crdt_test.exs:68-78).  Checked against the C oracle's tree over the same term
hashes (oracle/deltaref.c ref_merkle_build with dg_term_hashes)."""
import os
import random
import sys

import numpy as np
import pytest

from delta_crdt_ex_amd.interning import Universe
from oracle import awlww_term as T
from oracle import ref as R

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402


@pytest.fixture(scope="module")
def M(engine):
    from delta_crdt_ex_amd import aw_lww_map
    aw_lww_map._ENGINE = engine
    return aw_lww_map


def _terms_of(state):
    vals, nodes = set(), set()
    for k, entries in state.value.items():
        for (v, ts), dots in entries.items():
            vals.add(v)
            nodes.update(n for n, _ in dots)
    return vals, nodes


def _shuffled_universe(state, seed):
    """A Universe that interned the state's values and nodes in a shuffled order first."""
    from oracle.erlterm import tg, untg
    U = Universe()
    vals, nodes = _terms_of(state)
    vals = [untg(x) for x in {tg(v) for v in vals}]
    nodes = sorted(nodes, key=repr)
    rng = random.Random(seed)
    rng.shuffle(vals)
    rng.shuffle(nodes)
    for v in vals:
        U.value(v)
    for n in nodes:
        U.node(n)
    return U


@pytest.mark.parametrize("seed", [0, 1])
def test_equal_states_build_equal_trees_across_universes(M, seed):
    A = G.history(200 + seed, Universe(), values=G.TERM_VALUES)[0]
    U1, U2 = _shuffled_universe(A, seed), _shuffled_universe(A, seed + 100)
    s1 = M.from_terms(A.value, A.dots, U1)
    s2 = M.from_terms(A.value, A.dots, U2)
    # different interning: different value / node ids on the device
    assert not all(np.array_equal(x, y) for x, y in zip(s1.rows.to_numpy(), s2.rows.to_numpy()))
    for depth in (4, 9):
        t1, t2 = M.merkle_map(s1, depth), M.merkle_map(s2, depth)
        assert np.array_equal(t1.nodes.cpu().numpy(), t2.nodes.cpu().numpy())
        assert np.array_equal(t1.bucket_counts(), t2.bucket_counts())
        # the C oracle over the same term hashes
        r = R.merkle_build(s1.rows.to_numpy(), depth, terms=R.Terms(*U1.term_tables()))
        assert np.array_equal(t1.nodes.cpu().numpy().view(np.uint64), r.nodes)
        assert M.merkle_diff(s1, t1, s2, t2) == []
    # ids alone would not agree: the same build without term hashes differs
    i1 = M.engine().merkle_build(s1.rows, 9)
    i2 = M.engine().merkle_build(s2.rows, 9)
    assert i1.root() != i2.root()


def test_diff_across_universes_is_the_value_map_diff(M):
    reps = G.history(210, Universe(), values=G.TERM_VALUES)
    A, B = reps[0], reps[1]
    U1, U2 = _shuffled_universe(A, 1), _shuffled_universe(B, 2)
    sa, sb = M.from_terms(A.value, A.dots, U1), M.from_terms(B.value, B.dots, U2)
    for depth in (3, 8, 13):
        ta, tb = M.merkle_map(sa, depth), M.merkle_map(sb, depth)
        got = M.merkle_diff(sa, ta, sb, tb)
        want = {k for k in set(A.value) | set(B.value) if A.value.get(k) != B.value.get(k)}
        assert set(got) == want and len(got) == len(want)


def test_tree_survives_a_relabel(M):
    A = G.history(220, Universe(), values=G.TERM_VALUES)[0]
    U = _shuffled_universe(A, 3)
    st = M.from_terms(A.value, A.dots, U)
    before = M.merkle_map(st, 8)
    epoch = U.val_epoch
    lo, hi = 1.0, 1.25
    for _ in range(80):  # squeeze floats into one gap until the Universe relabels
        hi = (lo + hi) / 2
        U.value(hi)
    assert U.val_epoch > epoch
    after = M.merkle_map(st, 8)  # the store's ids were rewritten by dg_remap_values
    assert np.array_equal(before.nodes.cpu().numpy(), after.nodes.cpu().numpy())
    # equal as Erlang terms (the Universe holds "a" as the binary b"a": tg normalises)
    from oracle.erlterm import tg
    assert {k: tg(v) for k, v in T.read(A).items()} == {k: tg(v) for k, v in M.read(st).items()}


def test_tree_follows_new_terms_after_build(M):
    """a tree built, then values and a node interned (new terms the tree's
    tables lack), then updated through Engine.merkle_update: the update picks up the
    Universe's current tables, so the tree equals a fresh build and the C oracle's."""
    from oracle.erlterm import tg
    A = G.history(230, Universe(), values=G.TERM_VALUES)[0]
    U = _shuffled_universe(A, 4)
    st = M.from_terms(A.value, A.dots, U)
    tree = M.merkle_map(st, 9)
    v0 = U.terms_version
    nxt = st
    for i, (k, v) in enumerate([("fresh-1", ("a", "tuple", 1)), ("fresh-2", b"\x01new"),
                                 (next(iter(A.value)), 3.75)]):
        nxt = M.join(nxt, M.add(k, v, ("a new node", i), nxt, ts=10 ** 15 + i), [k])
    assert U.terms_version != v0  # the build's tables are stale now
    changed = M.engine().join2_changes(st.rows, st.ctx, nxt.rows, nxt.ctx)[2]
    M.engine().merkle_update(tree, nxt.rows, changed)
    fresh = M.merkle_map(nxt, 9)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    r = R.merkle_build(nxt.rows.to_numpy(), 9, terms=R.Terms(*U.term_tables()))
    assert np.array_equal(tree.nodes.cpu().numpy().view(np.uint64), r.nodes)
    assert {tg(k): tg(v) for k, v in M.read(nxt).items()}[tg("fresh-2")] == tg(b"\x01new")
