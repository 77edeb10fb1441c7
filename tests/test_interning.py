"""Interning (delta_crdt_ex_amd/interning.py) on the CPU: value ids follow Erlang term
order for every term class (the read tie-break, reference aw_lww_map.ex:211-216;
SURVEY.md §7 H2), survive relabels as a monotone map, and node ids are dense.
The term order itself is checked against the oracle's independent comparator
(oracle/erlterm.py)."""
import random

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from delta_crdt_ex_amd import workloads as W
from delta_crdt_ex_amd.interning import Universe
from delta_crdt_ex_amd.terms import Atom, EList, EMap, order_key
from oracle import erlterm as E

scalars = st.one_of(
    st.integers(-10, 10), st.integers(-(1 << 70), 1 << 70),
    st.floats(-20, 20, allow_nan=False, allow_infinity=False).filter(lambda x: x != 0.0 or
                                                                      str(x) == "0.0"),
    st.sampled_from([Atom("a"), Atom("b"), Atom("zz"), None, True, False]),
    st.text(max_size=3), st.binary(max_size=3))
terms = st.recursive(
    scalars,
    lambda ch: st.one_of(st.tuples(ch, ch), st.tuples(ch), st.lists(ch, max_size=3).map(EList),
                         st.dictionaries(st.integers(0, 3), ch, max_size=2).map(E.emap)),
    max_leaves=6)


@settings(max_examples=400, deadline=None)
@given(terms, terms)
def test_order_key_is_erlang_term_order(a, b):
    c = E.compare(a, b)
    ka, kb = order_key(a), order_key(b)
    assert (ka < kb) == (c < 0) and (ka == kb) == (c == 0)


@settings(max_examples=60, deadline=None)
@given(st.lists(terms, max_size=40))
def test_value_ids_follow_term_order(ts):
    U = Universe()
    ids = [U.value(t) for t in ts]
    for t, i in zip(ts, ids):
        assert U.value(t) == i and order_key(U.value_term(i)) == order_key(t)
    for x, y in zip(ts, ids):
        for z, w in zip(ts, ids):
            c = E.compare(x, z)
            assert (y < w) == (c < 0) and (y == w) == (c == 0)


def test_mixed_classes_rank_as_erlang():
    U = Universe()
    seq = ["b", "a", 7, 2.5, 3, Atom("x"), (1, 2), None, EList([1]), EList(), E.emap({1: 2}),
           (1,), 3.0, -(1 << 80), b"a"]
    for t in seq:
        U.value(t)
    got = sorted(seq, key=U.value)
    assert got == E.term_sorted(seq)
    # 1 and 1.0 (and True) are distinct values, also nested
    assert len({U.value(1), U.value(1.0), U.value(True)}) == 3
    assert U.value((1,)) != U.value((1.0,))
    # map-key order (OTP: "in maps key order integers types are considered less than
    # floats types"): every integer before every float, whatever the values
    assert U.value(1) < U.value(2) < U.value(1 << 70) < U.value(-5.0) < U.value(1.0) < U.value(1.5)
    assert U.value((2, 0)) < U.value((1.5, 0))


def test_canonical_integer_ids_are_universe_independent():
    from delta_crdt_ex_amd.interning import CANON_LO, CANON_HI, encode_int_value
    U, V = Universe(), Universe()
    for t in ("x", 2.5, Atom("a")):
        V.value(t)  # V's table differs from U's
    for v in (0, 1, -1, 7, CANON_LO, CANON_HI - 1, (1 << 62) - 5):
        assert U.value(v) == V.value(v) == int(encode_int_value([v])[0]) == v + (1 << 62)
        assert U.value_term(U.value(v)) == v
    # outside the canonical range: table ids, in order around the canonical block
    big_neg, big_pos = CANON_LO - 1, CANON_HI
    assert U.value(big_neg) < U.value(CANON_LO) < U.value(CANON_HI - 1) < U.value(big_pos)
    assert U.value(big_neg) < (1 << 58) and U.value(big_pos) >= (1 << 63)
    assert U.value_ids()[1] == [big_neg, big_pos]


def test_relabel_is_monotone_and_calls_the_hook():
    U = Universe()
    seen = []
    U.remap_hook = lambda old, new: seen.append((old.copy(), new.copy()))
    U.value(1.0)
    U.value(2.0)
    lo, hi = 1.0, 2.0
    for _ in range(80):  # every insert lands in the same, halving gap
        lo = (lo + hi) / 2
        U.value(lo)
    assert U.val_epoch >= 1 and seen
    for old, new in seen:
        assert np.all(np.diff(old.astype(object)) > 0) and np.all(np.diff(new.astype(object)) > 0)
    ids, ts = U.value_ids()
    assert ts == E.term_sorted(ts) and ids == sorted(ids)
    # ids handed out before the relabel map through the hook's table
    old, new = seen[-1]
    assert len(old) == len(new)


def test_random_inserts_stay_ordered_across_relabels():
    rng = random.Random(5)
    U = Universe()
    vals = []
    for _ in range(3000):
        x = rng.choice([rng.randint(-50, 50), rng.random() * 10, rng.choice("abcdef") * rng.randint(1, 3)])
        vals.append(x)
        U.value(x)
    ids, ts = U.value_ids()
    assert ts == E.term_sorted(ts)
    assert all(U.value(v) == i for v, i in zip(ts, ids))


def test_repeated_squeezes_keep_every_term():
    """Values squeezed into one gap again and again force relabel after relabel; a new
    evenly spaced id can equal an old id not yet moved (earlier midpoints), which the
    relabel must not mistake for the moved value (it used to lose terms: KeyError or a
    wrong term, found by the 1,500-op binding test)."""
    for seed in range(12):
        rng = random.Random(seed)
        U = Universe()
        vals = []
        for _ in range(6):
            a = rng.uniform(-1e6, 1e6)
            b = a + rng.uniform(1, 1000)
            seq = [a, b]
            for _ in range(rng.randrange(60, 140)):
                m = (a + b) / 2
                seq.append(m)
                if rng.random() < 0.5:
                    a = m
                else:
                    b = m
            seq += [rng.uniform(-1e6, 1e6) for _ in range(30)]
            seq += ["s%d" % rng.randrange(10**6) for _ in range(20)]
            for t in seq:
                U.value(t)
                vals.append(t)
        assert all(U.value_term(U.value(t)) == t for t in vals)
        ids, ts = U.value_ids()
        assert ids == sorted(set(ids)) and ts == E.term_sorted(ts)


def test_nodes_are_dense():
    U = Universe()
    assert [U.node(x) for x in (999_999_937, Atom("n"), 5, 999_999_937)] == [0, 1, 2, 0]
    assert U.node_term(1) == Atom("n")
    raw = np.array([700_000_001, 3, 700_000_001, 12], np.int64)
    V = Universe()
    d = V.node_ids(raw)
    assert d.tolist() == [2, 0, 2, 1] and V.node_term(2) == 700_000_001


def test_workload_node_ids_are_real_30bit_terms_interned_dense():
    a, b = W.config2(n_keys=2000, seed=3)
    N = a["nodes"]
    assert all(1 <= x <= 1_000_000_000 for x in N.raw.tolist())
    assert sorted(N.dense.tolist()) == [0, 1, 2]
    used = set(np.unique(np.concatenate([a["rows"][3], b["rows"][3], a["ctx"][1], b["ctx"][1]])))
    assert used <= {0, 1, 2}
    # config 3: 65 replicas -> dense ids 0..64, inside the one-pass fold's node tables
    base, deltas = W.config3(n_keys=5000, n_replicas=64, touch=0.01, seed=3)
    assert max(int(d["ctx"][1].max()) for d in deltas) == 64


def test_universe_tracks_device_stores_weakly():
    import gc

    from delta_crdt_ex_amd.store import Store
    U = Universe()
    s = Store.empty(4, "cpu")
    U.track(s)
    assert U.tracked() == [s]
    del s
    gc.collect()
    assert U.tracked() == []


def test_term_hash_tables_follow_their_universe():
    """tables made by TermHashes.of follow their Universe -- after new values
    or nodes are interned (or a relabel) `current()` hands out the new tables, so a tree
    never hashes a fresh id as itself; tables made from explicit arrays stay as they are."""
    from delta_crdt_ex_amd.store import TermHashes
    U = Universe()
    U.value("a")
    U.node("n1")
    th = TermHashes.of(U, "cpu")
    assert th.current() is th
    U.value(("a", "tuple"))
    U.node("n2")
    th2 = th.current()
    assert th2 is not th and th2.version == U.terms_version
    ids, _ = U.value_ids()
    assert len(th2.vid) >= len(ids) and th2.c.n_nodes == 2
    fixed = TermHashes(*U.term_tables(), "cpu")
    U.value("b")
    assert fixed.current() is fixed
