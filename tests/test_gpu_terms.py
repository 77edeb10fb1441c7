"""read/1 bit-exact for arbitrary terms through the GPU host mirror: LWW ties between
string, atom, tuple, float and mixed int/float values resolve to the smallest
{value, ts} in Erlang term order (reference aw_lww_map.ex:211-216),
whatever order the values were interned in, and across value relabels (the Universe
re-spaces its ids and dg_remap_values rewrites the live device stores).  Node ids are
30-bit :rand.uniform terms (causal_crdt.ex:65) interned to dense ids.  Checked against
the term oracle (oracle/awlww_term.py)."""
import random

import pytest

from delta_crdt_ex_amd.interning import Universe
from oracle import awlww_term as T
from oracle.erlterm import Atom, EList, emap

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(engine):
    from delta_crdt_ex_amd import aw_lww_map
    aw_lww_map._ENGINE = engine
    return aw_lww_map


def concurrent(M, U, key, writes, base=None):
    """Each (value, ts, node) is an add by its own replica from the same base; the
    replicas' deltas are then joined into one state (mirror and oracle)."""
    m0 = base[0] if base else M.compress_dots(M.new(U))
    t0 = base[1] if base else T.compress_dots(T.new())
    ms, ts = m0, t0
    for v, t, n in writes:
        ms = M.join_all(ms, M.join(m0, M.add(key, v, n, m0, ts=t), [key]))
        ts = T.join(ts, T.join(t0, T.add(key, v, n, t0, t), [key]), sorted({key} | set(ts.value), key=repr))
    return ms, ts


def test_verdict_case_string_tie_interned_in_reverse(M):
    U = Universe()
    U.value("b")  # 'b' interned first: ids must still rank 'a' < 'b'
    ms, ts = concurrent(M, U, "k", [("b", 7, 1), ("a", 7, 2)])
    assert T.read(ts) == {"k": "a"}
    assert M.read(ms) == {"k": "a"}


@pytest.mark.parametrize("vals", [
    ["b", "a", "ab", ""],
    [Atom("zeta"), Atom("alpha"), None, True],
    [(2, "x"), (1, "y"), (1,), (1, 2, 3)],
    [2.5, 2, 3, -1.0, 1.5],              # mixed int / float
    [EList([2]), EList(), EList([1, 5]), emap({1: 2})],
    ["s", 4, Atom("a"), (0,), 1.5, EList([0])],  # one of each class
])
def test_term_valued_ts_ties(M, vals):
    for perm_seed in range(3):
        U = Universe()
        order = list(vals)
        random.Random(perm_seed).shuffle(order)
        for v in order:  # intern in a shuffled order
            U.value(v)
        writes = [(v, 50, 100 + i) for i, v in enumerate(vals)]
        ms, ts = concurrent(M, U, "k", writes)
        want = T.read(ts)
        got = M.read(ms)
        assert list(got) == ["k"]
        assert repr(got["k"]) == repr(want["k"]) and type(got["k"]) is type(want["k"])
        assert ms.value == ts.value


def test_random_term_ties_many_keys(M):
    rng = random.Random(11)
    pool = ["a", "b", "c", Atom("x"), Atom("y"), 1, 2, 1.5, 2.5, (1,), (1, "a"), EList([3])]
    U = Universe()
    ms, ts = M.compress_dots(M.new(U)), T.compress_dots(T.new())
    for key in range(25):
        writes = [(rng.choice(pool), rng.randrange(3), 200 + r) for r in range(rng.randint(1, 4))]
        ms, ts = concurrent(M, U, key, writes, (ms, ts))
    assert {k: repr(v) for k, v in M.read(ms).items()} == {k: repr(v) for k, v in T.read(ts).items()}


def test_int_and_equal_float_tie(M):
    """2 and 2.0 are distinct map keys ({2, ts} and {2.0, ts}); the oracle's Python dicts
    cannot hold both, so the expected winner comes from its term order directly
    (oracle/erlterm.compare: the integer first on a numeric tie -- unpinned on the BEAM
    side, see erlterm.py)."""
    from oracle.erlterm import term_sorted
    U = Universe()
    U.value(2.0)
    ms, _ = concurrent(M, U, "k", [(2.0, 4, 1), (2, 4, 2), (3, 3, 3)])
    assert ms.rows.n == 3  # both entries survive the join
    assert repr(M.read(ms)["k"]) == repr(term_sorted([2.0, 2])[0]) == "2"


def test_relabel_keeps_live_states_exact(M):
    U = Universe()
    a, b = 1.0, 2.0
    ms, ts = concurrent(M, U, "k", [(a, 9, 1), (b, 9, 2)])
    other, other_t = concurrent(M, U, "j", [("p", 3, 3), ("q", 3, 4)])
    epoch = U.val_epoch
    lo = a
    for _ in range(70):  # squeeze values into one gap until the Universe relabels
        lo = (lo + b) / 2
        U.value(lo)
    assert U.val_epoch > epoch
    # the states built before the relabel were remapped on the device
    assert M.read(ms) == T.read(ts) == {"k": 1.0}
    assert M.read(other) == T.read(other_t) == {"j": "p"}
    # and still join with states built after it
    ms2, ts2 = concurrent(M, U, "k", [(lo, 9, 5)], (ms, ts))
    assert M.read(ms2) == T.read(ts2)
    assert ms2.value == ts2.value


def test_30bit_node_ids_are_dense_on_the_device(M):
    rng = random.Random(3)
    nodes = [rng.randint(1, 1_000_000_000) for _ in range(5)]
    U = Universe()
    ms, ts = concurrent(M, U, "k", [(f"v{i}", 1, n) for i, n in enumerate(nodes)])
    dev_nodes = set(int(x) for x in ms.rows.node[: ms.rows.n].cpu().tolist())
    assert dev_nodes <= set(range(len(nodes)))
    assert M.read(ms) == T.read(ts)
    assert ms.dots == ts.dots and ms.value == ts.value


def test_from_terms_marshals_through_the_device_sort(M):
    """A term-level state marshalled in map-walk order and sorted on the device
    (dg_sort_store / dg_sort_context) is the oracle's state, and joins / reads like it."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as G
    U = Universe()
    reps = G.history(21, U, values=G.TERM_VALUES)
    A, B = reps[0], reps[1]
    V = Universe()
    ma, mb = M.from_terms(A.value, A.dots, V), M.from_terms(B.value, B.dots, V)
    assert ma.dots == A.dots and ma.value == A.value
    keys = sorted(set(A.value) | set(B.value))
    j, tj = M.join(ma, mb, keys), T.join(A, B, keys)
    assert j.value == tj.value and j.dots == tj.dots
    assert {k: repr(v) for k, v in M.read(j).items()} == {k: repr(v) for k, v in T.read(tj).items()}
