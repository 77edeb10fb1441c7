"""The reference's AWLWWMap tests, run through the GPU-backed host mirror
(delta_crdt_ex_amd.aw_lww_map) and cross-checked state-for-state against the
term-level oracle.  Mirrors test/aw_lww_map_test.exs and
test/aw_lww_map_property_test.exs."""
import itertools

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from delta_crdt_ex_amd.interning import Universe
from oracle import awlww_term as T
from oracle.erlterm import Atom

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(engine):
    from delta_crdt_ex_amd import aw_lww_map
    aw_lww_map._ENGINE = engine
    return aw_lww_map


class Clock:
    def __init__(self, t=1000):
        self.t = t

    def __call__(self):
        self.t += 1
        return self.t


FOO = Atom("foo_node")


def same_state(m_state, t_state):
    """Mirror state == oracle state (contexts and every {v, ts} => dots entry)."""
    assert m_state.dots == t_state.dots
    assert m_state.value == t_state.value


def test_can_add_and_read_a_value(M):  # aw_lww_map_test.exs:7-11
    assert M.read(M.add(1, 2, FOO, M.new(Universe()), ts=5)) == {1: 2}


def test_can_join_two_adds(M):  # :13-20
    U = Universe()
    add1 = M.add(1, 2, FOO, M.new(U), ts=5)
    add2 = M.add(2, 2, FOO, add1, ts=6)
    assert M.read(M.join(add1, add2, [1, 2])) == {1: 2, 2: 2}
    t1 = T.add(1, 2, FOO, T.new(), 5)
    t2 = T.add(2, 2, FOO, t1, 6)
    same_state(M.join(add1, add2, [1, 2]), T.join(t1, t2, [1, 2]))


def test_can_remove_elements(M):  # :22-29
    U = Universe()
    add1 = M.add(1, 2, FOO, M.new(U), ts=5)
    assert M.read(M.join(add1, M.remove(1, FOO, add1), [1])) == {}


def test_can_resolve_conflicts(M):  # :31-40
    U = Universe()
    add1 = M.add(1, 2, FOO, M.new(U), ts=5)
    add2 = M.add(1, 3, FOO, add1, ts=6)
    j = M.join(add1, add2, [1])
    assert M.read(j) == {1: 3}
    t1 = T.add(1, 2, FOO, T.new(), 5)
    t2 = T.add(1, 3, FOO, t1, 6)
    same_state(j, T.join(t1, t2, [1]))


def test_can_compute_actual_dots_present(M):  # :42-49
    U = Universe()
    add1 = M.add(1, 2, FOO, M.new(U), ts=5)
    change1 = M.add(1, 3, FOO, add1, ts=6)
    final = M.join(add1, change1, [1])
    assert len(M.compress_dots(final).dots) == 1


def test_compress_dots_twice_raises(M):  # FunctionClauseError at aw_lww_map.ex:13
    from delta_crdt_ex_amd._abi import FunctionClauseError
    s = M.compress_dots(M.new(Universe()))
    with pytest.raises(FunctionClauseError):
        M.compress_dots(s)


keys_st = st.one_of(st.integers(0, 6), st.sampled_from(["a", "b", "c"]))
vals_st = st.one_of(st.integers(-3, 3), st.sampled_from(["x", "y", None]))
nodes_st = st.one_of(st.integers(0, 3), st.sampled_from([Atom("n1"), Atom("n2")]))
op_st = st.tuples(st.sampled_from(["add", "remove"]), keys_st, vals_st, nodes_st)


@settings(max_examples=25, deadline=None)
@given(st.lists(op_st, max_size=12))
def test_property_sequence_state_first(M, ops):  # aw_lww_map_property_test.exs:34-59
    U = Universe()
    c = Clock()
    ms = M.compress_dots(M.new(U))
    ts_ = T.compress_dots(T.new())
    model = {}
    for op, key, val, node in ops:
        if op == "add":
            t = c()
            ms = M.join(ms, M.add(key, val, node, ms, ts=t), [key])
            ts_ = T.join(ts_, T.add(key, val, node, ts_, t), [key])
            model[key] = val
        else:
            ms = M.join(ms, M.remove(key, node, ms), [key])
            ts_ = T.join(ts_, T.remove(key, node, ts_), [key])
            model.pop(key, None)
    assert M.read(ms) == model == T.read(ts_)
    same_state(ms, ts_)


@settings(max_examples=25, deadline=None)
@given(st.lists(op_st, max_size=12))
def test_property_sequence_delta_first(M, ops):  # aw_lww_map_test.exs:51-86
    U = Universe()
    c = Clock()
    ms = M.new(U)
    model = {}
    for op, key, val, node in ops:
        if op == "add":
            ms = M.join(M.add(key, val, node, ms, ts=c()), ms, [key])
            model[key] = val
        else:
            ms = M.join(M.remove(key, node, ms), ms, [key])
            model.pop(key, None)
    assert M.read(ms) == model


def test_convergence_after_partition(M):  # causal_crdt_test.exs:114-152 as pure joins
    U = Universe()
    c = Clock()
    reps = {1: M.compress_dots(M.new(U)), 2: M.compress_dots(M.new(U))}

    def mutate(i, f, *args):
        s = reps[i]
        d = M.add(args[0], args[1], i, s, ts=c()) if f == "add" else M.remove(args[0], i, s)
        reps[i] = M.join(s, d, [args[0]])

    def sync(i, j):
        # the receiver joins the sender's VV + values over all keys (send_diff shape)
        reps[j] = M.join_all(reps[j], reps[i])

    mutate(1, "add", "CRDT1", "represent")
    mutate(2, "add", "CRDT2", "also here")
    for i, j in itertools.permutations((1, 2)):
        sync(i, j)
    assert M.read(reps[1]) == {"CRDT1": "represent", "CRDT2": "also here"}
    mutate(1, "add", "CRDTa", "only present in 1")
    mutate(1, "remove", "CRDT1")
    assert "CRDTa" not in M.read(reps[2])
    for i, j in itertools.permutations((1, 2)):
        sync(i, j)
    for r in reps.values():
        out = M.read(r)
        assert "CRDTa" in out and "CRDT1" not in out
