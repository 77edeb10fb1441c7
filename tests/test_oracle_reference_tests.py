"""The reference's own tests, restated against the term-level oracle.

This pins oracle/awlww_term.py (and through tests/test_c_oracle.py the C oracle,
and through the gpu tests libdeltagpu) to the behaviour the reference asserts:

* test/aw_lww_map_test.exs:7-49   — five unit KATs
* test/aw_lww_map_test.exs:51-86  — sequential-model property (delta-first join)
* test/aw_lww_map_property_test.exs:18-76 — add / sequence / remove properties
  (state-first join, compressed start)
* test/causal_crdt_test.exs:28-54,114-171 — convergence scenarios, re-expressed as
  pure joins of sync-shaped deltas (causal_crdt.ex:112-118,324-335)

The reference itself cannot run here (no BEAM), see SURVEY.md §8(c).
"""
import itertools

from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import awlww_term as T
from oracle.erlterm import Atom, EList, tg

FOO = Atom("foo_node")


class Clock:
    """Stand-in for System.monotonic_time(:nanosecond): strictly increasing."""

    def __init__(self, start=1_000):
        self.t = start

    def __call__(self):
        self.t += 1
        return self.t


def add(key, val, node, state, clock):
    return T.add(key, val, node, state, clock())


# ------------------------------------------------------------- unit KATs

def test_can_add_and_read_a_value():  # aw_lww_map_test.exs:7-11
    c = Clock()
    assert T.read(add(1, 2, FOO, T.new(), c)) == {1: 2}


def test_can_join_two_adds():  # :13-20
    c = Clock()
    add1 = add(1, 2, FOO, T.new(), c)
    add2 = add(2, 2, FOO, add1, c)
    assert T.read(T.join(add1, add2, [1, 2])) == {1: 2, 2: 2}


def test_can_remove_elements():  # :22-29
    c = Clock()
    add1 = add(1, 2, FOO, T.new(), c)
    remove1 = T.remove(1, FOO, add1)
    assert T.read(T.join(add1, remove1, [1])) == {}


def test_can_resolve_conflicts():  # :31-40
    c = Clock()
    add1 = add(1, 2, FOO, T.new(), c)
    add2 = add(1, 3, FOO, add1, c)
    joined = T.join(add1, add2, [1])
    assert T.read(joined) == {1: 3}
    # the TODO at :35 — "assert that the state doesn't include anything about value 2"
    assert all(v != 2 for (v, _ts) in joined.value[1])


def test_can_compute_actual_dots_present():  # :42-49
    c = Clock()
    add1 = add(1, 2, FOO, T.new(), c)
    change1 = add(1, 3, FOO, add1, c)
    final = T.join(add1, change1, [1])
    assert len(T.compress_dots(final).dots) == 1


# ------------------------------------------------------------- properties

def terms():
    leaves = st.one_of(
        st.integers(-(1 << 70), 1 << 70),
        st.text(max_size=4),
        st.binary(max_size=4),
        st.sampled_from([None, True, False, Atom("a"), Atom("zz")]),
        st.floats(allow_nan=False, allow_infinity=False, width=32),
    )
    # wrapped so that oracle maps use Erlang's exact key equality (0 vs 0.0, ...)
    return st.recursive(
        leaves,
        lambda ch: st.one_of(st.tuples(ch, ch), st.lists(ch, max_size=3).map(EList)),
        max_leaves=4,
    ).map(tg)


op_gen = st.tuples(st.sampled_from(["add", "remove"]), terms(), terms(), terms())


def model(ops):
    m = {}
    for op, key, val, _node in ops:
        if op == "add":
            m[key] = val
        else:
            m.pop(key, None)
    return m


def _rekey(d):
    return d


@settings(max_examples=150, deadline=None)
@given(st.lists(op_gen, max_size=25))
def test_property_sequence_delta_first(ops):  # aw_lww_map_test.exs:51-86
    c = Clock()
    state = T.new()
    for op, key, val, node in ops:
        if op == "add":
            state = T.join(add(key, val, node, state, c), state, [key])
        else:
            state = T.join(T.remove(key, node, state), state, [key])
    assert _rekey(T.read(state)) == model(ops)


@settings(max_examples=150, deadline=None)
@given(terms(), terms(), terms())
def test_property_can_add_an_element(key, val, node):  # aw_lww_map_property_test.exs:18-33
    c = Clock()
    start = T.compress_dots(T.new())
    s = T.join(T.compress_dots(T.new()), add(key, val, node, start, c), [key])
    assert _rekey(T.read(s)) == {key: val}


@settings(max_examples=150, deadline=None)
@given(st.lists(op_gen, max_size=25))
def test_property_sequence_state_first(ops):  # aw_lww_map_property_test.exs:34-59
    c = Clock()
    state = T.compress_dots(T.new())
    for op, key, val, node in ops:
        if op == "add":
            state = T.join(state, add(key, val, node, state, c), [key])
        else:
            state = T.join(state, T.remove(key, node, state), [key])
    assert _rekey(T.read(state)) == model(ops)


@settings(max_examples=150, deadline=None)
@given(terms(), terms(), terms())
def test_property_can_remove_an_element(key, val, node):  # aw_lww_map_property_test.exs:61-75
    c = Clock()
    crdt = T.compress_dots(T.new())
    crdt = T.join(crdt, add(key, val, node, crdt, c), [key])
    crdt = T.join(crdt, T.remove(key, node, crdt), [key])
    assert T.read(crdt) == {}


# ------------------------------------------------------------- convergence as pure joins

class Replica:
    """A CausalCrdt reduced to its crdt_state (causal_crdt.ex:64-73) + handle_operation."""

    def __init__(self, node, clock):
        self.node = node
        self.clock = clock
        self.state = T.compress_dots(T.new())

    def mutate(self, f, *args):  # causal_crdt.ex:337-342 + :383-384
        key = args[0]
        if f == "add":
            delta = T.add(key, args[1], self.node, self.state, self.clock())
        else:
            delta = T.remove(key, self.node, self.state)
        self.state = T.join(self.state, delta, [key])

    def read(self):
        return T.read(self.state)


def diff_keys(a: T.AW, b: T.AW):
    """What MerkleMap's diff yields: keys whose raw value maps differ (causal_crdt.ex:392)."""
    keys = set(a.value) | set(b.value)
    return [k for k in keys if a.value.get(k) != b.value.get(k)]


def sync(frm: Replica, to: Replica):
    """One directional sync round: send_diff / get_diff (causal_crdt.ex:112-118,324-335)."""
    keys = diff_keys(frm.state, to.state)
    if not keys:
        return
    delta = T.AW(frm.state.dots, {k: frm.state.value[k] for k in keys if k in frm.state.value})
    to.state = T.join(to.state, delta, keys)


def test_conflicting_updates_resolve():  # causal_crdt_test.exs:28-36
    c = Clock()
    r = [Replica(n, c) for n in (11, 22, 33)]
    for v in ("one_wins", "two_wins", "three_wins"):
        r[0].mutate("add", "Derek", v)
    for a, b in itertools.permutations(r, 2):
        sync(a, b)
    for x in r:
        assert x.read() == {"Derek": "three_wins"}


def test_add_wins():  # :38-44
    c = Clock()
    c1, c2 = Replica(1, c), Replica(2, c)
    c1.mutate("add", "Derek", "add_wins")
    c2.mutate("remove", "Derek")
    sync(c1, c2)
    sync(c2, c1)
    assert c1.read() == {"Derek": "add_wins"} == c2.read()


def test_can_remove():  # :46-54
    c = Clock()
    c1, c2 = Replica(1, c), Replica(2, c)
    c1.mutate("add", "Derek", "add_wins")
    sync(c1, c2)
    assert c2.read() == {"Derek": "add_wins"}
    c1.mutate("remove", "Derek")
    sync(c1, c2)
    assert c1.read() == {} == c2.read()


def test_sync_is_directional():  # :57-66
    c = Clock()
    c1, c2 = Replica(1, c), Replica(2, c)
    c1.mutate("add", "Derek", "Kraan")
    c2.mutate("add", "Tonci", "Galic")
    sync(c1, c2)
    assert c1.read() == {"Derek": "Kraan"}
    assert c2.read() == {"Derek": "Kraan", "Tonci": "Galic"}


def test_sync_after_network_partition():  # :114-152
    c = Clock()
    c1, c2 = Replica(1, c), Replica(2, c)
    c1.mutate("add", "CRDT1", "represent")
    c2.mutate("add", "CRDT2", "also here")
    sync(c1, c2)
    sync(c2, c1)
    assert c1.read() == {"CRDT1": "represent", "CRDT2": "also here"}
    c1.mutate("add", "CRDTa", "only present in 1")
    c1.mutate("add", "CRDTb", "only present in 1")
    c1.mutate("remove", "CRDT1")
    assert "CRDTa" in c1.read() and "CRDTa" not in c2.read()
    sync(c1, c2)
    sync(c2, c1)
    for x in (c1, c2):
        assert "CRDTa" in x.read() and "CRDT1" not in x.read()


def test_syncing_when_values_happen_to_be_the_same():  # :154-171
    c = Clock()
    c1, c2 = Replica(1, c), Replica(2, c)
    c1.mutate("add", "key", "value")
    c2.mutate("add", "key", "value")
    sync(c1, c2)
    sync(c2, c1)
    c1.mutate("remove", "key")
    sync(c1, c2)
    sync(c2, c1)
    assert "key" not in c1.read() and "key" not in c2.read()


def test_add_nil_reads_as_nil():  # delta_subscriber_test.exs:26-27 (reported as {:remove, k})
    c = Clock()
    r = Replica(1, c)
    r.mutate("add", "Derek", "Kraan")
    r.mutate("add", "Derek", None)
    assert r.read() == {"Derek": None}


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 2), st.sampled_from(["add", "remove", "sync"]),
                          st.integers(0, 5), st.integers(0, 3), st.integers(0, 2)),
                max_size=40))
def test_random_histories_converge(steps):
    """Any interleaving of ops and directional syncs converges after a full sync
    round (the anti-entropy guarantee the reference's integration tests rely on)."""
    c = Clock()
    reps = [Replica(100 + i, c) for i in range(3)]
    for who, op, key, val, other in steps:
        if op == "sync":
            sync(reps[who], reps[other])
        else:
            reps[who].mutate(op, key, val)
    for _ in range(2):
        for a, b in itertools.permutations(reps, 2):
            sync(a, b)
    reads = [x.read() for x in reps]
    assert reads[0] == reads[1] == reads[2]
    assert T.canon(reps[0].state)[1] == T.canon(reps[1].state)[1] == T.canon(reps[2].state)[1]


# ------------------------------------------------------------- on_diffs (delta_subscriber_test.exs)

class Subscribed(Replica):
    """A replica whose mutations go through update_state_with_delta/3 and collect what
    its on_diffs subscriber receives (causal_crdt.ex:337-342,361-404)."""

    def __init__(self, node, clock):
        super().__init__(node, clock)
        self.received = []  # each on_diffs call's list (None calls are not made)

    def apply(self, delta, keys):
        self.state, got = T.update_state_with_delta(self.state, delta, keys)
        if got is not None:
            self.received.append(got)
        return got

    def mutate(self, f, *args):
        key = args[0]
        if f == "add":
            delta = T.add(key, args[1], self.node, self.state, self.clock())
        else:
            delta = T.remove(key, self.node, self.state)
        return self.apply(delta, [key])


def test_subscriber_receives_diffs():  # delta_subscriber_test.exs:11-28 (and :30-47)
    r = Subscribed(1, Clock())
    assert r.mutate("add", "Derek", "Kraan") == [("add", "Derek", "Kraan")]
    # the same value again: the raw map changed (fresh dot and ts), the read did not
    assert r.mutate("add", "Derek", "Kraan") == []
    # add k nil reports {:remove, k} (:26-27): Map.get of a nil value is nil
    assert r.mutate("add", "Derek", None) == [("remove", "Derek")]
    # and removing the nil value reports nothing: {nil, nil} matches {old, old}
    assert r.mutate("remove", "Derek") == []
    # removing an absent key changes no raw map: the callback is not called
    assert r.mutate("remove", "Derek") is None


def test_subscriber_updates_are_bundled():  # delta_subscriber_test.exs:49-77
    c = Clock()
    c1, c2 = Replica(1, c), Subscribed(2, c)
    for k in ("Derek", "Andrew", "Nathan"):
        c1.mutate("add", k, "Kraan")
    keys = diff_keys(c1.state, c2.state)
    delta = T.AW(c1.state.dots, {k: c1.state.value[k] for k in keys if k in c1.state.value})
    got = c2.apply(delta, keys)
    assert {k: v for _, k, v in got} == {"Derek": "Kraan", "Andrew": "Kraan", "Nathan": "Kraan"}


def _replay(received):
    m = {}
    for diffs in received:
        for d in diffs:
            if d[0] == "add":
                m[d[1]] = d[2]
            else:
                m.pop(d[1], None)
    return m


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["add", "remove"]), terms(), terms()), max_size=25))
def test_property_diff_stream_replays_to_the_model(ops):  # delta_subscriber_test.exs:79-117
    """The on_diffs stream, replayed into a map, equals Map.put/Map.delete over the ops
    -- with nil values dropped, since an add of nil is reported as a remove."""
    r = Subscribed(1, Clock())
    for op, key, val in ops:
        r.mutate(op, key, val)
    want = {k: v for k, v in model([(o, k, v, None) for o, k, v in ops]).items()
            if v != tg(None)}
    assert _replay(r.received) == want
