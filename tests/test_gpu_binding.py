"""The Elixir binding of INTEGRATION.md §3 (mirrored in tests/binding_mirror.py) over the
NIF's own device half (c_src/replica.c via delta_crdt_ex_amd/nif.py): a GPU-attached
replica must behave like the reference's immutable states.

* delta_subscriber_test.exs:11-28 and :49-77 through GPU-attached replicas (thresholds 0);
* read/2 of the PRE-join struct returns the pre-join values (diffs_to_callback reads the
  old state after the join, causal_crdt.ex:361-365), and the NIF refuses its version;
* a local mutation keeps the device attached, queued, and the next device call flushes it;
* send_diff / get_diff ship no device handle or queue (causal_crdt.ex:118,331);
* the sequential-model property (aw_lww_map_property_test.exs:34-59) with mutations
  interleaved with sync rounds between two GPU replicas, call for call against the same
  history on CPU-only replicas (the reference's code);
* two "BEAM nodes" (two engines, two universes): keys one node never interned cross the
  protocol as {:"$dg_key", id} and are resolved where they are known.
"""
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import binding_mirror as B
from oracle import awlww_term as T
from oracle.erlterm import tg

pytestmark = pytest.mark.gpu


class Clock:
    def __init__(self, start=1_000):
        self.t = start

    def __call__(self):
        self.t += 1
        return self.t


@pytest.fixture(scope="module", autouse=True)
def gpu_node():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X: torch.cuda.is_available() is False")
    saved = (B.GPU_MIN_DOTS, B.GPU_MIN_READ_KEYS)
    B.GPU_MIN_DOTS, B.GPU_MIN_READ_KEYS = 0, 0  # every replica and every read on the device
    B.GPU.load_nif(0)
    assert B.GPU.engine() is not None
    yield
    B.GPU.close()
    B.GPU_MIN_DOTS, B.GPU_MIN_READ_KEYS = saved


def attached(r):
    return r.crdt_state.gpu is not None


def test_subscriber_receives_diffs():  # delta_subscriber_test.exs:11-28
    r = B.Replica(1, Clock())
    assert attached(r)
    r.mutate("add", "Derek", "Kraan")
    assert r.received[-1] == [("add", tg("Derek"), tg("Kraan"))]
    r.mutate("add", "Derek", "Kraan")  # refute_received: same value, new dot
    assert r.received[-1] == []
    r.mutate("add", "Derek", None)  # add k nil -> {:remove, k} (:26-27)
    assert r.received[-1] == [("remove", tg("Derek"))]
    assert attached(r), "a local mutation must not detach the replica"
    # the three mutations are queued; a device call flushes them as one batch
    assert len(r.crdt_state.gpu[2]) == 3
    ver = r.crdt_state.gpu[1]
    r.crdt_state, _ = B.merkle_prepare(r.crdt_state, B.LEVELS)
    assert r.crdt_state.gpu[2] == () and r.crdt_state.gpu[1] == ver + 1
    assert r.read() == B.read_cpu(r.crdt_state) == {tg("Derek"): tg(None)}


def test_updates_are_bundled():  # delta_subscriber_test.exs:49-77
    c = Clock()
    c1, c2 = B.Replica(1, c), B.Replica(2, c)
    for k in ("Derek", "Andrew", "Nathan"):
        c1.mutate("add", k, "Kraan")
    c2.received.clear()
    trace = []
    c1.sync_to(c2, trace)
    assert trace.count("diff") >= 2, trace  # continuations, then the delta itself
    assert len(c2.received) == 1, c2.received
    assert {k: v for _, k, v in c2.received[0]} == {tg("Derek"): tg("Kraan"), tg("Andrew"): tg("Kraan"),
                                                    tg("Nathan"): tg("Kraan")}
    assert c2.read() == c1.read()
    assert attached(c1) and attached(c2)


def test_read_of_the_pre_join_struct():
    """diffs_to_callback reads the old struct after the join (causal_crdt.ex:361-365): its
    values, not the device's newer ones; the NIF refuses its version outright."""
    c = Clock()
    src = B.Replica(9, c, gpu=False)
    for i in range(40):
        src.mutate("add", f"k{i}", i)
    r = B.Replica(1, c)
    for i in range(0, 40, 2):
        r.mutate("add", f"k{i}", -i)
    r.crdt_state, _ = B.merkle_prepare(r.crdt_state, B.LEVELS)  # flushed: device == terms
    old = r.crdt_state
    keys = [tg(f"k{i}") for i in range(40)]
    before = B.read_cpu(old, keys)
    delta = B.detach(B.AW(src.crdt_state.dots, dict(src.crdt_state.value)))
    new = B.join(old, delta, keys)
    assert new.gpu is not None and new.gpu[1] == old.gpu[1] + 1
    assert B.read(old, keys) == before  # stale on the device: the old terms answer
    assert B.read(old) == B.read_cpu(old)
    assert B.read(new, keys) == B.read_cpu(new, keys) != before
    res, ver, _ = old.gpu
    assert B.GPU.read(res, ver, keys) == ("error", "stale")
    assert B.GPU.read(res, new.gpu[1], keys)[1] == B.read_cpu(new, keys)
    # the whole subscriber path: every key the join changed is reported
    r.crdt_state = old
    r.received.clear()
    r.update_state_with_delta(delta, keys)
    got = {k: v for _, k, v in r.received[-1]}
    assert got == {k: v for k, v in B.read_cpu(new, keys).items() if before.get(k) != v}
    assert len(got) == 20  # the odd keys: r's later writes win the even ones (LWW)


def test_a_stale_struct_joins_on_its_own_terms():
    c = Clock()
    r = B.Replica(1, c)
    for i in range(10):
        r.mutate("add", i, i)
    r.crdt_state, _ = B.merkle_prepare(r.crdt_state, B.LEVELS)
    s0 = r.crdt_state
    d1 = B.detach(B.add(tg(3), tg(33), tg(7), B.AW({tg(7): 0}, {}), c()))
    s1 = B.join(s0, B.AW({tg(7): 1}, d1.value), [tg(3)])
    assert s1.gpu is not None
    # joining the OLDER struct again: the device is at s1's version, so s0 detaches and
    # joins its own terms -- exactly what the reference computes from s0
    d2 = B.AW({tg(8): 1}, B.add(tg(4), tg(44), tg(8), B.AW({tg(8): 0}, {}), c()).value)
    s2 = B.join(s0, d2, [tg(4)])
    assert s2.gpu is None
    assert B.read_cpu(s2) == B.read_cpu(B.join_cpu(s0, d2, [tg(4)]))
    # and the current struct still joins on the device
    s3 = B.join(s1, d2, [tg(4)])
    assert s3.gpu is not None and B.read(s3) == B.read_cpu(s3)


def test_send_diff_ships_no_device_handle():
    c = Clock()
    c1, c2 = B.Replica(1, c), B.Replica(2, c)
    c1.mutate("add", "a", 1)
    c1.crdt_state, cont = B.merkle_prepare(c1.crdt_state, B.LEVELS)
    d = B.Diff(cont, c1.crdt_state.dots, c1, c2, c1)
    msgs = [(c2, ("diff", d))]
    shipped = []
    while msgs:
        dest, msg = msgs.pop(0)
        if msg[0] == "diff" and len(msg) == 3:
            shipped.append(msg[1])
        msgs.extend(dest.handle(msg))
    assert shipped and all(m.gpu is None for m in shipped)
    assert c2.read() == {tg("a"): tg(1)}


def _pair(gpu, node_engines=None, max_sync_size=200):
    c = Clock()
    e1, e2 = node_engines or (None, None)
    return c, B.Replica(1, c, gpu=gpu, engine=e1, max_sync_size=max_sync_size), \
        B.Replica(2, c, gpu=gpu, engine=e2, max_sync_size=max_sync_size)


KEYS = st.integers(0, 6)
VALS = st.sampled_from([0, 1, 1.0, True, None, "x", b"y", (1, 2)])
STEP = st.one_of(
    st.tuples(st.just("add"), st.integers(0, 1), KEYS, VALS),
    st.tuples(st.just("remove"), st.integers(0, 1), KEYS, st.just(None)),
    st.tuples(st.just("sync"), st.integers(0, 1), st.just(0), st.just(None)),
)


def _run(steps, gpu, node_engines=None):
    c, r1, r2 = _pair(gpu, node_engines)
    rs = (r1, r2)
    for op, who, k, v in steps:
        if op == "sync":
            rs[who].sync_to(rs[1 - who])
        else:
            rs[who].mutate(op, k, *(() if op == "remove" else (v,)))
    return rs


def _model(steps):
    """aw_lww_map_property_test.exs:34-59's model on ONE replica: Map.put / Map.delete"""
    m = {}
    for op, _who, k, v in steps:
        if op == "add":
            m[tg(k)] = tg(v)
        elif op == "remove":
            m.pop(tg(k), None)
    return m


@settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck))
@given(st.lists(STEP, min_size=1, max_size=18))
def test_histories_match_the_reference(steps):
    """Mutations interleaved with sync rounds on two GPU replicas equal the same history on
    two CPU replicas (the reference's code): reads, on_diffs streams, raw states."""
    g = _run(steps, True)
    p = _run(steps, False)
    for a, b in zip(g, p):
        assert B.read(a.crdt_state) == B.read_cpu(b.crdt_state)
        assert T.canon(T.AW(a.crdt_state.dots, a.crdt_state.value)) == \
            T.canon(T.AW(b.crdt_state.dots, b.crdt_state.value))
        # (per callback the keys come in MerkleMap's order, which the reference leaves open)
        assert [sorted(map(repr, x)) for x in a.received] == [sorted(map(repr, x)) for x in b.received]
        assert a.crdt_state.gpu is not None
    # one replica, no syncs: the sequential model itself
    solo = [s for s in steps if s[0] != "sync" and s[1] == 0]
    r = _run(solo, True)[0]
    assert B.read(r.crdt_state) == _model(solo)


def test_two_nodes_keys_known_only_to_one_side():
    """Two engines = two BEAM nodes with their own universes: r1's keys are unknown to r2's
    engine, so r2's continue names them by id ({:"$dg_key", id}); r1's get_diff resolves
    them; removals of keys the originator never interned still propagate.
    (max_sync_size :infinite: with 200, the continuation itself is truncated at :98 and a
    round moves part of the keys -- while the receiver's context takes the sender's whole
    VV snapshot, as in the reference (H5), so its next round removes the rows it was not
    sent; that is the reference's behaviour, not a property to test here.)"""
    e1 = B.nif.engine_open(0, wrap=tg, unwrap=B.untg)[1]
    e2 = B.nif.engine_open(0, wrap=tg, unwrap=B.untg)[1]
    try:
        c, r1, r2 = _pair(True, (e1, e2), max_sync_size="infinite")
        for i in range(30):
            r1.mutate("add", f"only1-{i}", i)
            r2.mutate("add", f"only2-{i}", -i)
        r1.sync_to(r2)
        r2.sync_to(r1)
        assert r1.read() == r2.read() and len(r1.read()) == 60
        # a removal on r2 of keys r1 knows; then r1 -> r2 and r2 -> r1 converge
        for i in range(0, 30, 3):
            r2.mutate("remove", f"only1-{i}")
        r2.sync_to(r1)
        r1.sync_to(r2)
        assert r1.read() == r2.read() and len(r1.read()) == 50
        ref = _run([("add", 0, f"only1-{i}", i) for i in range(3)], False)[0]
        assert ref.read() == B.read_cpu(ref.crdt_state)
    finally:
        e1.close()
        e2.close()


# ---------------------------------------------------------------- storage and read(crdt, key)
# causal_crdt.ex:216-250: the replica persists {node_id, seq, crdt_state, merkle_map} after
# every delta and restores it at start; INTEGRATION §3.3 persists the struct detached and
# re-attaches a restored one from its terms (never trusting a handle it carries).

def _engine():
    return B.nif.engine_open(0, wrap=tg, unwrap=B.untg)[1]


def test_storage_backend_can_store_and_retrieve_state():  # causal_crdt_test.exs:80-85
    store = B.MemoryStorage()
    r = B.Replica(1, Clock(), storage_module=store, name="storage_test")
    assert attached(r)
    r.mutate("add", "Derek", "Kraan")
    assert r.read() == {tg("Derek"): tg("Kraan")}
    _node, _seq, persisted, _mm = store.read("storage_test")
    assert persisted.gpu is None  # detached: no device handle, no queue
    assert B.read_cpu(persisted) == {tg("Derek"): tg("Kraan")}


@pytest.mark.parametrize("n_keys,min_dots", [(3, 0), (300, 0), (40, 100), (200, 100)])
def test_storage_rehydrates_after_a_crash_on_a_new_engine(n_keys, min_dots):
    """causal_crdt_test.exs:87-102 through GPU replicas: the VM goes (its engine and every
    state resource with it), a NEW engine restores the replica from the snapshot -- on the
    device at or above the attach threshold, on the BEAM below it -- even from a snapshot
    that still carries the dead handle; then it mutates and syncs both ways with a live
    replica (device trees with gpu_min_dots 0, the CPU MerkleMap otherwise)."""
    store = B.MemoryStorage()
    c = Clock()
    gm = min_dots == 0
    e1, e2 = _engine(), None
    try:
        r = B.Replica(1, c, storage_module=store, name="st", engine=e1, min_dots=min_dots, gpu_merkle=gm)
        for i in range(n_keys):
            r.mutate("add", f"k{i}", i)
        r.mutate("remove", "k1")
        if attached(r):  # a snapshot written before the patch: the struct with its handle
            node, seq, persisted, mm = store.read("st")
            assert persisted.gpu is None
            store.write("st", (node, seq, B.replace(persisted, gpu=r.crdt_state.gpu), mm))
        e1.close()  # the VM is gone: the handle's state is freed
        e2 = _engine()
        r2 = B.Replica(77, c, storage_module=store, name="st", engine=e2, min_dots=min_dots, gpu_merkle=gm,
                       max_sync_size="infinite")  # (one round moves every key: see the test above)
        assert r2.node_id == tg(1)
        assert attached(r2) == (n_keys - 1 >= min_dots)
        want = {tg(f"k{i}"): tg(i) for i in range(n_keys) if i != 1}
        assert r2.read() == want
        p = B.Replica(2, c, engine=e2, min_dots=min_dots, gpu_merkle=gm, max_sync_size="infinite")
        for j in range(5):
            p.mutate("add", f"p{j}", -j)
        p.mutate("add", "k0", "from-p")  # later clock: p's write wins (LWW)
        r2.mutate("add", "k2", "again")
        r2.sync_to(p)
        p.sync_to(r2)
        want.update({tg(f"p{j}"): tg(-j) for j in range(5)})
        want[tg("k0")] = tg("from-p")
        want[tg("k2")] = tg("again")
        assert r2.read() == p.read() == want
        assert attached(r2) == (n_keys - 1 >= min_dots)
        # the restored replica keeps persisting: a third start sees the synced state
        r3 = B.Replica(78, c, storage_module=store, name="st", engine=e2, min_dots=min_dots, gpu_merkle=gm)
        assert r3.read() == want
    finally:
        e1.close()
        if e2 is not None:
            e2.close()


def test_a_map_keyed_by_the_atom_all():
    """read(crdt, key) reads the one key (aw_lww_map.ex:222-224), the atom :all included:
    the dispatch reaches the NIF's whole-map read from read/1 only."""
    from delta_crdt_ex_amd.terms import Atom
    r = B.Replica(1, Clock())
    r.mutate("add", Atom("all"), 1)
    r.mutate("add", "x", 2)
    r.crdt_state, _ = B.merkle_prepare(r.crdt_state, B.LEVELS)  # flushed: the device answers
    s = r.crdt_state
    a = tg(Atom("all"))
    assert B.read(s, a) == B.read(s, [a]) == B.read_cpu(s, a) == {a: tg(1)}
    assert B.read(s) == B.read_cpu(s) == {a: tg(1), tg("x"): tg(2)}
    assert B.read(s, [tg("x")]) == {tg("x"): tg(2)}


def test_large_batches_and_sync_deltas_match_the_reference():
    """Batches and sync deltas past the one-workgroup path's 512 keys (the NIF's
    mutate_batch and join_delta then take dg_mutate_batch_async + dg_join_delta_out's
    one-wait keyed path): 1,500 queued mutations flushed as one batch, and syncs moving
    hundreds of keys both ways (max_sync_size :infinite), equal to the same history on CPU
    replicas -- reads, raw states, on_diffs streams."""
    import random
    rnd = random.Random(7)
    steps = []
    for i in range(1500):
        k = rnd.randrange(900)
        if rnd.random() < 0.8:
            steps.append(("add", 0, k, rnd.choice([i, str(i), None, (i, 1)])))
        else:
            steps.append(("remove", 0, k, None))
    steps.append(("sync", 0, 0, None))
    for i in range(700):
        steps.append(("add", 1, 300 + i, -i))
    steps.append(("sync", 1, 0, None))
    steps.append(("sync", 0, 0, None))

    def run(gpu):
        c, r1, r2 = _pair(gpu, max_sync_size="infinite")
        rs = (r1, r2)
        for op, who, k, v in steps:
            if op == "sync":
                rs[who].sync_to(rs[1 - who])
            else:
                rs[who].mutate(op, k, *(() if op == "remove" else (v,)))
        return rs

    g, p = run(True), run(False)
    for a, b in zip(g, p):
        assert B.read(a.crdt_state) == B.read_cpu(b.crdt_state)
        assert T.canon(T.AW(a.crdt_state.dots, a.crdt_state.value)) == \
            T.canon(T.AW(b.crdt_state.dots, b.crdt_state.value))
        assert [sorted(map(repr, x)) for x in a.received] == [sorted(map(repr, x)) for x in b.received]
        assert a.crdt_state.gpu is not None
    assert g[0].read() == g[1].read() and len(g[0].read()) > 512
