"""SoA snapshots (delta_crdt_ex_amd/storage.py): the term codec and the
interning tables round-trip exactly on the CPU; the committed golden snapshot
(tests/golden/snapshot_terms.dgsnap, made by tests/golden/make_golden.py from the term
oracle) holds exactly the oracle's rows, context, read/1 and Merkle tree; a device state
and its Merkle tree round-trip through a file on the GPU as the reference's 4-tuple
{node_id, sequence_number, crdt_state, merkle_map} (causal_crdt.ex:242-250, read back
at :220-230), and a damaged file is refused."""
import os

import numpy as np
import pytest

from delta_crdt_ex_amd import interning, storage
from delta_crdt_ex_amd.terms import Atom, EList, EMap

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "snapshot_terms.dgsnap")


def _oracle_replica():
    """The replica the golden snapshot was made from (make_golden.snapshot_case)."""
    import sys
    sys.path.insert(0, os.path.dirname(GOLDEN))
    import make_golden as G
    from oracle import convert as CV
    U = interning.Universe()
    A = G.history(7, U, values=G.TERM_VALUES)[0]
    return A


TERMS = [None, True, False, Atom("ok"), 0, -5, 1 << 70, 2.5, "txt", b"\x00\xff",
         (1, "a", Atom("x")), EList([1, 2, EList([])]), EMap([(1, "a"), ("k", (2, 3))])]


def test_term_codec_round_trip():
    for t in TERMS:
        back = storage._unpack(storage._pack(t))
        assert back == t and type(back) is type(t)


def test_universe_tables_round_trip():
    U = interning.Universe()
    ids = [(U.key(t), U.value(t), U.node(t)) for t in TERMS if not isinstance(t, float)]
    V = storage._universe_from(storage._universe_tables(U))
    for t, (k, v, n) in zip([t for t in TERMS if not isinstance(t, float)], ids):
        assert V.key(t) == k and V.value(t) == v and V.node(t) == n
        assert V.key_term(k) == t and V.value_term(v) == t
    # a new term after the restore gets a fresh id, as it would have before
    assert V.value("new") == U.value("new")


def test_golden_snapshot_matches_the_oracle():
    from oracle import awlww_term as T
    from oracle import convert as CV
    from oracle import ref as R
    A = _oracle_replica()
    node_id, seq, rows, ctx, U, merkle = storage.read_arrays(GOLDEN)
    assert node_id == Atom("replica_a") and seq == 3
    # the rows, read back into terms through the snapshot's own Universe, are the oracle's
    assert CV.soa_canon(rows, ctx, U) == CV.term_canon(A)
    # read/1 on those rows (C oracle, ids) equals the term oracle's read/1
    ok, ov = R.read_lww(rows)
    got = {U.key_term(int(k)): U.value_term(int(v)) for k, v in zip(ok, ov)}
    assert {k: repr(v) for k, v in got.items()} == {k: repr(v) for k, v in T.read(A).items()}
    depth, sb, shard, nodes, counts, terms = merkle
    assert (depth, sb, shard, terms) == (6, 0, 0, True)
    want = R.merkle_build(rows, 6, terms=R.Terms(*U.term_tables()))  # a tree over terms
    assert np.array_equal(nodes, want.nodes) and np.array_equal(counts, want.counts)


def test_old_snapshot_layout_is_refused(tmp_path):
    p = tmp_path / "old.dgsnap"
    p.write_bytes(b"DGSNAP01" + bytes(16))
    with pytest.raises(ValueError, match="DGSNAP01"):
        storage.read_arrays(p)


def test_snapshot_write_is_atomic(tmp_path):
    """A crash mid-write (simulated: the temporary file is left half written) never
    damages the previous snapshot (write-then-rename)."""
    p = tmp_path / "r.dgsnap"
    U = interning.Universe()
    rows = tuple(np.zeros(0, dt) for dt in (np.uint64, np.uint64, np.int64, np.uint32, np.uint64))
    storage.write_arrays(p, 1, 1, rows, (0, np.zeros(0, np.uint32), np.zeros(0, np.uint64)), U)
    good = p.read_bytes()
    (tmp_path / "r.dgsnap.tmp").write_bytes(good[: len(good) // 2])
    assert storage.read_arrays(p)[1] == 1
    storage.write_arrays(p, 1, 2, rows, (0, np.zeros(0, np.uint32), np.zeros(0, np.uint64)), U)
    assert storage.read_arrays(p)[1] == 2 and not (tmp_path / "r.dgsnap.tmp").exists()


def test_snapshot_records_the_tree_kind(tmp_path):
    """the header says whether the persisted tree hashed terms or ids, and the
    reader restores that kind (a tree over ids must not come back term-hashed)."""
    U = interning.Universe()
    rows = tuple(np.zeros(0, dt) for dt in (np.uint64, np.uint64, np.int64, np.uint32, np.uint64))
    ctx = (0, np.zeros(0, np.uint32), np.zeros(0, np.uint64))
    nodes, counts = np.zeros(7, np.uint64), np.zeros(4, np.uint16)
    for terms in (True, False):
        p = tmp_path / f"t{terms}.dgsnap"
        storage.write_arrays(p, 1, 1, rows, ctx, U, (2, 0, 0, nodes, counts, terms))
        assert storage.read_arrays(p)[5][5] is terms
    # a 5-tuple (no flag) is a term-hashed tree, as every earlier DGSNAP02 file is
    storage.write_arrays(tmp_path / "d.dgsnap", 1, 1, rows, ctx, U, (2, 0, 0, nodes, counts))
    assert storage.read_arrays(tmp_path / "d.dgsnap")[5][5] is True


@pytest.mark.gpu
def test_golden_snapshot_on_the_device():
    """The golden snapshot read into device state: rows, context and read/1 equal the
    term oracle's; the persisted Merkle tree equals dg_merkle_build of the restored rows
    and diffs against it to nothing."""
    from delta_crdt_ex_amd import aw_lww_map as M
    from oracle import awlww_term as T
    from oracle import convert as CV
    A = _oracle_replica()
    node_id, seq, st, tree = storage.read(GOLDEN)
    assert node_id == Atom("replica_a") and seq == 3
    rows = st.rows.to_numpy()
    ctx = (st.ctx.kind,) + tuple(st.ctx.to_numpy())
    assert CV.soa_canon(rows, ctx, st.universe) == CV.term_canon(A)
    assert {k: repr(v) for k, v in M.read(st).items()} == {k: repr(v) for k, v in T.read(A).items()}
    fresh = M.merkle_map(st, tree.depth)
    assert np.array_equal(tree.nodes.cpu().numpy(), fresh.nodes.cpu().numpy())
    assert np.array_equal(tree.bucket_counts(), fresh.bucket_counts())
    assert M.engine().merkle_diff(tree, fresh).numel() == 0


@pytest.mark.gpu
def test_snapshot_round_trip(tmp_path):
    from delta_crdt_ex_amd import aw_lww_map as M
    st = M.compress_dots(M.new())
    for i, (k, v) in enumerate([("a", 1), (Atom("b"), "two"), ((3, 4), EList([5])), ("a", 9)]):
        st = M.join(st, M.add(k, v, Atom("node1"), st, ts=100 + i), [k])
    st = M.join(st, M.remove(Atom("b"), Atom("node1"), st), [Atom("b")])
    p = tmp_path / "replica.dgsnap"
    tree = M.merkle_map(st, 5)
    storage.write(p, Atom("node1"), 7, st, tree)
    node, seq, back, back_tree = storage.read(p)
    assert node == Atom("node1") and seq == 7
    assert back_tree.depth == 5 and back_tree.root() == tree.root()
    assert np.array_equal(back_tree.nodes.cpu().numpy(), M.merkle_map(back, 5).nodes.cpu().numpy())
    for x, y in zip(st.rows.to_numpy(), back.rows.to_numpy()):
        assert np.array_equal(x, y)
    for x, y in zip(st.ctx.to_numpy(), back.ctx.to_numpy()):
        assert np.array_equal(x, y)
    assert M.read(back) == M.read(st) == {"a": 9, (3, 4): EList([5])}
    # a damaged column is refused; a missing file reads as nil
    raw = bytearray(p.read_bytes())
    raw[-3] ^= 0xFF
    p.write_bytes(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        storage.read(p)
    assert storage.read(tmp_path / "absent") is None


@pytest.mark.gpu
def test_snapshot_keeps_an_id_tree(tmp_path):
    """A tree built over ids (terms=None) comes back as one: after an update it still
    equals a fresh id-hashed build of the new rows."""
    from delta_crdt_ex_amd import aw_lww_map as M
    st = M.compress_dots(M.new())
    for i in range(40):
        st = M.join(st, M.add(i, f"v{i}", 1, st, ts=10 + i), [i])
    tree = M.engine().merkle_build(st.rows, 6)  # terms=None: ids
    p = tmp_path / "ids.dgsnap"
    storage.write(p, 1, 1, st, tree)
    _, _, back, bt = storage.read(p)
    assert bt.terms is None and bt.root() == tree.root()
    nxt = M.join(back, M.add(3, "new value", 1, back, ts=99), [3])
    changed = M.engine().join2_changes(back.rows, back.ctx, nxt.rows, nxt.ctx)[2]
    M.engine().merkle_update(bt, nxt.rows, changed)
    assert bt.root() == M.engine().merkle_build(nxt.rows, 6).root()
