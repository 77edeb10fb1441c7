"""SoA snapshots (delta_crdt_ex_amd/storage.py): the term codec and the
interning tables round-trip exactly on the CPU; a device state round-trips through a
file on the GPU (rows, context, terms, read/1), and a damaged file is refused."""
import numpy as np
import pytest

from delta_crdt_ex_amd import interning, storage
from delta_crdt_ex_amd.terms import Atom, EList, EMap


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


@pytest.mark.gpu
def test_snapshot_round_trip(tmp_path):
    from delta_crdt_ex_amd import aw_lww_map as M
    st = M.compress_dots(M.new())
    for i, (k, v) in enumerate([("a", 1), (Atom("b"), "two"), ((3, 4), EList([5])), ("a", 9)]):
        st = M.join(st, M.add(k, v, Atom("node1"), st, ts=100 + i), [k])
    st = M.join(st, M.remove(Atom("b"), Atom("node1"), st), [Atom("b")])
    p = tmp_path / "replica.dgsnap"
    storage.write(p, Atom("node1"), 7, st)
    node, seq, back = storage.read(p)
    assert node == Atom("node1") and seq == 7
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
